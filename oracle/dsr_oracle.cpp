// dsr_oracle.cpp — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
//
// CPU restatement of the differentiable 3D-Gaussian tile rasterizer that the
// reference calls through `diff_gaussian_rasterization` (cuda_splatting.py:5-8,
// call site cuda_splatting.py:98-123; pinned by requirements.txt:23 as
// git+https://github.com/dcharatan/diff-gaussian-rasterization-modified, no commit).
// That library is NOT vendored in /root/reference and cannot be built or imported
// here, so this file restates the published 3DGS algorithm (graphdeco-inria
// rasterizer, 2-output API) as described in SURVEY.md §8(a) rows A6-A10:
//
//   preprocess  (A7): frustum cull z_view <= 0.2, EWA cov2D with 1.3*tanfov clamp and
//                     +0.3 px low-pass, conic, radius = ceil(3 sqrt(lambda_max)),
//                     ndc2Pix, 16x16 tile rect, SH (deg <= 3) -> RGB (+0.5, clamp >= 0)
//   binning     (A8): key = (tile << 32) | float_bits(depth), value = gaussian id,
//                     stable sort, per-tile [start, end)
//   render fwd  (A9): front-to-back alpha compositing, alpha = min(0.99, o*exp(power)),
//                     skip alpha < 1/255, stop when T*(1-alpha) < 1e-4, out = C + T*bg
//   render bwd / preprocess bwd (A10): back-to-front with T recovered by division,
//                     cov2D bwd -> dL/dcov3D(6) and dL/dmean3D, projection + SH bwd.
//
// PARITY STATUS: the rasterizer itself is "parity unpinned" against the reference
// (no reference output exists anywhere). This restatement is pinned by
// (i) analytic known-answer tests (tests/test_oracle_raster.py), (ii) torch autograd of
// a dense differentiable restatement for the backward, and (iii) golden fixtures of the
// reference's own wrapper (cuda_splatting.py) captured with a recording stub
// (tests/golden/make_golden.py). Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library.
//
// Floating-point order: every expression that feeds the bit-exact outputs (depth,
// radius, xy, tile rect) is written with a fixed evaluation order and compiled with
// -ffp-contract=off, matching the HIP kernels in my_depthsplat_amd/csrc/; the multiply-adds
// of the projection chain (transforms, EWA, eigenvalues, SH) are explicit std::fma calls in
// the kernels' order (upstream nvcc contracts such expressions into FMAs by default too).

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

constexpr int BX = 16, BY = 16;
constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                            -1.0925484305920792f, 0.5462742152960396f};
constexpr float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                            0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                            -0.5900435899266435f};

template <typename R>
struct V3T { R x, y, z; };
using V3 = V3T<float>;

// Column-major 4x4 (the layout of GaussianRasterizationSettings.viewmatrix/projmatrix,
// i.e. the row-major storage of the transposed torch matrices, cuda_splatting.py:83-86).
template <typename R>
inline V3T<R> xform43(const float* m, V3T<R> p) {
  V3T<R> r;
  r.x = std::fma(R(m[0]), p.x, std::fma(R(m[4]), p.y, std::fma(R(m[8]), p.z, R(m[12]))));
  r.y = std::fma(R(m[1]), p.x, std::fma(R(m[5]), p.y, std::fma(R(m[9]), p.z, R(m[13]))));
  r.z = std::fma(R(m[2]), p.x, std::fma(R(m[6]), p.y, std::fma(R(m[10]), p.z, R(m[14]))));
  return r;
}
inline float xform44w(const float* m, V3 p) {
  return std::fma(m[3], p.x, std::fma(m[7], p.y, std::fma(m[11], p.z, m[15])));
}

inline float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

template <typename R>
struct Cov2DWorkT {
  // T = J*W (2 x 3, the only non-zero rows), cov2D (a, b, c) after the +0.3 filter
  R T[2][3];
  R a, b, c;
  R tx, ty, tz;
  R xmul, ymul;
};
using Cov2DWork = Cov2DWorkT<float>;

// EWA splatting: cov2D = J W Sigma W^T J^T.
// R = float: the forward's (and the float backward's) arithmetic; R = double: the
// high-precision gradient reference (orc_backward_f64) of the same function.
template <typename R>
inline void cov2d(V3T<R> mean, R fx, R fy, R tanx, R tany, const float* c6, const float* view, Cov2DWorkT<R>& w) {
  V3T<R> t = xform43(view, mean);
  const R limx = R(1.3f) * tanx;
  const R limy = R(1.3f) * tany;
  const R txtz = t.x / t.z;
  const R tytz = t.y / t.z;
  w.xmul = (txtz < -limx || txtz > limx) ? R(0) : R(1);
  w.ymul = (tytz < -limy || tytz > limy) ? R(0) : R(1);
  t.x = std::min(limx, std::max(-limx, txtz)) * t.z;
  t.y = std::min(limy, std::max(-limy, tytz)) * t.z;
  w.tx = t.x; w.ty = t.y; w.tz = t.z;
  // Jacobian rows: J0 = (fx/z, 0, -fx x/z^2), J1 = (0, fy/z, -fy y/z^2)
  const R j00 = fx / t.z;
  const R j02 = -(fx * t.x) / (t.z * t.z);
  const R j11 = fy / t.z;
  const R j12 = -(fy * t.y) / (t.z * t.z);
  // W = rotation part of world->camera: Wr[r][c] = view[c*4 + r]
  const R W00 = view[0], W01 = view[4], W02 = view[8];
  const R W10 = view[1], W11 = view[5], W12 = view[9];
  const R W20 = view[2], W21 = view[6], W22 = view[10];
  // T = J * Wr  (2x3)
  w.T[0][0] = std::fma(j00, W00, j02 * W20);
  w.T[0][1] = std::fma(j00, W01, j02 * W21);
  w.T[0][2] = std::fma(j00, W02, j02 * W22);
  w.T[1][0] = std::fma(j11, W10, j12 * W20);
  w.T[1][1] = std::fma(j11, W11, j12 * W21);
  w.T[1][2] = std::fma(j11, W12, j12 * W22);
  // V = Sigma (symmetric from cov6 = xx, xy, xz, yy, yz, zz)
  const R V[3][3] = {{c6[0], c6[1], c6[2]}, {c6[1], c6[3], c6[4]}, {c6[2], c6[4], c6[5]}};
  // U = T * V (2x3), cov = U * T^T
  R U[2][3];
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 3; ++c)
      U[r][c] = std::fma(w.T[r][0], V[0][c], std::fma(w.T[r][1], V[1][c], w.T[r][2] * V[2][c]));
  const R a = std::fma(U[0][0], w.T[0][0], std::fma(U[0][1], w.T[0][1], U[0][2] * w.T[0][2]));
  const R b = std::fma(U[0][0], w.T[1][0], std::fma(U[0][1], w.T[1][1], U[0][2] * w.T[1][2]));
  const R c = std::fma(U[1][0], w.T[1][0], std::fma(U[1][1], w.T[1][1], U[1][2] * w.T[1][2]));
  w.a = a + R(0.3f);
  w.b = b;
  w.c = c + R(0.3f);
}

inline V3 sh_to_rgb(int deg, const float* sh /*[M][3]*/, V3 pos, const float* campos, uint8_t* clamped) {
  V3 dir = {pos.x - campos[0], pos.y - campos[1], pos.z - campos[2]};
  const float len = std::sqrt(std::fma(dir.x, dir.x, std::fma(dir.y, dir.y, dir.z * dir.z)));
  dir.x = dir.x / len; dir.y = dir.y / len; dir.z = dir.z / len;
  float r[3];
  for (int ch = 0; ch < 3; ++ch) {
    auto s = [&](int k) { return sh[k * 3 + ch]; };
    // basis values first, then one fused multiply-add per coefficient (the kernels' order)
    float v = SH_C0 * s(0);
    if (deg > 0) {
      const float x = dir.x, y = dir.y, z = dir.z;
      v = std::fma(-(SH_C1 * y), s(1), v);
      v = std::fma(SH_C1 * z, s(2), v);
      v = std::fma(-(SH_C1 * x), s(3), v);
      if (deg > 1) {
        const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        v = std::fma(SH_C2[0] * xy, s(4), v);
        v = std::fma(SH_C2[1] * yz, s(5), v);
        v = std::fma(SH_C2[2] * (2.0f * zz - xx - yy), s(6), v);
        v = std::fma(SH_C2[3] * xz, s(7), v);
        v = std::fma(SH_C2[4] * (xx - yy), s(8), v);
        if (deg > 2) {
          v = std::fma(SH_C3[0] * y * (3.0f * xx - yy), s(9), v);
          v = std::fma(SH_C3[1] * xy * z, s(10), v);
          v = std::fma(SH_C3[2] * y * (4.0f * zz - xx - yy), s(11), v);
          v = std::fma(SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy), s(12), v);
          v = std::fma(SH_C3[4] * x * (4.0f * zz - xx - yy), s(13), v);
          v = std::fma(SH_C3[5] * z * (xx - yy), s(14), v);
          v = std::fma(SH_C3[6] * x * (xx - 3.0f * yy), s(15), v);
        }
      }
    }
    v += 0.5f;
    clamped[ch] = v < 0.f ? 1 : 0;
    r[ch] = std::max(v, 0.0f);
  }
  return {r[0], r[1], r[2]};
}

struct State {
  int P, D, M, W, H, gx, gy;
  bool precomp;
  std::vector<float> means, shs, colors, opac, cov6, view, proj, campos, bg;
  float tanx, tany;
  // geometry
  std::vector<float> depth, xy, conic_o, rgb;
  std::vector<int> radii;
  std::vector<uint8_t> clamped;
  std::vector<uint32_t> touched;
  // binning
  std::vector<uint64_t> keys;
  std::vector<uint32_t> vals;
  std::vector<uint32_t> ranges;  // [T][2]
  // image
  std::vector<float> color, finalT;
  std::vector<uint32_t> ncontrib;
};

void preprocess(State& s) {
  const float fx = s.W / (2.0f * s.tanx);
  const float fy = s.H / (2.0f * s.tany);
  s.depth.assign(s.P, 0.f); s.xy.assign(2 * s.P, 0.f); s.conic_o.assign(4 * s.P, 0.f);
  s.rgb.assign(3 * s.P, 0.f); s.radii.assign(s.P, 0); s.clamped.assign(3 * s.P, 0); s.touched.assign(s.P, 0);
#pragma omp parallel for schedule(static)
  for (int i = 0; i < s.P; ++i) {
    const V3 p = {s.means[3 * i], s.means[3 * i + 1], s.means[3 * i + 2]};
    const V3 pv = xform43(s.view.data(), p);
    if (pv.z <= 0.2f) continue;  // in_frustum
    const V3 ph = xform43(s.proj.data(), p);
    const float pw = 1.0f / (xform44w(s.proj.data(), p) + 0.0000001f);
    const float ndx = ph.x * pw, ndy = ph.y * pw;
    Cov2DWork w;
    cov2d(p, fx, fy, s.tanx, s.tany, &s.cov6[6 * i], s.view.data(), w);
    const float det = std::fma(w.a, w.c, -(w.b * w.b));
    if (det == 0.0f) continue;
    const float det_inv = 1.f / det;
    const float mid = 0.5f * (w.a + w.c);
    const float disc = std::sqrt(std::max(0.1f, std::fma(mid, mid, -det)));
    const float l1 = mid + disc, l2 = mid - disc;
    const float radius = std::ceil(3.f * std::sqrt(std::max(l1, l2)));
    const int r = (int)radius;
    const float px = ndc2pix(ndx, s.W), py = ndc2pix(ndy, s.H);
    const int x0 = std::min(s.gx, std::max(0, (int)((px - r) / BX)));
    const int y0 = std::min(s.gy, std::max(0, (int)((py - r) / BY)));
    const int x1 = std::min(s.gx, std::max(0, (int)((px + r + BX - 1) / BX)));
    const int y1 = std::min(s.gy, std::max(0, (int)((py + r + BY - 1) / BY)));
    if ((x1 - x0) * (y1 - y0) == 0) continue;
    if (!s.precomp) {
      const V3 c = sh_to_rgb(s.D, &s.shs[(size_t)i * s.M * 3], p, s.campos.data(), &s.clamped[3 * i]);
      s.rgb[3 * i] = c.x; s.rgb[3 * i + 1] = c.y; s.rgb[3 * i + 2] = c.z;
    } else {
      for (int ch = 0; ch < 3; ++ch) s.rgb[3 * i + ch] = s.colors[3 * i + ch];
    }
    s.depth[i] = pv.z;
    s.radii[i] = r;
    s.xy[2 * i] = px; s.xy[2 * i + 1] = py;
    s.conic_o[4 * i] = w.c * det_inv;
    s.conic_o[4 * i + 1] = -w.b * det_inv;
    s.conic_o[4 * i + 2] = w.a * det_inv;
    s.conic_o[4 * i + 3] = s.opac[i];
    s.touched[i] = (uint32_t)((y1 - y0) * (x1 - x0));
  }
}

void rect_of(const State& s, int i, int& x0, int& y0, int& x1, int& y1) {
  const float px = s.xy[2 * i], py = s.xy[2 * i + 1];
  const int r = s.radii[i];
  x0 = std::min(s.gx, std::max(0, (int)((px - r) / BX)));
  y0 = std::min(s.gy, std::max(0, (int)((py - r) / BY)));
  x1 = std::min(s.gx, std::max(0, (int)((px + r + BX - 1) / BX)));
  y1 = std::min(s.gy, std::max(0, (int)((py + r + BY - 1) / BY)));
}

void binning(State& s) {
  // inclusive scan of tiles_touched (emission order = gaussian id, then tile y, then x)
  std::vector<uint64_t> off(s.P + 1, 0);
  for (int i = 0; i < s.P; ++i) off[i + 1] = off[i] + (s.radii[i] > 0 ? s.touched[i] : 0);
  const size_t N = off[s.P];
  std::vector<std::pair<uint64_t, uint32_t>> kv(N);
  for (int i = 0; i < s.P; ++i) {
    if (s.radii[i] <= 0) continue;
    int x0, y0, x1, y1;
    rect_of(s, i, x0, y0, x1, y1);
    size_t o = off[i];
    uint32_t dbits;
    std::memcpy(&dbits, &s.depth[i], 4);
    for (int y = y0; y < y1; ++y)
      for (int x = x0; x < x1; ++x) {
        const uint64_t tile = (uint64_t)(y * s.gx + x);
        kv[o++] = {(tile << 32) | dbits, (uint32_t)i};
      }
  }
  std::stable_sort(kv.begin(), kv.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  s.keys.resize(N); s.vals.resize(N);
  for (size_t k = 0; k < N; ++k) { s.keys[k] = kv[k].first; s.vals[k] = kv[k].second; }
  const int T = s.gx * s.gy;
  s.ranges.assign(2 * (size_t)T, 0);
  for (size_t k = 0; k < N; ++k) {
    const uint32_t t = (uint32_t)(s.keys[k] >> 32);
    if (k == 0 || (uint32_t)(s.keys[k - 1] >> 32) != t) s.ranges[2 * t] = (uint32_t)k;
    if (k == N - 1 || (uint32_t)(s.keys[k + 1] >> 32) != t) s.ranges[2 * t + 1] = (uint32_t)(k + 1);
  }
}

void render(State& s) {
  const int HW = s.H * s.W;
  s.color.assign(3 * (size_t)HW, 0.f); s.finalT.assign(HW, 0.f); s.ncontrib.assign(HW, 0);
  const int T = s.gx * s.gy;
#pragma omp parallel for schedule(dynamic, 1)
  for (int t = 0; t < T; ++t) {
    const int tx = t % s.gx, ty = t / s.gx;
    const uint32_t b = s.ranges[2 * t], e = s.ranges[2 * t + 1];
    for (int ly = 0; ly < BY; ++ly)
      for (int lx = 0; lx < BX; ++lx) {
        const int x = tx * BX + lx, y = ty * BY + ly;
        if (x >= s.W || y >= s.H) continue;
        const float pfx = (float)x, pfy = (float)y;
        float Tr = 1.0f, C[3] = {0, 0, 0};
        uint32_t contributor = 0, last = 0;
        for (uint32_t k = b; k < e; ++k) {
          contributor++;
          const uint32_t id = s.vals[k];
          const float* co = &s.conic_o[4 * id];
          const float dx = s.xy[2 * id] - pfx, dy = s.xy[2 * id + 1] - pfy;
          const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
          if (power > 0.0f) continue;
          const float alpha = std::min(0.99f, co[3] * std::exp(power));
          if (alpha < 1.0f / 255.0f) continue;
          const float testT = Tr * (1 - alpha);
          if (testT < 0.0001f) break;
          for (int ch = 0; ch < 3; ++ch) C[ch] += s.rgb[3 * id + ch] * alpha * Tr;
          Tr = testT;
          last = contributor;
        }
        const int pix = y * s.W + x;
        s.finalT[pix] = Tr;
        s.ncontrib[pix] = last;
        for (int ch = 0; ch < 3; ++ch) s.color[(size_t)ch * HW + pix] = C[ch] + Tr * s.bg[ch];
      }
  }
}

template <typename R>
void backward_t(State& s, const float* dL_dpix, float* dmean2D, float* dconic, float* dopac, float* dcolor,
                float* dmean3D, float* dcov6, float* dsh) {
  const int P = s.P, HW = s.H * s.W, T = s.gx * s.gy;
  std::memset(dmean2D, 0, 3 * (size_t)P * 4); std::memset(dconic, 0, 3 * (size_t)P * 4);
  std::memset(dopac, 0, (size_t)P * 4); std::memset(dcolor, 0, 3 * (size_t)P * 4);
  std::memset(dmean3D, 0, 3 * (size_t)P * 4); std::memset(dcov6, 0, 6 * (size_t)P * 4);
  if (dsh) std::memset(dsh, 0, (size_t)P * s.M * 3 * 4);
  const R ddelx_dx = 0.5f * s.W, ddely_dy = 0.5f * s.H;
  std::vector<double> acc_m2(2 * (size_t)P, 0), acc_con(3 * (size_t)P, 0), acc_op(P, 0), acc_col(3 * (size_t)P, 0);
  // --- render backward (serial; double accumulators make the checker order-insensitive) ---
  for (int t = 0; t < T; ++t) {
    const int tx = t % s.gx, ty = t / s.gx;
    const uint32_t b = s.ranges[2 * t], e = s.ranges[2 * t + 1];
    for (int ly = 0; ly < BY; ++ly)
      for (int lx = 0; lx < BX; ++lx) {
        const int x = tx * BX + lx, y = ty * BY + ly;
        if (x >= s.W || y >= s.H) continue;
        const int pix = y * s.W + x;
        const R pfx = (float)x, pfy = (float)y;
        const R Tfin = s.finalT[pix];
        R Tr = Tfin;
        const uint32_t last_contrib = s.ncontrib[pix];
        R dpix[3], accum[3] = {0, 0, 0}, last_color[3] = {0, 0, 0}, last_alpha = 0.f;
        for (int ch = 0; ch < 3; ++ch) dpix[ch] = dL_dpix[(size_t)ch * HW + pix];
        R bg_dot = 0.f;
        for (int ch = 0; ch < 3; ++ch) bg_dot += s.bg[ch] * dpix[ch];
        // positions >= last_contrib never blended: start the back-to-front walk below them
        for (uint32_t k = b + std::min(e - b, last_contrib); k > b; --k) {
          const uint32_t id = s.vals[k - 1];
          const float* co = &s.conic_o[4 * id];
          // which entries blend: decided in float, exactly as the forward decided it
          {
            const float fdx = s.xy[2 * id] - (float)x, fdy = s.xy[2 * id + 1] - (float)y;
            const float fpower = -0.5f * (co[0] * fdx * fdx + co[2] * fdy * fdy) - co[1] * fdx * fdy;
            if (fpower > 0.0f) continue;
            if (std::min(0.99f, co[3] * std::exp(fpower)) < 1.0f / 255.0f) continue;
          }
          const R dx = R(s.xy[2 * id]) - pfx, dy = R(s.xy[2 * id + 1]) - pfy;
          const R power = R(-0.5f) * (R(co[0]) * dx * dx + R(co[2]) * dy * dy) - R(co[1]) * dx * dy;
          const R G = std::exp(power);
          const R alpha = std::min(R(0.99f), R(co[3]) * G);
          Tr = Tr / (1.f - alpha);
          const R dchannel_dcolor = alpha * Tr;
          R dL_dalpha = 0.f;
          for (int ch = 0; ch < 3; ++ch) {
            const R c = s.rgb[3 * id + ch];
            accum[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum[ch];
            last_color[ch] = c;
            dL_dalpha += (c - accum[ch]) * dpix[ch];
            acc_col[3 * id + ch] += dchannel_dcolor * dpix[ch];
          }
          dL_dalpha *= Tr;
          last_alpha = alpha;
          dL_dalpha += (-Tfin / (1.f - alpha)) * bg_dot;
          const R dL_dG = co[3] * dL_dalpha;
          const R gdx = G * dx, gdy = G * dy;
          const R dG_ddelx = -gdx * co[0] - gdy * co[1];
          const R dG_ddely = -gdy * co[2] - gdx * co[1];
          acc_m2[2 * id] += dL_dG * dG_ddelx * ddelx_dx;
          acc_m2[2 * id + 1] += dL_dG * dG_ddely * ddely_dy;
          acc_con[3 * id] += -0.5f * gdx * dx * dL_dG;
          acc_con[3 * id + 1] += -0.5f * gdx * dy * dL_dG;
          acc_con[3 * id + 2] += -0.5f * gdy * dy * dL_dG;
          acc_op[id] += G * dL_dalpha;
        }
      }
  }
  for (int i = 0; i < P; ++i) {
    dmean2D[3 * i] = (float)acc_m2[2 * i]; dmean2D[3 * i + 1] = (float)acc_m2[2 * i + 1];
    for (int c = 0; c < 3; ++c) { dconic[3 * i + c] = (float)acc_con[3 * i + c]; dcolor[3 * i + c] = (float)acc_col[3 * i + c]; }
    dopac[i] = (float)acc_op[i];
  }
  // --- preprocess backward ---
  const R fx = R(s.W) / (R(2.0f) * R(s.tanx));
  const R fy = R(s.H) / (R(2.0f) * R(s.tany));
  const float* proj = s.proj.data();
  for (int i = 0; i < P; ++i) {
    if (!(s.radii[i] > 0)) continue;
    const V3T<R> m = {s.means[3 * i], s.means[3 * i + 1], s.means[3 * i + 2]};
    const float* c6 = &s.cov6[6 * i];
    // the forward's 2D covariance, Jacobian and clamps, in float exactly as the forward
    // computed them (the conic the compositing used is the inverse of THIS cov2D): the
    // derivative is evaluated at the forward's own point. For needle-shaped Gaussians
    // (det(cov2D) << a c) the inverse is ill-conditioned, and a cov2D recomputed in double
    // would be a measurably different point.
    Cov2DWork wf;
    cov2d(V3{s.means[3 * i], s.means[3 * i + 1], s.means[3 * i + 2]}, (float)s.W / (2.0f * s.tanx),
          (float)s.H / (2.0f * s.tany), s.tanx, s.tany, c6, s.view.data(), wf);
    Cov2DWorkT<R> w;
    for (int r = 0; r < 2; ++r)
      for (int c = 0; c < 3; ++c) w.T[r][c] = wf.T[r][c];
    w.a = wf.a; w.b = wf.b; w.c = wf.c; w.tx = wf.tx; w.ty = wf.ty; w.tz = wf.tz; w.xmul = wf.xmul; w.ymul = wf.ymul;
    // conic = inverse(cov2D); gradient of the symmetric-matrix inverse, dL/dcov2D =
    // -S dL/dS S with S the conic the forward stored (conic_gradient: the same formula as the
    // kernels; upstream writes it through det(cov2D)^2 + 1e-7, whose a c - b^2 cancels for
    // needle-shaped Gaussians — the forms agree to 1e-7 / det^2 <= 1.2e-5 relative since
    // cov2D >= 0.3 I). The render bwd accumulates dconic.y as HALF the derivative w.r.t. the
    // off-diagonal entry (it appears twice in the quadratic form), so dL/db = 2 M01.
    const R ga = R(acc_con[3 * i]), gb = R(acc_con[3 * i + 1]), gc = R(acc_con[3 * i + 2]);
    const R A = R(s.conic_o[4 * i]), B = R(s.conic_o[4 * i + 1]), C = R(s.conic_o[4 * i + 2]);
    const R sg00 = A * ga + B * gb, sg01 = A * gb + B * gc, sg10 = B * ga + C * gb, sg11 = B * gb + C * gc;
    const R dL_da = -(sg00 * A + sg01 * B);
    const R dL_dc = -(sg10 * B + sg11 * C);
    const R dL_db = -2 * (sg00 * B + sg01 * C);
    // cov2D = T V T^T  (a = T0 V T0^T, b = T0 V T1^T, c = T1 V T1^T)
    const R (*T)[3] = w.T;
    // dL/dV (symmetric, cov6 order xx, xy, xz, yy, yz, zz; off-diagonals carry both halves)
    float* dc = &dcov6[6 * i];
    dc[0] = T[0][0] * T[0][0] * dL_da + T[0][0] * T[1][0] * dL_db + T[1][0] * T[1][0] * dL_dc;
    dc[3] = T[0][1] * T[0][1] * dL_da + T[0][1] * T[1][1] * dL_db + T[1][1] * T[1][1] * dL_dc;
    dc[5] = T[0][2] * T[0][2] * dL_da + T[0][2] * T[1][2] * dL_db + T[1][2] * T[1][2] * dL_dc;
    dc[1] = 2 * T[0][0] * T[0][1] * dL_da + (T[0][0] * T[1][1] + T[0][1] * T[1][0]) * dL_db + 2 * T[1][0] * T[1][1] * dL_dc;
    dc[2] = 2 * T[0][0] * T[0][2] * dL_da + (T[0][0] * T[1][2] + T[0][2] * T[1][0]) * dL_db + 2 * T[1][0] * T[1][2] * dL_dc;
    dc[4] = 2 * T[0][2] * T[0][1] * dL_da + (T[0][1] * T[1][2] + T[0][2] * T[1][1]) * dL_db + 2 * T[1][1] * T[1][2] * dL_dc;
    // dL/dT (2x3): dA/dT0 = 2 V T0, dB/dT0 = V T1, dB/dT1 = V T0, dC/dT1 = 2 V T1
    const R V[3][3] = {{c6[0], c6[1], c6[2]}, {c6[1], c6[3], c6[4]}, {c6[2], c6[4], c6[5]}};
    R VT0[3], VT1[3];
    for (int r = 0; r < 3; ++r) {
      VT0[r] = V[r][0] * T[0][0] + V[r][1] * T[0][1] + V[r][2] * T[0][2];
      VT1[r] = V[r][0] * T[1][0] + V[r][1] * T[1][1] + V[r][2] * T[1][2];
    }
    R dT0[3], dT1[3];
    for (int r = 0; r < 3; ++r) {
      dT0[r] = 2 * VT0[r] * dL_da + VT1[r] * dL_db;
      dT1[r] = 2 * VT1[r] * dL_dc + VT0[r] * dL_db;
    }
    // T = J Wr -> dL/dJ = dL/dT Wr^T ; only J00, J02, J11, J12 are live
    const float* vw = s.view.data();
    const R W00 = vw[0], W01 = vw[4], W02 = vw[8];
    const R W10 = vw[1], W11 = vw[5], W12 = vw[9];
    const R W20 = vw[2], W21 = vw[6], W22 = vw[10];
    const R dJ00 = dT0[0] * W00 + dT0[1] * W01 + dT0[2] * W02;
    const R dJ02 = dT0[0] * W20 + dT0[1] * W21 + dT0[2] * W22;
    const R dJ11 = dT1[0] * W10 + dT1[1] * W11 + dT1[2] * W12;
    const R dJ12 = dT1[0] * W20 + dT1[1] * W21 + dT1[2] * W22;
    const R tz = 1.f / w.tz, tz2 = tz * tz, tz3 = tz2 * tz;
    const R dtx = w.xmul * -fx * tz2 * dJ02;
    const R dty = w.ymul * -fy * tz2 * dJ12;
    const R dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2 * fx * w.tx) * tz3 * dJ02 + (2 * fy * w.ty) * tz3 * dJ12;
    // camera -> world: dL/dmean = Wr^T dL/dt
    R dm[3];
    dm[0] = W00 * dtx + W10 * dty + W20 * dtz;
    dm[1] = W01 * dtx + W11 * dty + W21 * dtz;
    dm[2] = W02 * dtx + W12 * dty + W22 * dtz;
    // projection: ndc = (P p).xy / (P p).w
    const R mhx = proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12];
    const R mhy = proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13];
    const R mw = R(1) / (proj[3] * m.x + proj[7] * m.y + proj[11] * m.z + proj[15] + R(0.0000001f));
    const R mul1 = mhx * mw * mw, mul2 = mhy * mw * mw;
    const R g2x = R(acc_m2[2 * i]), g2y = R(acc_m2[2 * i + 1]);
    dm[0] += (proj[0] * mw - proj[3] * mul1) * g2x + (proj[1] * mw - proj[3] * mul2) * g2y;
    dm[1] += (proj[4] * mw - proj[7] * mul1) * g2x + (proj[5] * mw - proj[7] * mul2) * g2y;
    dm[2] += (proj[8] * mw - proj[11] * mul1) * g2x + (proj[9] * mw - proj[11] * mul2) * g2y;
    // SH backward (view-dependent colour): dL/dsh and dL/dmean through the view direction
    if (!s.precomp) {
      const float* sh = &s.shs[(size_t)i * s.M * 3];
      float* dshi = &dsh[(size_t)i * s.M * 3];
      const R dirx0 = m.x - s.campos[0], diry0 = m.y - s.campos[1], dirz0 = m.z - s.campos[2];
      const R len = std::sqrt(dirx0 * dirx0 + diry0 * diry0 + dirz0 * dirz0);
      const R x = dirx0 / len, y = diry0 / len, z = dirz0 / len;
      R dRGB[3];
      for (int ch = 0; ch < 3; ++ch) dRGB[ch] = s.clamped[3 * i + ch] ? R(0) : R(acc_col[3 * i + ch]);
      R ddx[3] = {0, 0, 0}, ddy[3] = {0, 0, 0}, ddz[3] = {0, 0, 0};  // dRGB/ddir per channel
      for (int ch = 0; ch < 3; ++ch) {
        auto sv = [&](int k) { return sh[k * 3 + ch]; };
        const R g = dRGB[ch];
        dshi[0 * 3 + ch] = SH_C0 * g;
        if (s.D > 0) {
          dshi[1 * 3 + ch] = -SH_C1 * y * g;
          dshi[2 * 3 + ch] = SH_C1 * z * g;
          dshi[3 * 3 + ch] = -SH_C1 * x * g;
          ddx[ch] = -SH_C1 * sv(3);
          ddy[ch] = -SH_C1 * sv(1);
          ddz[ch] = SH_C1 * sv(2);
          if (s.D > 1) {
            const R xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            dshi[4 * 3 + ch] = SH_C2[0] * xy * g;
            dshi[5 * 3 + ch] = SH_C2[1] * yz * g;
            dshi[6 * 3 + ch] = SH_C2[2] * (2.f * zz - xx - yy) * g;
            dshi[7 * 3 + ch] = SH_C2[3] * xz * g;
            dshi[8 * 3 + ch] = SH_C2[4] * (xx - yy) * g;
            ddx[ch] += SH_C2[0] * y * sv(4) + SH_C2[2] * 2.f * -x * sv(6) + SH_C2[3] * z * sv(7) + SH_C2[4] * 2.f * x * sv(8);
            ddy[ch] += SH_C2[0] * x * sv(4) + SH_C2[1] * z * sv(5) + SH_C2[2] * 2.f * -y * sv(6) + SH_C2[4] * 2.f * -y * sv(8);
            ddz[ch] += SH_C2[1] * y * sv(5) + SH_C2[2] * 2.f * 2.f * z * sv(6) + SH_C2[3] * x * sv(7);
            if (s.D > 2) {
              dshi[9 * 3 + ch] = SH_C3[0] * y * (3.f * xx - yy) * g;
              dshi[10 * 3 + ch] = SH_C3[1] * xy * z * g;
              dshi[11 * 3 + ch] = SH_C3[2] * y * (4.f * zz - xx - yy) * g;
              dshi[12 * 3 + ch] = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy) * g;
              dshi[13 * 3 + ch] = SH_C3[4] * x * (4.f * zz - xx - yy) * g;
              dshi[14 * 3 + ch] = SH_C3[5] * z * (xx - yy) * g;
              dshi[15 * 3 + ch] = SH_C3[6] * x * (xx - 3.f * yy) * g;
              ddx[ch] += SH_C3[0] * sv(9) * 3.f * 2.f * xy + SH_C3[1] * sv(10) * yz +
                         SH_C3[2] * sv(11) * -2.f * xy + SH_C3[3] * sv(12) * -3.f * 2.f * xz +
                         SH_C3[4] * sv(13) * (-3.f * xx + 4.f * zz - yy) + SH_C3[5] * sv(14) * 2.f * xz +
                         SH_C3[6] * sv(15) * 3.f * (xx - yy);
              ddy[ch] += SH_C3[0] * sv(9) * 3.f * (xx - yy) + SH_C3[1] * sv(10) * xz +
                         SH_C3[2] * sv(11) * (-3.f * yy + 4.f * zz - xx) + SH_C3[3] * sv(12) * -3.f * 2.f * yz +
                         SH_C3[4] * sv(13) * -2.f * xy + SH_C3[5] * sv(14) * -2.f * yz +
                         SH_C3[6] * sv(15) * -3.f * 2.f * xy;
              ddz[ch] += SH_C3[1] * sv(10) * xy + SH_C3[2] * sv(11) * 4.f * 2.f * yz +
                         SH_C3[3] * sv(12) * 3.f * (2.f * zz - xx - yy) + SH_C3[4] * sv(13) * 4.f * 2.f * xz +
                         SH_C3[5] * sv(14) * (xx - yy);
            }
          }
        }
      }
      // dL/ddir (normalised), then through the normalisation
      const R gdx = ddx[0] * dRGB[0] + ddx[1] * dRGB[1] + ddx[2] * dRGB[2];
      const R gdy = ddy[0] * dRGB[0] + ddy[1] * dRGB[1] + ddy[2] * dRGB[2];
      const R gdz = ddz[0] * dRGB[0] + ddz[1] * dRGB[1] + ddz[2] * dRGB[2];
      const R sum2 = dirx0 * dirx0 + diry0 * diry0 + dirz0 * dirz0;
      const R invsum32 = 1.0f / std::sqrt(sum2 * sum2 * sum2);
      dm[0] += ((sum2 - dirx0 * dirx0) * gdx - diry0 * dirx0 * gdy - dirz0 * dirx0 * gdz) * invsum32;
      dm[1] += (-dirx0 * diry0 * gdx + (sum2 - diry0 * diry0) * gdy - dirz0 * diry0 * gdz) * invsum32;
      dm[2] += (-dirx0 * dirz0 * gdx - diry0 * dirz0 * gdy + (sum2 - dirz0 * dirz0) * gdz) * invsum32;
    }
    dmean3D[3 * i] = dm[0]; dmean3D[3 * i + 1] = dm[1]; dmean3D[3 * i + 2] = dm[2];
  }
}


}  // namespace

extern "C" {

// Forward pass for ONE view (the upstream per-call granularity, cuda_splatting.py:90-125).
// Inputs follow the rasterizer call at cuda_splatting.py:116-123: shs [P][M][3] xor colors [P][3],
// opacities [P], cov3D_precomp [P][6]; view/proj column-major [16]; campos [3]; bg [3].
void* orc_forward(int P, int D, int M, int W, int H, const float* bg, const float* means,
                  const float* shs, const float* colors, const float* opac, const float* cov6,
                  const float* view, const float* proj, const float* campos, float tanx, float tany) {
  State* s = new State();
  s->P = P; s->D = D; s->M = M; s->W = W; s->H = H;
  s->gx = (W + BX - 1) / BX; s->gy = (H + BY - 1) / BY;
  s->precomp = (shs == nullptr);
  s->means.assign(means, means + 3 * (size_t)P);
  if (shs) s->shs.assign(shs, shs + (size_t)P * M * 3);
  if (colors) s->colors.assign(colors, colors + 3 * (size_t)P);
  s->opac.assign(opac, opac + P);
  s->cov6.assign(cov6, cov6 + 6 * (size_t)P);
  s->view.assign(view, view + 16); s->proj.assign(proj, proj + 16);
  s->campos.assign(campos, campos + 3); s->bg.assign(bg, bg + 3);
  s->tanx = tanx; s->tany = tany;
  preprocess(*s);
  binning(*s);
  render(*s);
  return s;
}

void orc_free(void* h) { delete static_cast<State*>(h); }
int orc_num_rendered(void* h) { return (int)static_cast<State*>(h)->keys.size(); }
int orc_num_tiles(void* h) { auto* s = static_cast<State*>(h); return s->gx * s->gy; }

void orc_get_image(void* h, float* color, float* finalT, uint32_t* ncontrib) {
  auto* s = static_cast<State*>(h);
  std::memcpy(color, s->color.data(), s->color.size() * 4);
  if (finalT) std::memcpy(finalT, s->finalT.data(), s->finalT.size() * 4);
  if (ncontrib) std::memcpy(ncontrib, s->ncontrib.data(), s->ncontrib.size() * 4);
}

void orc_get_geom(void* h, float* depth, int* radii, float* xy, float* conic_o, float* rgb,
                  uint32_t* touched, uint8_t* clamped) {
  auto* s = static_cast<State*>(h);
  const size_t P = s->P;
  if (depth) std::memcpy(depth, s->depth.data(), P * 4);
  if (radii) std::memcpy(radii, s->radii.data(), P * 4);
  if (xy) std::memcpy(xy, s->xy.data(), 2 * P * 4);
  if (conic_o) std::memcpy(conic_o, s->conic_o.data(), 4 * P * 4);
  if (rgb) std::memcpy(rgb, s->rgb.data(), 3 * P * 4);
  if (touched) std::memcpy(touched, s->touched.data(), P * 4);
  if (clamped) std::memcpy(clamped, s->clamped.data(), 3 * P);
}

void orc_get_binning(void* h, uint64_t* keys, uint32_t* vals, uint32_t* ranges) {
  auto* s = static_cast<State*>(h);
  if (keys) std::memcpy(keys, s->keys.data(), s->keys.size() * 8);
  if (vals) std::memcpy(vals, s->vals.data(), s->vals.size() * 4);
  if (ranges) std::memcpy(ranges, s->ranges.data(), s->ranges.size() * 4);
}

// Backward for ONE view. dL_dpix [3][H][W]. Outputs (all [P]-major, zero-filled here):
// dmean2D [P][3] (ndc units, z = 0), dconic [P][3] (a, b, c as accumulated by the render bwd),
// dopac [P], dcolor [P][3], dmean3D [P][3], dcov6 [P][6], dsh [P][M][3] (or NULL when precomp).
void orc_backward(void* h, const float* dL_dpix, float* dmean2D, float* dconic, float* dopac,
                  float* dcolor, float* dmean3D, float* dcov6, float* dsh) {
  backward_t<float>(*static_cast<State*>(h), dL_dpix, dmean2D, dconic, dopac, dcolor, dmean3D, dcov6, dsh);
}

// The same backward evaluated in double (per-pixel chain, transmittance recovery, Jacobians;
// which entries blend is still decided in float, as the forward decided it): the gradient of
// the very function the float forward computed, to ~1e-15. Tests use it as the reference
// for device gradients whose per-pixel terms cancel heavily (a float implementation's error
// relative to the largest gradient is then limited by its float terms, not by the checker).
void orc_backward_f64(void* h, const float* dL_dpix, float* dmean2D, float* dconic, float* dopac,
                      float* dcolor, float* dmean3D, float* dcov6, float* dsh) {
  backward_t<double>(*static_cast<State*>(h), dL_dpix, dmean2D, dconic, dopac, dcolor, dmean3D, dcov6, dsh);
}

// Gradient of the conic (inverse 2D covariance) w.r.t. cov2D = [[a, b], [b, c]] (b counted once:
// dL/db is the derivative along the symmetric perturbation of both off-diagonal entries), in
// double, from dconic as the render backward accumulates it (dL/dA, HALF the derivative w.r.t.
// the conic's off-diagonal B, dL/dC). form 0: -S G S with S the exact inverse (the kernels' and
// backward_t's form); form 1: the upstream computeCov2DCUDA formula through
// denom2inv = 1 / (det^2 + 1e-7) [U]. out = (dL/da, dL/db, dL/dc). Test hook: pins that the
// two forms agree (they differ by the 1e-7 regulariser only).
void orc_conic_grad(double a, double b, double c, const double* dconic, int form, double* out) {
  const double gA = dconic[0], gB = dconic[1], gC = dconic[2];
  const double det = a * c - b * b;
  if (form == 0) {
    const double A = c / det, B = -b / det, C = a / det;
    const double sg00 = A * gA + B * gB, sg01 = A * gB + B * gC, sg10 = B * gA + C * gB, sg11 = B * gB + C * gC;
    out[0] = -(sg00 * A + sg01 * B);
    out[1] = -2 * (sg00 * B + sg01 * C);
    out[2] = -(sg10 * B + sg11 * C);
    (void)sg10;
    return;
  }
  const double denom2inv = 1.0 / (det * det + 0.0000001);
  out[0] = denom2inv * (-c * c * gA + 2 * b * c * gB + (det - a * c) * gC);
  out[2] = denom2inv * (-a * a * gC + 2 * a * b * gB + (det - a * c) * gA);
  out[1] = denom2inv * 2 * (b * c * gA - (det + 2 * b * b) * gB + a * b * gC);
}

}  // extern "C"
