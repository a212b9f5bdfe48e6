// dga_adapter.hip — fused Gaussian adapter (head channels -> world-space Gaussians) for gfx950.
//
// One thread per (scene b, context view v, pixel p) replaces the encoder glue and adapter
// (SURVEY §8a rows A13-A16), which in torch are ~30 small kernels plus batched 3x3 GEMMs:
//   opacity = sigmoid(head[0])                                  encoder_depthsplat.py:258
//   xy = pixel centre + (sigmoid(head[1:3]) - 0.5) / (W, H)      encoder_depthsplat.py:263-273
//   scale = clamp(softplus(head[3:6] - 4), min, max)             gaussian_adapter.py:64-67
//   q = head[6:10] / (|head[6:10]| + 1e-8)  (xyzw)               gaussian_adapter.py:72
//   sh = head[10:].view(3, d_sh) * sh_mask; sh[:, 0] += (rgb - 0.5) / C0   :75-82
//   cov = Rc (R S S^T R^T) Rc^T                                  :85-87, gaussians.py:8-44
//   mean = t + Rc (K^-1 [x, y, 1] / z) * depth                  :90-91, projection.py:91-114
//   harmonics = D_l(Rc) sh  (per degree block)                   :96, sh_rotation.py:10-30
// and the backward of all of it w.r.t. head and depth. Per-view constants (Rc, t, K^-1 and
// the Wigner-D blocks of Rc) come precomputed in a [B*V, 104] float block.
// The operation order follows the torch modules (matmul sums in k = 0, 1, 2 order).

#include "dsplat_common.h"
#include "dga_math.h"

namespace {

using namespace dga;
constexpr int NT = 256;

// UNI (host picks it when H W S % NT == 0): all rows of a workgroup belong to one view, so the
// camera block address is workgroup-uniform and its ~55 reads per row are scalar loads instead
// of per-lane vector loads (the per-lane form kept the adapter at ~3.6 TB/s in config C).
template <int NSH, bool GLUE, bool UNI>
__global__ __launch_bounds__(NT) void k_adapter_fwd(AdIn a, float* __restrict__ means, float* __restrict__ covs,
                                                    float* __restrict__ harm, float* __restrict__ opac,
                                                    float* __restrict__ scales_out, float* __restrict__ rot_out) {
  constexpr int KH = Rows<NSH, GLUE>::kHead, O = Rows<NSH, GLUE>::kOff;
  extern __shared__ __attribute__((aligned(16))) float lds[];  // adapter_fwd_lds(): NT * max(C, 3 NSH + 12) floats
  const size_t total = (size_t)a.BV * a.H * a.W * a.S;
  const size_t n0 = (size_t)blockIdx.x * NT;
  const int nrows = (int)min((size_t)NT, total - n0);
  const int tid = threadIdx.x;
  const int C = a.C;
  Pix px{};
  const bool valid = pixel_of(n0 + tid, a, px);  // outputs share the row order
  const size_t HW = (size_t)a.H * a.W;
  dsplat::stage_in<NT>(a.rows + n0 * C, (size_t)nrows * C, lds);
  __syncthreads();
  float h[KH];
#pragma unroll
  for (int k = 0; k < KH; ++k) h[k] = valid ? lds[tid * C + k] : 0.f;
  __syncthreads();
  float mo[3], Cw[9], ho[3 * NSH], sc[3], q[4];
  if (valid) {
    const float* cam = a.cams + (UNI ? n0 / ((size_t)a.H * a.W * a.S) : px.bv) * kCamFloats;
    adapter_row_fwd<NSH, GLUE>(a, px, cam, h, opac, mo, Cw, ho, sc, q);
  }
  // coalesced row writes through LDS: the three main outputs land in LDS together (harmonics,
  // covariances, means blocks back to back) and leave behind one barrier
  constexpr int kOC = NT * 3 * NSH, kOM = kOC + NT * 9;
  if (valid) {
#pragma unroll
    for (int k = 0; k < 3 * NSH; ++k) lds[tid * (3 * NSH) + k] = ho[k];
#pragma unroll
    for (int k = 0; k < 9; ++k) lds[kOC + tid * 9 + k] = Cw[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) lds[kOM + tid * 3 + k] = mo[k];
  }
  __syncthreads();
  dsplat::stage_out<NT>(harm + n0 * (3 * NSH), (size_t)nrows * (3 * NSH), lds);
  dsplat::stage_out<NT>(covs + n0 * 9, (size_t)nrows * 9, lds + kOC);
  dsplat::stage_out<NT>(means + n0 * 3, (size_t)nrows * 3, lds + kOM);
  const auto put = [&](float* dst, const float* v, int width) {
    __syncthreads();
    if (valid)
      for (int k = 0; k < width; ++k) lds[tid * width + k] = v[k];
    __syncthreads();
    dsplat::stage_out<NT>(dst + n0 * width, (size_t)nrows * width, lds);
  };
  if constexpr (!GLUE) {
    if (scales_out) put(scales_out, sc, 3);
    if (rot_out) put(rot_out, q, 4);
  }
}

template <int NSH, bool GLUE, bool UNI>
__global__ __launch_bounds__(NT) void k_adapter_bwd(AdIn a, const float* __restrict__ dmeans,
                                                    const float* __restrict__ dcovs,
                                                    const float* __restrict__ dharm,
                                                    const float* __restrict__ dopac,
                                                    const float* __restrict__ dscales,
                                                    const float* __restrict__ drot, float* __restrict__ drows,
                                                    float* __restrict__ ddepth, float* __restrict__ dcoords) {
  constexpr int KH = Rows<NSH, GLUE>::kHead, O = Rows<NSH, GLUE>::kOff;
  extern __shared__ __attribute__((aligned(16))) float lds[];  // adapter_lds(): NT * max(C, 3 NSH, 9) floats
  const size_t total = (size_t)a.BV * a.H * a.W * a.S;
  const size_t n0 = (size_t)blockIdx.x * NT;
  const int nrows = (int)min((size_t)NT, total - n0);
  const int tid = threadIdx.x;
  const int C = a.C;
  Pix px{};
  const bool valid = pixel_of(n0 + tid, a, px);
  // rows in: head, then the output gradients (each staged through the same LDS buffer)
  const auto get = [&](const float* src, float* v, int width) {
    if (!src) {
      for (int k = 0; k < width; ++k) v[k] = 0.f;
      return;
    }
    dsplat::stage_in<NT>(src + n0 * width, (size_t)nrows * width, lds);
    __syncthreads();
    for (int k = 0; k < width; ++k) v[k] = valid ? lds[tid * width + k] : 0.f;
    __syncthreads();
  };
  float h[KH], gh[3 * NSH], gCw[9], gm[3], gsc[3], grot[4];
  // the three output-gradient row blocks are prefetched into registers with the head rows
  // (one round trip per workgroup instead of four) when all are present and 16-byte aligned
  constexpr int PH = (3 * NSH + 3) / 4;
  const bool pf = NSH <= 9 && dharm && dcovs && dmeans && dsplat::aligned16(dharm) && dsplat::aligned16(dcovs) &&
                  dsplat::aligned16(dmeans);
  float4 vh[PH], vc[3], vm[1];
  if (pf) {
    dsplat::pref_get<NT>(dharm + n0 * (3 * NSH), (size_t)nrows * (3 * NSH), vh);
    dsplat::pref_get<NT>(dcovs + n0 * 9, (size_t)nrows * 9, vc);
    dsplat::pref_get<NT>(dmeans + n0 * 3, (size_t)nrows * 3, vm);
  }
  const float z = valid ? a.depths[px.n] : 0.f;
  const float gop = (GLUE && valid && dopac) ? dopac[px.n] : 0.f;
  dsplat::stage_in<NT>(a.rows + n0 * C, (size_t)nrows * C, lds);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KH; ++k) h[k] = valid ? lds[tid * C + k] : 0.f;
  __syncthreads();
  if (pf) {
    const auto put_get = [&](const float* src, const auto& v, float* dst, int width) {
      dsplat::pref_put<NT>(src + n0 * width, (size_t)nrows * width, v, lds);
      __syncthreads();
      for (int k = 0; k < width; ++k) dst[k] = valid ? lds[tid * width + k] : 0.f;
      __syncthreads();
    };
    put_get(dharm, vh, gh, 3 * NSH);
    put_get(dcovs, vc, gCw, 9);
    put_get(dmeans, vm, gm, 3);
  } else {
    get(dharm, gh, 3 * NSH);
    get(dcovs, gCw, 9);
    get(dmeans, gm, 3);
  }
  get(GLUE ? nullptr : dscales, gsc, 3);
  get(GLUE ? nullptr : drot, grot, 4);
  float dh[KH];
#pragma unroll
  for (int k = 0; k < KH; ++k) dh[k] = 0.f;
  float gxy[2] = {0.f, 0.f};
  if (valid) {
    const float* cam = a.cams + (UNI ? n0 / ((size_t)a.H * a.W * a.S) : px.bv) * kCamFloats;
    adapter_row_bwd<NSH, GLUE>(a, px, cam, h, z, gm, gCw, gh, gop, dopac != nullptr, gsc, grot, dh, gxy, ddepth);
  }
  // drows out through LDS (channels past the used ones are 0)
  if (valid) {
#pragma unroll
    for (int k = 0; k < KH; ++k) lds[tid * C + k] = dh[k];
    for (int k = KH; k < C; ++k) lds[tid * C + k] = 0.f;
  }
  __syncthreads();
  dsplat::stage_out<NT>(drows + n0 * C, (size_t)nrows * C, lds);
  if constexpr (!GLUE) {
    if (dcoords) {
      __syncthreads();
      if (valid) {
        lds[tid * 2] = gxy[0];
        lds[tid * 2 + 1] = gxy[1];
      }
      __syncthreads();
      dsplat::stage_out<NT>(dcoords + n0 * 2, (size_t)nrows * 2, lds);
    }
  }
}

// Per-view constant blocks (dga_adapter_cameras): R, t of c2w, K^-1 (double, adjugate) and
// the Wigner-D matrices of R for degrees 1..3, solved exactly as sh_rotation.wigner_d does:
// D_l = Y_l(R x_n)^T pinv(Y_l(x_n))^T over fixed probe directions x_n (same probes and
// pseudo-inverses, passed in double), so the fused and torch adapters rotate identically.
__device__ void e3nn_sh(int l, double x, double y, double z, double* out) {
  const double s3 = 1.7320508075688772;
  if (l == 1) {
    out[0] = x;
    out[1] = y;
    out[2] = z;
    return;
  }
  const double y2 = y * y, x2z2 = x * x + z * z, s20 = s3 * x * z, s24 = s3 / 2.0 * (z * z - x * x);
  if (l == 2) {
    out[0] = s20;
    out[1] = s3 * x * y;
    out[2] = y2 - 0.5 * x2z2;
    out[3] = s3 * y * z;
    out[4] = s24;
    return;
  }
  out[0] = sqrt(5.0 / 6.0) * (s20 * z + s24 * x);
  out[1] = sqrt(5.0) * s20 * y;
  out[2] = sqrt(3.0 / 8.0) * (4 * y2 - x2z2) * x;
  out[3] = 0.5 * y * (2 * y2 - 3 * x2z2);
  out[4] = sqrt(3.0 / 8.0) * z * (4 * y2 - x2z2);
  out[5] = sqrt(5.0) * s24 * y;
  out[6] = sqrt(5.0 / 6.0) * (s24 * z - s20 * x);
}

__global__ void k_adapter_cams(int BV, const float* __restrict__ ext, const float* __restrict__ intr, int sh_degree,
                               const double* __restrict__ probes, float* __restrict__ cams) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= BV) return;
  const float* E = ext + (size_t)v * 16;
  const float* K = intr + (size_t)v * 9;
  float* o = cams + (size_t)v * kCamFloats;
  double R[9];
  for (int a = 0; a < 3; ++a) {
    for (int c = 0; c < 3; ++c) {
      R[a * 3 + c] = E[a * 4 + c];
      o[kOffR + a * 3 + c] = E[a * 4 + c];
    }
    o[kOffT + a] = E[a * 4 + 3];
  }
  {
    const double a = K[0], b = K[1], c = K[2], d = K[3], e = K[4], f = K[5], g = K[6], h = K[7], i = K[8];
    const double A = e * i - f * h, Bc = -(d * i - f * g), Cc = d * h - e * g;
    const double id = 1.0 / (a * A + b * Bc + c * Cc);
    const double inv[9] = {A * id, -(b * i - c * h) * id, (b * f - c * e) * id,
                           Bc * id, (a * i - c * g) * id, -(a * f - c * d) * id,
                           Cc * id, -(a * h - b * g) * id, (a * e - b * d) * id};
    for (int k = 0; k < 9; ++k) o[kOffKinv + k] = (float)inv[k];
  }
  const double* pr = probes;
  for (int l = 1; l <= 3; ++l) {
    const int n = 2 * l + 1, np = 4 * n + 8;
    const double* pts = pr;             // [np, 3]
    const double* pinv = pr + 3 * np;   // [n, np]
    pr += 3 * np + n * np;
    float* D = o + (l == 1 ? kOffD1 : l == 2 ? kOffD2 : kOffD3);
    if (l > sh_degree) {
      for (int k = 0; k < n * n; ++k) D[k] = 0.f;
      continue;
    }
    double acc[49];
    for (int k = 0; k < n * n; ++k) acc[k] = 0.0;
    for (int p = 0; p < np; ++p) {
      const double x = pts[3 * p], y = pts[3 * p + 1], z = pts[3 * p + 2];
      const double rx = R[0] * x + R[1] * y + R[2] * z;
      const double ry = R[3] * x + R[4] * y + R[5] * z;
      const double rz = R[6] * x + R[7] * y + R[8] * z;
      double Y[7];
      e3nn_sh(l, rx, ry, rz, Y);
      for (int k = 0; k < n; ++k)
        for (int m = 0; m < n; ++m) acc[k * n + m] += Y[k] * pinv[m * np + p];
    }
    for (int k = 0; k < n * n; ++k) D[k] = (float)acc[k];
  }
}

}  // namespace

namespace {
size_t adapter_lds(int C, int d_sh) { return (size_t)NT * (size_t)max(max(C, 3 * d_sh), 9) * sizeof(float); }
// forward: also the three output blocks at once (3 d_sh + 9 + 3 floats per row)
size_t adapter_fwd_lds(int C, int d_sh) { return (size_t)NT * (size_t)max(C, 3 * d_sh + 12) * sizeof(float); }

template <int NS, bool GLUE>
int launch_fwd(const AdIn& a, float* means, float* covs, float* harm, float* opac, float* scales, float* rots,
               hipStream_t st) {
  const size_t n = (size_t)a.BV * a.H * a.W * a.S;
  const size_t lds = adapter_fwd_lds(a.C, NS);
  if (lds > 64 * 1024 &&
      (hipFuncSetAttribute((const void*)k_adapter_fwd<NS, GLUE, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)lds) != hipSuccess ||
       hipFuncSetAttribute((const void*)k_adapter_fwd<NS, GLUE, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)lds) != hipSuccess))
    return dsplat::check_launch("hipFuncSetAttribute(k_adapter_fwd)");
  if ((size_t)a.H * a.W * a.S % NT == 0)
    k_adapter_fwd<NS, GLUE, true><<<(unsigned)((n + NT - 1) / NT), NT, lds, st>>>(a, means, covs, harm, opac, scales, rots);
  else
    k_adapter_fwd<NS, GLUE, false><<<(unsigned)((n + NT - 1) / NT), NT, lds, st>>>(a, means, covs, harm, opac, scales, rots);
  return dsplat::check_launch("k_adapter_fwd");
}
template <int NS, bool GLUE>
int launch_bwd(const AdIn& a, const float* dmeans, const float* dcovs, const float* dharm, const float* dopac,
               const float* dscales, const float* drot, float* drows, float* ddepth, float* dcoords, hipStream_t st) {
  const size_t n = (size_t)a.BV * a.H * a.W * a.S;
  const size_t lds = adapter_lds(a.C, NS);
  if (lds > 64 * 1024 &&
      (hipFuncSetAttribute((const void*)k_adapter_bwd<NS, GLUE, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)lds) != hipSuccess ||
       hipFuncSetAttribute((const void*)k_adapter_bwd<NS, GLUE, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)lds) != hipSuccess))
    return dsplat::check_launch("hipFuncSetAttribute(k_adapter_bwd)");
  if ((size_t)a.H * a.W * a.S % NT == 0)
    k_adapter_bwd<NS, GLUE, true><<<(unsigned)((n + NT - 1) / NT), NT, lds, st>>>(a, dmeans, dcovs, dharm, dopac,
                                                                                 dscales, drot, drows, ddepth, dcoords);
  else
    k_adapter_bwd<NS, GLUE, false><<<(unsigned)((n + NT - 1) / NT), NT, lds, st>>>(a, dmeans, dcovs, dharm, dopac,
                                                                                  dscales, drot, drows, ddepth, dcoords);
  return dsplat::check_launch("k_adapter_bwd");
}
#define DGA_DISPATCH(d_sh, CALL) \
  switch (d_sh) {                \
    case 1: return CALL(1);      \
    case 4: return CALL(4);      \
    case 9: return CALL(9);      \
    default: return CALL(16);    \
  }

// ---- head rows: pixel shuffle + "(b v) c h w -> b v (h w) c" in one LDS-tiled pass ---------
// rows[bv][(hh r + i) W + ww r + j][c] = x[bv][c r^2 + i r + j][hh][ww] (W = w r): the head's
// conv output [BV, C r^2, h, w] to the per-pixel rows the adapter reads (encoder_depthsplat.py
// rearranges its head output the same way), and the inverse for the backward. One workgroup
// per (bv, output row hh r + i, kRowTile columns ww): the C r x kRowTile input block is read as
// kRowTile-float runs, transposed through LDS, and written as one contiguous run of
// kRowTile r C floats (a strided torch permute of the 1.2 GB config-D head moved ~1 TB/s).
template <int kRowTile>  // columns ww per workgroup: 32 = whole 128-byte lines when the tile fits
__global__ __launch_bounds__(256) void k_head_rows(int C, int r, int h, int w, float* __restrict__ x,
                                                   float* __restrict__ rows, int inverse) {
  extern __shared__ float s_tile[];  // [kRowTile r][C] (+1 pad per r C row group)
  const int bv = blockIdx.z, hr = blockIdx.y, hh = hr / r, i = hr - hh * r;
  const int ww0 = blockIdx.x * kRowTile, nw = min(kRowTile, w - ww0);
  const int W = w * r, CR = C * r, stride = C + 1;  // odd row stride: the transposed accesses spread over banks
  const size_t plane = (size_t)h * w;
  float* xb = x + ((size_t)bv * C * r * r + (size_t)i * r) * plane + (size_t)hh * w + ww0;
  const size_t rbase = ((size_t)bv * h * r * W + (size_t)hr * W + (size_t)ww0 * r) * C;
  const int n_in = CR * kRowTile, n_out = nw * r * C;
  if (!inverse) {
    for (int e = threadIdx.x; e < n_in; e += 256) {
      const int q = e / kRowTile, k = e - q * kRowTile;  // q = c r + j
      if (k >= nw) continue;
      const int c = q / r, j = q - c * r;
      s_tile[(k * r + j) * stride + c] = xb[((size_t)c * r * r + j) * plane + k];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < n_out; e += 256) {
      const int p = e / C, c = e - p * C;
      rows[rbase + e] = s_tile[p * stride + c];
    }
  } else {
    for (int e = threadIdx.x; e < n_out; e += 256) {
      const int p = e / C, c = e - p * C;
      s_tile[p * stride + c] = rows[rbase + e];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < n_in; e += 256) {
      const int q = e / kRowTile, k = e - q * kRowTile;
      if (k >= nw) continue;
      const int c = q / r, j = q - c * r;
      xb[((size_t)c * r * r + j) * plane + k] = s_tile[(k * r + j) * stride + c];
    }
  }
}
size_t head_rows_lds(int tile, int C, int r) { return sizeof(float) * (size_t)tile * r * (C + 1); }
int head_rows_launch(int BV, int C, int r, int h, int w, float* x, float* rows, int inverse, hipStream_t st) {
  const int tile = head_rows_lds(32, C, r) <= 64 * 1024 ? 32 : 16;
  const size_t lds = head_rows_lds(tile, C, r);
  DSPLAT_REQUIRE(lds <= 64 * 1024, "dga_head_rows: %d channels x %d exceed the LDS tile", C, r);
  if (tile == 32)
    k_head_rows<32><<<dim3((w + 31) / 32, h * r, BV), 256, lds, st>>>(C, r, h, w, x, rows, inverse);
  else
    k_head_rows<16><<<dim3((w + 15) / 16, h * r, BV), 256, lds, st>>>(C, r, h, w, x, rows, inverse);
  return dsplat::check_launch("k_head_rows");
}
}  // namespace

extern "C" {

int dga_adapter_cameras(int BV, const float* extrinsics, const float* intrinsics, int sh_degree, const double* probes,
                        float* cams, void* stream) {
  DSPLAT_REQUIRE(BV > 0 && sh_degree >= 0 && sh_degree <= 3, "dga_adapter_cameras: BV=%d sh_degree=%d", BV, sh_degree);
  DSPLAT_REQUIRE(extrinsics && intrinsics && probes && cams, "dga_adapter_cameras: null pointer");
  k_adapter_cams<<<(BV + 63) / 64, 64, 0, (hipStream_t)stream>>>(BV, extrinsics, intrinsics, sh_degree, probes, cams);
  return dsplat::check_launch("k_adapter_cams");
}


int dga_adapter_fwd(int B, int V, int H, int W, int d_sh, int C, const float* head, const float* depths,
                    const float* images, const float* cams, float scale_min, float scale_max, const float* sh_mask,
                    float* means, float* covariances, float* harmonics, float* opacities, void* stream) {
  DSPLAT_REQUIRE(B > 0 && V > 0 && H > 0 && W > 0, "dga_adapter_fwd: bad sizes");
  DSPLAT_REQUIRE(d_sh == 1 || d_sh == 4 || d_sh == 9 || d_sh == 16, "dga_adapter_fwd: d_sh=%d (1, 4, 9, 16)", d_sh);
  DSPLAT_REQUIRE(C >= 10 + 3 * d_sh, "dga_adapter_fwd: %d head channels < 10 + 3*d_sh", C);
  DSPLAT_REQUIRE(head && depths && images && cams && sh_mask && means && covariances && harmonics && opacities,
                 "dga_adapter_fwd: null pointer");
  DSPLAT_REQUIRE(adapter_fwd_lds(C, d_sh) <= 160 * 1024, "dga_adapter_fwd: %d head channels exceed the LDS row staging", C);
  const AdIn a{head, nullptr, depths, images, cams, sh_mask, scale_min, scale_max, 1e-8f, C, B * V, H, W, 1};
  hipStream_t st = (hipStream_t)stream;
#define DGA_F(NS) launch_fwd<NS, true>(a, means, covariances, harmonics, opacities, nullptr, nullptr, st)
  DGA_DISPATCH(d_sh, DGA_F)
#undef DGA_F
}

int dga_adapter_bwd(int B, int V, int H, int W, int d_sh, int C, const float* head, const float* depths,
                    const float* cams, float scale_min, float scale_max, const float* sh_mask, const float* dmeans,
                    const float* dcovariances, const float* dharmonics, const float* dopacities, float* dhead,
                    float* ddepths, void* stream) {
  DSPLAT_REQUIRE(B > 0 && V > 0 && H > 0 && W > 0, "dga_adapter_bwd: bad sizes");
  DSPLAT_REQUIRE(d_sh == 1 || d_sh == 4 || d_sh == 9 || d_sh == 16, "dga_adapter_bwd: d_sh=%d (1, 4, 9, 16)", d_sh);
  DSPLAT_REQUIRE(C >= 10 + 3 * d_sh, "dga_adapter_bwd: %d head channels < 10 + 3*d_sh", C);
  DSPLAT_REQUIRE(head && depths && cams && sh_mask && dhead, "dga_adapter_bwd: null pointer");
  DSPLAT_REQUIRE(adapter_lds(C, d_sh) <= 160 * 1024, "dga_adapter_bwd: %d head channels exceed the LDS row staging", C);
  const AdIn a{head, nullptr, depths, nullptr, cams, sh_mask, scale_min, scale_max, 1e-8f, C, B * V, H, W, 1};
  hipStream_t st = (hipStream_t)stream;
#define DGA_B(NS) \
  launch_bwd<NS, true>(a, dmeans, dcovariances, dharmonics, dopacities, nullptr, nullptr, dhead, ddepths, nullptr, st)
  DGA_DISPATCH(d_sh, DGA_B)
#undef DGA_B
}

int dga_adapter_forward(int BV, int H, int W, int S, int d_sh, int C, const float* raw, const float* coordinates,
                        const float* depths, const float* images, const float* cams, float scale_min,
                        float scale_max, const float* sh_mask, float eps, float* means, float* covariances,
                        float* harmonics, float* scales, float* rotations, void* stream) {
  DSPLAT_REQUIRE(BV > 0 && H > 0 && W > 0 && S > 0, "dga_adapter_forward: bad sizes");
  DSPLAT_REQUIRE(d_sh == 1 || d_sh == 4 || d_sh == 9 || d_sh == 16, "dga_adapter_forward: d_sh=%d (1, 4, 9, 16)", d_sh);
  DSPLAT_REQUIRE(C >= 7 + 3 * d_sh, "dga_adapter_forward: %d raw channels < 7 + 3*d_sh", C);
  DSPLAT_REQUIRE(raw && coordinates && depths && images && cams && sh_mask && means && covariances && harmonics,
                 "dga_adapter_forward: null pointer");
  DSPLAT_REQUIRE(adapter_fwd_lds(C, d_sh) <= 160 * 1024, "dga_adapter_forward: %d channels exceed the LDS row staging", C);
  const AdIn a{raw, coordinates, depths, images, cams, sh_mask, scale_min, scale_max, eps, C, BV, H, W, S};
  hipStream_t st = (hipStream_t)stream;
#define DGA_F(NS) launch_fwd<NS, false>(a, means, covariances, harmonics, nullptr, scales, rotations, st)
  DGA_DISPATCH(d_sh, DGA_F)
#undef DGA_F
}

int dga_adapter_backward(int BV, int H, int W, int S, int d_sh, int C, const float* raw, const float* coordinates,
                         const float* depths, const float* cams, float scale_min, float scale_max,
                         const float* sh_mask, float eps, const float* dmeans, const float* dcovariances,
                         const float* dharmonics, const float* dscales, const float* drotations, float* draw,
                         float* dcoordinates, float* ddepths, void* stream) {
  DSPLAT_REQUIRE(BV > 0 && H > 0 && W > 0 && S > 0, "dga_adapter_backward: bad sizes");
  DSPLAT_REQUIRE(d_sh == 1 || d_sh == 4 || d_sh == 9 || d_sh == 16, "dga_adapter_backward: d_sh=%d", d_sh);
  DSPLAT_REQUIRE(C >= 7 + 3 * d_sh, "dga_adapter_backward: %d raw channels < 7 + 3*d_sh", C);
  DSPLAT_REQUIRE(raw && coordinates && depths && cams && sh_mask && draw, "dga_adapter_backward: null pointer");
  DSPLAT_REQUIRE(adapter_lds(C, d_sh) <= 160 * 1024, "dga_adapter_backward: %d channels exceed the LDS row staging", C);
  const AdIn a{raw, coordinates, depths, nullptr, cams, sh_mask, scale_min, scale_max, eps, C, BV, H, W, S};
  hipStream_t st = (hipStream_t)stream;
#define DGA_B(NS) \
  launch_bwd<NS, false>(a, dmeans, dcovariances, dharmonics, nullptr, dscales, drotations, draw, ddepths, dcoordinates, st)
  DGA_DISPATCH(d_sh, DGA_B)
#undef DGA_B
}

int dga_head_rows(int BV, int C, int r, int h, int w, const float* x, float* rows, void* stream) {
  DSPLAT_REQUIRE(BV > 0 && C > 0 && r > 0 && h > 0 && w > 0, "dga_head_rows: bad sizes");
  DSPLAT_REQUIRE(x && rows, "dga_head_rows: null pointer");
  return head_rows_launch(BV, C, r, h, w, const_cast<float*>(x), rows, 0, (hipStream_t)stream);  // x only read
}

int dga_head_rows_bwd(int BV, int C, int r, int h, int w, const float* drows, float* dx, void* stream) {
  DSPLAT_REQUIRE(BV > 0 && C > 0 && r > 0 && h > 0 && w > 0, "dga_head_rows_bwd: bad sizes");
  DSPLAT_REQUIRE(drows && dx, "dga_head_rows_bwd: null pointer");
  return head_rows_launch(BV, C, r, h, w, dx, const_cast<float*>(drows), 1, (hipStream_t)stream);  // drows only read
}

}  // extern "C"
