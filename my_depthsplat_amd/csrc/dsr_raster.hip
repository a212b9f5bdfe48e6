// dsr_raster.hip — MI355X (gfx950, wave64) differentiable 3D-Gaussian tile rasterizer.
//
// Replaces the external CUDA library `diff_gaussian_rasterization` that the reference
// calls at src/model/decoder/cuda_splatting.py:112-123 (requirements.txt:23). The
// algorithm is the published 3DGS one; the structure is
// MI355X-first:
//   * one launch sequence renders a whole batch of views of many scenes (no per-view
//     Python loop, no .item() syncs, no Gaussian x views materialisation);
//   * binning is a per-(view, tile) bucket pass (LDS histogram + one global atomic per
//     bucket per workgroup) followed by a per-tile LSD radix sort of (depth, id) keys in
//     LDS (wave64 ballot ranking) — no device-wide sort passes over HBM;
//   * the backward reduces each Gaussian's per-pixel gradients across the wave in
//     registers first and issues one 64-bit fixed-point atomic per (sub-tile wave, Gaussian,
//     component) instead of one float atomic per pixel: integer sums are order-independent,
//     so the gradients are bit-identical run to run.
// All floating-point expressions feeding the bit-exact outputs (depth, radius, xy, tile
// rect, sort keys) keep the evaluation order of oracle/dsr_oracle.cpp (-ffp-contract=off).

#include <cstdlib>
#include <type_traits>
#include <utility>

#include "dsplat_common.h"
#include "dga_math.h"

namespace {

using dsplat::kWave;
constexpr int BX = DSR_TILE, BY = DSR_TILE;
constexpr int NT = BX * BY;  // 256 threads = 4 waves per tile
constexpr int GS = DSR_GEOM_STRIDE;
constexpr uint32_t kSortCap = 8192;           // max keys sorted in LDS (2 x 64 KiB)
constexpr int kSortNT = 256;       // threads per segment in the LDS sort
constexpr int kSortNBinLog2 = 13;  // counting-sort depth bins (8192)
constexpr int kSortWPE = 3;        // waves per EU of the sort kernels: all config-B segments resident
// LDS words of the sort's counter area: the LSD passes' u16 counters (16 per thread) or the
// counting sort's u16 bins, whichever is larger
template <int NTH, int NBL = kSortNBinLog2>
constexpr int sort_cnt_words() {
  return NTH * 8 > (1 << NBL) / 2 ? NTH * 8 : (1 << NBL) / 2;
}
constexpr int kHistLdsMax = 32768;            // tiles per view histogrammed in LDS

constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f, SH_C2_1 = -1.0925484305920792f,
                SH_C2_2 = 0.31539156525252005f, SH_C2_3 = -1.0925484305920792f,
                SH_C2_4 = 0.5462742152960396f;
constexpr float SH_C3_0 = -0.5900435899266435f, SH_C3_1 = 2.890611442640554f,
                SH_C3_2 = -0.4570457994644658f, SH_C3_3 = 0.3731763325901154f,
                SH_C3_4 = -0.4570457994644658f, SH_C3_5 = 1.445305721320277f,
                SH_C3_6 = -0.5900435899266435f;

struct F3 {
  float x, y, z;
};

// The projection chain is written with explicit FMAs in a fixed order (the file is compiled
// with -ffp-contract=off, so no other contraction happens); oracle/dsr_oracle.cpp evaluates
// the same sequence with std::fma, which keeps depth, radius, xy, conic, rgb and the tile
// lists bit-identical while each multiply-add is one instruction.
__device__ __forceinline__ F3 xform43(const float* m, F3 p) {
  F3 r;
  r.x = fmaf(m[0], p.x, fmaf(m[4], p.y, fmaf(m[8], p.z, m[12])));
  r.y = fmaf(m[1], p.x, fmaf(m[5], p.y, fmaf(m[9], p.z, m[13])));
  r.z = fmaf(m[2], p.x, fmaf(m[6], p.y, fmaf(m[10], p.z, m[14])));
  return r;
}
__device__ __forceinline__ float xform44w(const float* m, F3 p) {
  return fmaf(m[3], p.x, fmaf(m[7], p.y, fmaf(m[11], p.z, m[15])));
}
// Upstream (and the oracle) evaluate ((v + 1.0) * S - 1.0) * 0.5 in double: every step is exact
// there (a float v, an integer S < 2^24), so the result is the exact value rounded once to
// float. One float FMA gives the same single rounding of (v + 1) S - 1 = v S + (S - 1), and the
// halving is exact: bit-identical, two float instructions instead of six double ones.
__device__ __forceinline__ float ndc2pix(float v, int S) {
  return 0.5f * fmaf(v, (float)S, (float)(S - 1));
}
__device__ __forceinline__ void tile_rect(float px, float py, int r, int gx, int gy, int& x0, int& y0,
                                          int& x1, int& y1) {
  x0 = min(gx, max(0, (int)((px - r) / BX)));
  y0 = min(gy, max(0, (int)((py - r) / BY)));
  x1 = min(gx, max(0, (int)((px + r + BX - 1) / BX)));
  y1 = min(gy, max(0, (int)((py + r + BY - 1) / BY)));
}

// Per-wave balanced expansion of tile rectangles: the wave's (Gaussian, tile) pairs are
// numbered by an exclusive scan of the rect areas and handed out 64 at a time, so one lane
// with a huge rect no longer serialises its whole wave (radii are heavy-tailed: a few
// Gaussians touch hundreds of tiles, the median touches one or two). f(tile, owner lane)
// runs once per pair; ws_* are this wave's 64-entry LDS slots.
// Workgroup -> (view, block) placement by XCD. Workgroups are dispatched round-robin over
// the 8 XCDs (id % 8), each with its own L2. The (view, block) items are cut into 8
// contiguous ranges, one per XCD, so a view's segments are written (keys) and counted
// (atomics) through one or two L2s instead of all eight: 8-byte key stores to a segment's
// frontier lines then merge in that L2 before write-back, and count atomics stay local.
// grid.x = 8 * ceil(items / 8); returns false for the padding workgroups.
__device__ __forceinline__ bool xcd_item(int blocks_per_view, int V, int& v, int& blk) {
  const int items = blocks_per_view * V;
  const int per = (items + 7) >> 3;
  const int item = (int)(blockIdx.x & 7u) * per + (int)(blockIdx.x >> 3);
  if ((int)(blockIdx.x >> 3) >= per || item >= items) return false;
  v = item / blocks_per_view;
  blk = item - v * blocks_per_view;
  return true;
}
__host__ __device__ constexpr unsigned xcd_grid(int blocks_per_view, int V) {
  return 8u * (unsigned)((blocks_per_view * V + 7) / 8);
}
// Placement that keeps the views of one Gaussian block together instead: the items are
// (major, minor) pairs in major-major order (major = Gaussian block, minor = view), cut into 8
// contiguous per-XCD ranges as above. The V views of a block then run in consecutive slots
// of one XCD and read the block's 148 B per Gaussian from HBM once, from that XCD's L2 after
// (project / preprocess kernels; k_project_emit at config B: 95 -> 54 MB of HBM traffic per
// launch). Same grid size as xcd_grid(n_major, n_minor).
__device__ __forceinline__ bool xcd_pair(int n_major, int n_minor, int& major, int& minor) {
  const int items = n_major * n_minor;
  const int per = (items + 7) >> 3;
  const int item = (int)(blockIdx.x & 7u) * per + (int)(blockIdx.x >> 3);
  if ((int)(blockIdx.x >> 3) >= per || item >= items) return false;
  major = item / n_minor;
  minor = item - major * n_minor;
  return true;
}

// Scene-major variant for views grouped by scene (views_per_scene vps > 0: views s vps .. s vps
// + vps - 1 render scene s): items ordered (scene, block, view of the scene), cut into the 8
// per-XCD ranges. With S >= 8 scenes an XCD holds whole scenes: the views of a block still
// share its inputs through one L2, and every tile segment of a scene's views receives its
// keys from one XCD (frontier lines merge in one L2 instead of coming back as up to 8 partial
// writes). vps = 0: xcd_pair(n_blocks, V).
__device__ __forceinline__ bool xcd_scene_major(int n_blocks, int V, int vps, int& blk, int& v) {
  if (vps <= 0) return xcd_pair(n_blocks, V, blk, v);
  const int items = n_blocks * V;
  const int per = (items + 7) >> 3;
  const int item = (int)(blockIdx.x & 7u) * per + (int)(blockIdx.x >> 3);
  if ((int)(blockIdx.x >> 3) >= per || item >= items) return false;
  const int per_scene = n_blocks * vps;
  const int s = item / per_scene, r = item - s * per_scene;
  blk = r / vps;
  v = s * vps + (r - blk * vps);
  return true;
}

struct WaveRects {
  uint32_t ex[64];    // exclusive scan of areas
  uint32_t org[64];   // x0 | y0 << 16
  uint32_t wid[64];   // rect width in tiles
  uint32_t mark[64];  // owner + 1 of each window slot where a rect's run of pairs begins
};
// Pairs are handed out 64 per step: the owner of pair j is the lane whose run [ex, ex + area)
// holds j, found per window by marking each run's first slot and a wave max-scan of the
// marks (DPP, no dependent LDS search); the tile comes from (j - ex) / width with a hardware
// reciprocal and exact integer fix-ups. f(tile, owner lane[, tile x, tile y]).
// pre(owner) runs on every lane of each 64-pair window before f, outside the j < total
// branch, so it may use cross-lane operations (ds_bpermute needs its source lanes active).
struct NoPre {
  __device__ void operator()(int) const {}
};
template <typename F, typename P = NoPre>
__device__ __forceinline__ uint32_t for_each_rect_tile(WaveRects& wr, int lane, int x0, int y0, int x1, int y1,
                                                       bool has, int gx, F f, P pre = P{}) {
  const uint32_t area = has ? (uint32_t)((x1 - x0) * (y1 - y0)) : 0u;
  const uint32_t incl = dsplat::wave_incl_add_dpp(area);
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  const uint32_t ex = incl - area;
  wr.ex[lane] = ex;
  wr.org[lane] = (uint32_t)x0 | ((uint32_t)y0 << 16);
  wr.wid[lane] = (uint32_t)max(x1 - x0, 1);
  uint32_t carry = 0u;  // owner + 1 of the window's first slot when no run starts there
  for (uint32_t base = 0; base < total; base += 64) {
    wr.mark[lane] = 0u;
    __builtin_amdgcn_wave_barrier();
    if (area != 0u && ex - base < 64u) wr.mark[ex - base] = (uint32_t)lane + 1u;
    __builtin_amdgcn_wave_barrier();
    uint32_t m = wr.mark[lane];
    if (lane == 0) m = max(m, carry);
    const uint32_t own = dsplat::wave_incl_max_dpp(m);
    carry = (uint32_t)__builtin_amdgcn_readlane((int)own, 63);
    pre(max((int)own - 1, 0));
    const uint32_t j = base + (uint32_t)lane;
    if (j < total) {
      const int o = (int)own - 1;
      const uint32_t local = j - wr.ex[o];
      const uint32_t wd = wr.wid[o];
      uint32_t dy = (uint32_t)(((float)local + 0.5f) * __builtin_amdgcn_rcpf((float)wd));
      if (dy * wd > local) --dy;
      if ((dy + 1) * wd <= local) ++dy;
      const uint32_t og = wr.org[o];
      const int tx = (int)((og & 0xFFFFu) + local - dy * wd), ty = (int)((og >> 16) + dy);
      if constexpr (std::is_invocable_v<F, int, int, int, int>)
        f(ty * gx + tx, o, tx, ty);
      else
        f(ty * gx + tx, o);
    }
    __builtin_amdgcn_wave_barrier();
  }
  return total;
}

// The same balanced hand-out, with f(valid, tile, owner, tile x, tile y) called on EVERY lane of
// each 64-pair window (valid: this lane holds a pair), so f may itself run wave-wide code (a
// nested for_each_rect_tile over a second WaveRects).
template <typename F>
__device__ __forceinline__ void for_each_rect_window(WaveRects& wr, int lane, int x0, int y0, int x1, int y1,
                                                     bool has, int gx, F f) {
  const uint32_t area = has ? (uint32_t)((x1 - x0) * (y1 - y0)) : 0u;
  const uint32_t incl = dsplat::wave_incl_add_dpp(area);
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  const uint32_t ex = incl - area;
  wr.ex[lane] = ex;
  wr.org[lane] = (uint32_t)x0 | ((uint32_t)y0 << 16);
  wr.wid[lane] = (uint32_t)max(x1 - x0, 1);
  uint32_t carry = 0u;
  for (uint32_t base = 0; base < total; base += 64) {
    wr.mark[lane] = 0u;
    __builtin_amdgcn_wave_barrier();
    if (area != 0u && ex - base < 64u) wr.mark[ex - base] = (uint32_t)lane + 1u;
    __builtin_amdgcn_wave_barrier();
    uint32_t m = wr.mark[lane];
    if (lane == 0) m = max(m, carry);
    const uint32_t own = dsplat::wave_incl_max_dpp(m);
    carry = (uint32_t)__builtin_amdgcn_readlane((int)own, 63);
    const uint32_t j = base + (uint32_t)lane;
    const int o = max((int)own - 1, 0);
    const uint32_t local = j < total ? j - wr.ex[o] : 0u;
    const uint32_t wd = wr.wid[o];
    uint32_t dy = (uint32_t)(((float)local + 0.5f) * __builtin_amdgcn_rcpf((float)wd));
    if (dy * wd > local) --dy;
    if ((dy + 1) * wd <= local) ++dy;
    const uint32_t og = wr.org[o];
    const int tx = (int)((og & 0xFFFFu) + local - dy * wd), ty = (int)((og >> 16) + dy);
    __builtin_amdgcn_wave_barrier();
    f(j < total, ty * gx + tx, o, tx, ty);
    __builtin_amdgcn_wave_barrier();
  }
}

struct Cov2D {
  float T[2][3];
  float a, b, c;
  float tx, ty, tz;
  float xmul, ymul;
};

// EWA: cov2D = J Wr Sigma Wr^T J^T + 0.3 I. Same evaluation order as
// the oracle so radius/conic are bit-identical.
__device__ __forceinline__ void cov2d(F3 mean, float fx, float fy, float tanx, float tany,
                                      const float c6[6], const float* view, Cov2D& w) {
  F3 t = xform43(view, mean);
  const float limx = 1.3f * tanx;
  const float limy = 1.3f * tany;
  const float txtz = t.x / t.z;
  const float tytz = t.y / t.z;
  w.xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
  w.ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
  t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
  t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
  w.tx = t.x;
  w.ty = t.y;
  w.tz = t.z;
  const float j00 = fx / t.z;
  const float j02 = -(fx * t.x) / (t.z * t.z);
  const float j11 = fy / t.z;
  const float j12 = -(fy * t.y) / (t.z * t.z);
  const float W00 = view[0], W01 = view[4], W02 = view[8];
  const float W10 = view[1], W11 = view[5], W12 = view[9];
  const float W20 = view[2], W21 = view[6], W22 = view[10];
  w.T[0][0] = fmaf(j00, W00, j02 * W20);
  w.T[0][1] = fmaf(j00, W01, j02 * W21);
  w.T[0][2] = fmaf(j00, W02, j02 * W22);
  w.T[1][0] = fmaf(j11, W10, j12 * W20);
  w.T[1][1] = fmaf(j11, W11, j12 * W21);
  w.T[1][2] = fmaf(j11, W12, j12 * W22);
  const float V[3][3] = {{c6[0], c6[1], c6[2]}, {c6[1], c6[3], c6[4]}, {c6[2], c6[4], c6[5]}};
  float U[2][3];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) U[r][c] = fmaf(w.T[r][0], V[0][c], fmaf(w.T[r][1], V[1][c], w.T[r][2] * V[2][c]));
  const float a = fmaf(U[0][0], w.T[0][0], fmaf(U[0][1], w.T[0][1], U[0][2] * w.T[0][2]));
  const float b = fmaf(U[0][0], w.T[1][0], fmaf(U[0][1], w.T[1][1], U[0][2] * w.T[1][2]));
  const float c = fmaf(U[1][0], w.T[1][0], fmaf(U[1][1], w.T[1][1], U[1][2] * w.T[1][2]));
  w.a = a + 0.3f;
  w.b = b;
  w.c = c + 0.3f;
}

// SH (degree DEG) -> one colour channel; s(k) = coefficient k of this channel.
// The basis values (channel-independent) are formed first, then each channel is accumulated
// coefficient by coefficient with one FMA each (oracle: sh_to_rgb, same order).
template <int DEG>
__device__ __forceinline__ float sh_eval(const float* sh, int ch, float x, float y, float z) {
  auto s = [&](int k) { return sh[k * 3 + ch]; };
  float v = SH_C0 * s(0);
  if constexpr (DEG > 0) {
    v = fmaf(-(SH_C1 * y), s(1), v);
    v = fmaf(SH_C1 * z, s(2), v);
    v = fmaf(-(SH_C1 * x), s(3), v);
    if constexpr (DEG > 1) {
      const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
      v = fmaf(SH_C2_0 * xy, s(4), v);
      v = fmaf(SH_C2_1 * yz, s(5), v);
      v = fmaf(SH_C2_2 * (2.0f * zz - xx - yy), s(6), v);
      v = fmaf(SH_C2_3 * xz, s(7), v);
      v = fmaf(SH_C2_4 * (xx - yy), s(8), v);
      if constexpr (DEG > 2) {
        v = fmaf(SH_C3_0 * y * (3.0f * xx - yy), s(9), v);
        v = fmaf(SH_C3_1 * xy * z, s(10), v);
        v = fmaf(SH_C3_2 * y * (4.0f * zz - xx - yy), s(11), v);
        v = fmaf(SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy), s(12), v);
        v = fmaf(SH_C3_4 * x * (4.0f * zz - xx - yy), s(13), v);
        v = fmaf(SH_C3_5 * z * (xx - yy), s(14), v);
        v = fmaf(SH_C3_6 * x * (xx - 3.0f * yy), s(15), v);
      }
    }
  }
  return v;
}

// Input layouts (dsr_preprocess_* `layout` bits). bit 0: SH channel-major [S,G,3,M] (the
// decoder's Gaussians.harmonics) instead of the rasterizer's coefficient-major [S,G,M,3];
// bit 1: full covariance [S,G,3,3] instead of cov6 — the upper triangle is read, exactly
// what cuda_splatting.py:114,122's triu gather hands the rasterizer.
constexpr int kLayoutShChannelMajor = DSR_LAYOUT_SH_CHANNEL_MAJOR, kLayoutCovFull = DSR_LAYOUT_COV_FULL,
              kLayoutCountsZeroed = DSR_LAYOUT_COUNTS_ZEROED, kLayoutRectBinning = DSR_LAYOUT_RECT_BINNING,
              kLayoutExactBinning = DSR_LAYOUT_EXACT_BINNING, kLayoutDeferGeom = DSR_LAYOUT_DEFER_GEOM;
__device__ __forceinline__ float load_cov(const float* cov, size_t sg, int k, int layout) {
  if (layout & kLayoutCovFull) {
    constexpr int idx[6] = {0, 1, 2, 4, 5, 8};
    return cov[9 * sg + idx[k]];
  }
  return cov[6 * sg + k];
}
template <int NC>
__device__ __forceinline__ void load_sh(const float* shs, size_t sg, int M, int layout, float* out) {
  const float* p = shs + sg * (size_t)M * 3;
  if (layout & kLayoutShChannelMajor) {
#pragma unroll
    for (int k = 0; k < NC; ++k)
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) out[k * 3 + ch] = p[ch * M + k];
  } else {
#pragma unroll
    for (int k = 0; k < NC * 3; ++k) out[k] = p[k];
  }
}

// Segment (view, tile) bounds in the key buffer. stride == 0: prefix layout, segment s is
// [start[s], start[s + 1]). stride > 0: fixed capacity, [s * stride, s * stride + count[s]).
// stride == DSR_SEG_ENDS: [start[s], count[s]) — count holds absolute end offsets (the
// depth-cut binning writes only the near part of each prefix-layout segment).
constexpr uint32_t kSegEnds = DSR_SEG_ENDS;
__device__ __forceinline__ void seg_bounds(const uint32_t* __restrict__ start, const uint32_t* __restrict__ count,
                                           uint32_t stride, int seg, uint32_t& b, uint32_t& e) {
  if (stride == kSegEnds) {
    b = start[seg];
    e = count[seg];
  } else if (stride) {
    b = (uint32_t)seg * stride;
    e = b + count[seg];
  } else {
    b = start[seg];
    e = start[seg + 1];
  }
}

template <typename Real>
__device__ void inv4(const Real* m, Real* o) {  // row-major 4x4 inverse (cofactors)
  Real inv[16];
  inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
  inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
  inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
  inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
  inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
  inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
  inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
  inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
  inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
  inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
  inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
  inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
  inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
  inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
  inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
  inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
  const Real rdet = Real(1) / (m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12]);
  for (int i = 0; i < 16; ++i) o[i] = inv[i] * rdet;
}

template <typename Real>
__device__ void inv3(const Real* k, Real* o) {
  const Real a = k[0], b = k[1], c = k[2], d = k[3], e = k[4], f = k[5], g = k[6], h = k[7], i = k[8];
  const Real A = e * i - f * h, B = -(d * i - f * g), C = d * h - e * g;
  const Real r = Real(1) / (a * A + b * B + c * C);
  o[0] = A * r; o[1] = -(b * i - c * h) * r; o[2] = (b * f - c * e) * r;
  o[3] = B * r; o[4] = (a * i - c * g) * r; o[5] = -(a * f - c * d) * r;
  o[6] = C * r; o[7] = -(a * h - b * g) * r; o[8] = (a * e - b * d) * r;
}

// tan(fov / 2) for the angle between the rays through two image-edge midpoints (get_fov,
// projection.py:233-247, takes acos of their normalised dot product; the reference then takes
// tan of half of it): tan(t / 2) = |u x w| / (|u| |w| + u . w), no transcendental calls.
template <typename Real>
__device__ Real edge_tan_half(const Real* ki, Real x0, Real y0, Real x1, Real y1) {
  Real u[3], w[3];
  for (int r = 0; r < 3; ++r) {
    u[r] = ki[3 * r] * x0 + ki[3 * r + 1] * y0 + ki[3 * r + 2];
    w[r] = ki[3 * r] * x1 + ki[3 * r + 1] * y1 + ki[3 * r + 2];
  }
  const Real nu = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
  const Real nw = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const Real cx = u[1] * w[2] - u[2] * w[1], cy = u[2] * w[0] - u[0] * w[2], cz = u[0] * w[1] - u[1] * w[0];
  return sqrt(cx * cx + cy * cy + cz * cz) / (nu * nw + (u[0] * w[0] + u[1] * w[1] + u[2] * w[2]));
}

// One camera of dsr_build_cameras: the render_cuda set-up (cuda_splatting.py:62-86):
// scale-invariant rescale, K^-1 and tan(fov / 2) (get_fov), projection matrix, world->camera
// inverse, and their transposed (column-major) storage. Real = double in dsr_build_cameras;
// float where every workgroup of the binning kernel sets its camera up (the reference computes
// all of this in float32 torch; the two agree to ~1e-7 relative).
template <typename Real>
__device__ void make_camera(int v, const float* __restrict__ ext, const float* __restrict__ intr,
                            const float* __restrict__ near, const float* __restrict__ far,
                            const float* __restrict__ bg, const int32_t* __restrict__ view_scene,
                            int scale_invariant, dsr_camera& c) {
  Real E[16], K[9], Ki[9], Wc[16];
  for (int i = 0; i < 16; ++i) E[i] = ext[16 * v + i];
  for (int i = 0; i < 9; ++i) K[i] = intr[9 * v + i];
  Real n = near[v], f = far[v];
  float sc = 1.f;
  if (scale_invariant) {
    sc = 1.0f / near[v];  // float, as the reference's `scale = 1 / near`
    for (int r = 0; r < 3; ++r) E[4 * r + 3] *= (Real)sc;
    n *= (Real)sc;
    f *= (Real)sc;
  }
  inv3(K, Ki);
  const Real tx = edge_tan_half<Real>(Ki, 0, 0.5, 1, 0.5);
  const Real ty = edge_tan_half<Real>(Ki, 0.5, 0, 0.5, 1);
  // P (row-major) = get_projection_matrix
  Real P[16] = {0};
  const Real top = ty * n, right = tx * n;
  P[0] = 2 * n / (2 * right);
  P[5] = 2 * n / (2 * top);
  P[14] = 1;  // [3][2]
  P[10] = f / (f - n);
  P[11] = -(f * n) / (f - n);
  inv4(E, Wc);  // world -> camera, row-major
  // viewmatrix storage = (W2C)^T row-major  -> element [r*4 + c] = Wc[c*4 + r]
  for (int r = 0; r < 4; ++r)
    for (int q = 0; q < 4; ++q) c.viewmatrix[r * 4 + q] = (float)Wc[q * 4 + r];
  // projmatrix storage = (P W2C)^T
  for (int r = 0; r < 4; ++r)
    for (int q = 0; q < 4; ++q) {
      Real s = 0;
      for (int k = 0; k < 4; ++k) s += P[r * 4 + k] * Wc[k * 4 + q];
      c.projmatrix[q * 4 + r] = (float)s;
    }
  c.campos[0] = (float)E[3];
  c.campos[1] = (float)E[7];
  c.campos[2] = (float)E[11];
  c.tanfovx = (float)tx;
  c.tanfovy = (float)ty;
  c.bg[0] = bg[3 * v];
  c.bg[1] = bg[3 * v + 1];
  c.bg[2] = bg[3 * v + 2];
  c.scene = view_scene[v];
  c.scale = sc;
  c._pad[0] = 0;
  c._pad[1] = 0;
}

// render_cuda camera inputs for the in-kernel camera set-up (dsr_project_bin_cameras)
struct CamIn {
  const float *ext, *intr, *near, *far, *bg;
  const int32_t* view_scene;
  int scale_invariant;
};

// make_camera in float, spread over one wave so that no lane holds more than a few values
// (a one-lane set-up inside the binning kernel raised its VGPR count 60 -> 178 and cut its
// occupancy from 8 to 2 waves/SIMD). Lane i < 16 owns E[i] and the cofactor (r, c) = (i / 4,
// i % 4) of the 4x4 inverse; lanes 16..24 own K and the cofactors of the 3x3 inverse. Values
// move between lanes with ds_bpermute (__shfl), which every lane of the wave executes.
// focal (optional): (W / (2 tanfovx), H / (2 tanfovy)) of the camera, the projection's two
// per-camera divisions done once here instead of by every lane of every workgroup.
__device__ void make_camera_wave(int v, const CamIn& ci, int lane, dsr_camera& c, int H = 0, int W = 0,
                                 float2* focal = nullptr) {
  const float sc = ci.scale_invariant ? 1.0f / ci.near[v] : 1.0f;
  float x = 0.f;
  if (lane < 16) {
    x = ci.ext[16 * v + lane];
    if (ci.scale_invariant && (lane & 3) == 3 && lane < 12) x *= sc;
  } else if (lane < 25) {
    x = ci.intr[9 * v + lane - 16];
  }
  // cofactor of the element this lane owns, transposed (adjugate entry); 4x4 on lanes 0..15,
  // 3x3 on lanes 16..24
  float adj = 0.f;
  {
    const bool big = lane < 16;
    const int j = big ? lane : (lane < 25 ? lane - 16 : 0);
    const int N = big ? 4 : 3, base = big ? 0 : 16;
    const int r = j / N, col = j % N;  // adj[r][col] = (-1)^(r+col) * minor(row col, col r)
    // minor rows skip row `col`, minor columns skip column `r`
    auto at = [&](int a, int b) { return __shfl(x, base + (a + (a >= col)) * N + (b + (b >= r))); };
    float d;
    if (big) {
      const float m00 = at(0, 0), m01 = at(0, 1), m02 = at(0, 2);
      const float m10 = at(1, 0), m11 = at(1, 1), m12 = at(1, 2);
      const float m20 = at(2, 0), m21 = at(2, 1), m22 = at(2, 2);
      d = m00 * (m11 * m22 - m12 * m21) - m01 * (m10 * m22 - m12 * m20) + m02 * (m10 * m21 - m11 * m20);
    } else {
      const float m00 = at(0, 0), m01 = at(0, 1);
      const float m10 = at(1, 0), m11 = at(1, 1);
      d = m00 * m11 - m01 * m10;
    }
    adj = ((r + col) & 1) ? -d : d;
  }
  // determinants: row 0 of the matrix times column 0 of the adjugate
  const float det4 = __shfl(x, 0) * __shfl(adj, 0) + __shfl(x, 1) * __shfl(adj, 4) +
                     __shfl(x, 2) * __shfl(adj, 8) + __shfl(x, 3) * __shfl(adj, 12);
  const float det3 = __shfl(x, 16) * __shfl(adj, 16) + __shfl(x, 17) * __shfl(adj, 19) +
                     __shfl(x, 18) * __shfl(adj, 22);
  const float inv = adj * (1.0f / (lane < 16 ? det4 : det3));  // Wc on 0..15, K^-1 on 16..24
  float ki[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) ki[k] = __shfl(inv, 16 + k);
  const float tx = edge_tan_half<float>(ki, 0.f, 0.5f, 1.f, 0.5f);
  const float ty = edge_tan_half<float>(ki, 0.5f, 0.f, 0.5f, 1.f);
  const float n = ci.near[v] * sc, f = ci.far[v] * sc;
  const float top = ty * n, right = tx * n;
  // projmatrix storage = (P W2C)^T: lane o = q*4 + r holds (P W2C)[r][q]; P row r from
  // get_projection_matrix (only its non-zero terms)
  const int o = lane & 15, q = o >> 2, r = o & 3;
  const float w0 = __shfl(inv, q), w1 = __shfl(inv, 4 + q), w2 = __shfl(inv, 8 + q), w3 = __shfl(inv, 12 + q);
  float pm;
  if (r == 0) pm = (2 * n / (2 * right)) * w0;
  else if (r == 1) pm = (2 * n / (2 * top)) * w1;
  else if (r == 2) pm = (f / (f - n)) * w2 + (-(f * n) / (f - n)) * w3;
  else pm = w2;
  const float vm = __shfl(inv, (o & 3) * 4 + (o >> 2));  // viewmatrix storage = W2C^T
  const float cx = __shfl(x, 3), cy = __shfl(x, 7), cz = __shfl(x, 11);
  if (lane < 16) {
    c.viewmatrix[lane] = vm;
    c.projmatrix[lane] = pm;
  }
  if (lane == 0) {
    c.campos[0] = cx;
    c.campos[1] = cy;
    c.campos[2] = cz;
    c.tanfovx = tx;
    c.tanfovy = ty;
    c.bg[0] = ci.bg[3 * v];
    c.bg[1] = ci.bg[3 * v + 1];
    c.bg[2] = ci.bg[3 * v + 2];
    c.scene = ci.view_scene[v];
    c.scale = sc;
    c._pad[0] = 0;
    c._pad[1] = 0;
    if (focal) *focal = make_float2(W / (2.0f * tx), H / (2.0f * ty));
  }
}

// ------------------------------------------------------------------------------------
// K1 building blocks: one Gaussian's scene inputs (loaded once) and its projection into one
// view (upstream preprocessCUDA, rows A7 of the survey).
template <int DEG>
struct GaussIn {
  static constexpr int NC = DEG >= 0 ? (DEG + 1) * (DEG + 1) : 1;
  float m[3];
  float c6[6];
  float op;
  size_t sg;  // scene-Gaussian index: SH / colours are read only once the Gaussian survives culling
};

template <int DEG>
__device__ __forceinline__ void load_gauss(GaussIn<DEG>& in, size_t sg, const float* __restrict__ means,
                                           const float* __restrict__ opac, const float* __restrict__ cov6,
                                           int layout) {
#pragma unroll
  for (int k = 0; k < 3; ++k) in.m[k] = means[3 * sg + k];
#pragma unroll
  for (int k = 0; k < 6; ++k) in.c6[k] = load_cov(cov6, sg, k, layout);
  in.op = opac[sg];
  in.sg = sg;
}

// The camera's focal lengths in pixels (cuda_splatting's rasterizer: W / (2 tan(fovx / 2))).
__device__ __forceinline__ float2 focal_of(const dsr_camera* cam, int H, int W) {
  return make_float2(W / (2.0f * cam->tanfovx), H / (2.0f * cam->tanfovy));
}
// Fills rec (GS floats, zero when culled) and the tile rect; returns the radius (0 = culled).
// focal = focal_of(cam, H, W) (precomputed once per camera where the kernel has it).
// COLOR = false: the geometry only (rec[6..8] and the clamp bits stay zero, no SH read).
template <int DEG, bool COLOR = true>
__device__ __forceinline__ int project_gauss(const GaussIn<DEG>& in, const dsr_camera* __restrict__ cam, float2 focal,
                                             int H, int W, int gx, int gy, int M, const float* __restrict__ shs,
                                             const float* __restrict__ colors, int layout, float* rec, int& x0,
                                             int& y0, int& x1, int& y1) {
  int r = 0;
#pragma unroll
  for (int k = 0; k < GS; ++k) rec[k] = 0.f;
  x0 = y0 = x1 = y1 = 0;
  const float gsc = cam->scale;
  const F3 p = {in.m[0] * gsc, in.m[1] * gsc, in.m[2] * gsc};
  const float* view = cam->viewmatrix;
  const float* proj = cam->projmatrix;
  const F3 pv = xform43(view, p);
  if (pv.z > 0.2f) {
    const F3 ph = xform43(proj, p);
    const float pw = 1.0f / (xform44w(proj, p) + 0.0000001f);
    const float ndx = ph.x * pw, ndy = ph.y * pw;
    float c6[6];
    const float gsc2 = gsc * gsc;
#pragma unroll
    for (int k = 0; k < 6; ++k) c6[k] = in.c6[k] * gsc2;
    Cov2D w;
    cov2d(p, focal.x, focal.y, cam->tanfovx, cam->tanfovy, c6, view, w);
    const float det = fmaf(w.a, w.c, -(w.b * w.b));
    if (det != 0.0f) {
      const float det_inv = 1.f / det;
      const float mid = 0.5f * (w.a + w.c);
      const float disc = sqrtf(fmaxf(0.1f, fmaf(mid, mid, -det)));
      const float l1 = mid + disc, l2 = mid - disc;
      const int rr = (int)ceilf(3.f * sqrtf(fmaxf(l1, l2)));
      const float px = ndc2pix(ndx, W), py = ndc2pix(ndy, H);
      tile_rect(px, py, rr, gx, gy, x0, y0, x1, y1);
      if ((x1 - x0) * (y1 - y0) != 0) {
        r = rr;
        uint32_t clamp_bits = 0;
        if constexpr (!COLOR) {
        } else if constexpr (DEG >= 0) {
          float sh[GaussIn<DEG>::NC * 3];
          load_sh<GaussIn<DEG>::NC>(shs, in.sg, M, layout, sh);
          float dx = p.x - cam->campos[0], dy = p.y - cam->campos[1], dz = p.z - cam->campos[2];
          const float len = sqrtf(fmaf(dx, dx, fmaf(dy, dy, dz * dz)));
          dx = dx / len;
          dy = dy / len;
          dz = dz / len;
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) {
            float c = sh_eval<DEG>(sh, ch, dx, dy, dz) + 0.5f;
            clamp_bits |= (c < 0.f ? 1u : 0u) << ch;
            rec[6 + ch] = fmaxf(c, 0.0f);
          }
        } else {
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) rec[6 + ch] = colors[3 * in.sg + ch];
        }
        rec[0] = px;
        rec[1] = py;
        rec[2] = w.c * det_inv;
        rec[3] = -w.b * det_inv;
        rec[4] = w.a * det_inv;
        rec[5] = in.op;
        rec[9] = pv.z;
        rec[10] = __int_as_float(r);
        rec[11] = __uint_as_float(clamp_bits);
      } else {
        x0 = y0 = x1 = y1 = 0;
      }
    }
  }
  return r;
}

// dzero (optional): the backward's fixed-point gradient accumulator [V, G, DSR_DGEOM_WORDS];
// the row of every rendered (view, Gaussian) is zeroed here, in the kernel that writes its
// record anyway (no separate HBM fill pass; culled rows are never read by the backward).
__device__ __forceinline__ void store_geom(float* __restrict__ geom, int32_t* __restrict__ radii, size_t vg,
                                           const float* rec, int r, long long* __restrict__ dzero) {
  float4* out = reinterpret_cast<float4*>(geom + vg * GS);
  out[0] = make_float4(rec[0], rec[1], rec[2], rec[3]);
  out[1] = make_float4(rec[4], rec[5], rec[6], rec[7]);
  out[2] = make_float4(rec[8], rec[9], rec[10], rec[11]);
  radii[vg] = r;
  if (dzero != nullptr && r > 0) {
    long long* z = dzero + vg * DSR_DGEOM_WORDS;
#pragma unroll
    for (int k = 0; k < DSR_DGEOM_WORDS; ++k) z[k] = 0ll;
  }
}

// Exact tile test of the inference binning (k_project_emit EXACT): can the alpha >= 1/255 ellipse of a
// Gaussian reach a pixel centre of the tile box [x0, x0 + BX - 1] x [y0, y0 + BY - 1]? The
// same continuous-box minimum of the conic as the compositor's rect_hit (defined with it
// below), with the per-Gaussian terms computed once by the owner lane (TileEll) and moved to
// the pair's lane by ds_bpermute. A tile it rejects is one where the compositor's per-pixel
// test fails at every pixel, so dropping the pair leaves every blend unchanged.
struct TileEll {
  float x, y, a, b, c, t2, ia, ic;  // t2 < 0: opacity below 1/255 (reaches nothing)
};
__device__ __forceinline__ TileEll tile_ell(const float* rec, int r) {
  TileEll e;
  e.x = rec[0];
  e.y = rec[1];
  e.a = rec[2];
  e.b = rec[3];
  e.c = rec[4];
  const float op = rec[5];
  e.t2 = (r > 0 && op >= 1.0f / 255.0f) ? 2.0f * __logf(255.0f * op) * 1.002f + 0.02f : -1.0f;
  e.ia = __builtin_amdgcn_rcpf(e.a);  // edge minimiser only (see rect_hit)
  e.ic = __builtin_amdgcn_rcpf(e.c);
  return e;
}
__device__ __forceinline__ TileEll tile_ell_of(const TileEll& e, int o) {
  return TileEll{__shfl(e.x, o), __shfl(e.y, o), __shfl(e.a, o), __shfl(e.b, o),
                 __shfl(e.c, o), __shfl(e.t2, o), __shfl(e.ia, o), __shfl(e.ic, o)};
}
__device__ __forceinline__ bool tile_reach(const TileEll& e, int tx, int ty) {
  if (!(e.t2 >= 0.f)) return false;
  const float a = e.a, b = e.b, c = e.c;
  if (!(a > 0.f && c > 0.f && a * c - b * b > 0.f)) return true;  // degenerate / NaN: keep
  const float lx = (float)(tx * BX) - e.x, hx = lx + (float)(BX - 1);
  const float ly = (float)(ty * BY) - e.y, hy = ly + (float)(BY - 1);
  if (lx <= 0.f && hx >= 0.f && ly <= 0.f && hy >= 0.f) return true;
  float m = 3.4e38f;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float dx = k ? hx : lx;
    const float dy = fminf(fmaxf(-b * dx * e.ic, ly), hy);
    m = fminf(m, a * dx * dx + 2.f * b * dx * dy + c * dy * dy);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float dy = k ? hy : ly;
    const float dx = fminf(fmaxf(-b * dy * e.ia, lx), hx);
    m = fminf(m, a * dx * dx + 2.f * b * dx * dy + c * dy * dy);
  }
  return !(m > e.t2);
}
// Tile rect of the alpha >= 1/255 ellipse's bounding box (half extents sqrt(t2 c / det),
// sqrt(t2 a / det), padded), intersected with the 3-sigma rect [x0, x1) x [y0, y1): fewer
// pairs to expand before tile_reach. Degenerate / NaN conics keep the 3-sigma rect.
__device__ __forceinline__ void tile_rect_alpha(const TileEll& e, int& x0, int& y0, int& x1, int& y1) {
  if (!(e.t2 >= 0.f)) {
    x1 = x0;
    y1 = y0;
    return;
  }
  // only a candidate box for tile_reach (which decides): hardware reciprocal and square root
  // (1 ulp each) sit far inside the 1.002 / +0.05 margin, and count, emission and the
  // bounded-capacity rebuild all evaluate this same function
  const float det = e.a * e.c - e.b * e.b;
  const float rdet = __builtin_amdgcn_rcpf(det);
  const float hx = __builtin_amdgcn_sqrtf(e.t2 * e.c * rdet) * 1.002f + 0.05f;
  const float hy = __builtin_amdgcn_sqrtf(e.t2 * e.a * rdet) * 1.002f + 0.05f;
  if (!(e.a > 0.f && e.c > 0.f && det > 0.f) || !(hx == hx) || !(hy == hy)) return;
  const float lim = 65536.f;
  x0 = max(x0, (int)floorf(fminf(fmaxf((e.x - hx) * (1.0f / BX), -1.f), lim)));
  x1 = min(x1, (int)floorf(fminf(fmaxf((e.x + hx) * (1.0f / BX), -1.f), lim)) + 1);
  y0 = max(y0, (int)floorf(fminf(fmaxf((e.y - hy) * (1.0f / BY), -1.f), lim)));
  y1 = min(y1, (int)floorf(fminf(fmaxf((e.y + hy) * (1.0f / BY), -1.f), lim)) + 1);
  if (x1 <= x0 || y1 <= y0) {
    x1 = x0;
    y1 = y0;
  }
}

// K1: preprocess + per-(view, tile) entry counts (two-phase binning path).
// grid = (ceil(G/256), V), block = 256. DEG = -1 -> colors_precomp path.
template <int DEG, bool EXACT>
__global__ __launch_bounds__(NT) void k_preprocess(int G, int V, int H, int W, int gx, int gy, int M,
                                                   const float* __restrict__ means,
                                                   const float* __restrict__ shs,
                                                   const float* __restrict__ colors,
                                                   const float* __restrict__ opac,
                                                   const float* __restrict__ cov6,
                                                   const dsr_camera* __restrict__ cams,
                                                   float* __restrict__ geom, int32_t* __restrict__ radii,
                                                   long long* __restrict__ dzero,
                                                   uint32_t* __restrict__ seg_count, int lds_hist, int layout) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];
  int v, blk;
  if (!xcd_pair((G + NT - 1) / NT, V, blk, v)) return;
  const int T = gx * gy;
  const int tid = threadIdx.x;
  const dsr_camera* cam = cams + v;
  if (lds_hist) {
    for (int t = tid; t < T; t += NT) s_hist[t] = 0;
    __syncthreads();
  }
  const int g = blk * NT + tid;
  int r = 0, x0 = 0, y0 = 0, x1 = 0, y1 = 0;
  TileEll ell{0.f, 0.f, 0.f, 0.f, 0.f, -1.f, 0.f, 0.f};
  if (g < G) {
    GaussIn<DEG> in;
    load_gauss<DEG>(in, (size_t)cam->scene * G + g, means, opac, cov6, layout);
    float rec[GS];
    r = project_gauss<DEG>(in, cam, focal_of(cam, H, W), H, W, gx, gy, M, shs, colors, layout, rec, x0, y0, x1,
                           y1);
    store_geom(geom, radii, (size_t)v * G + g, rec, r, dzero);
    if constexpr (EXACT) {  // same terms as k_scatter<true> recomputes from the stored record
      ell = tile_ell(rec, r);
      if (r > 0) tile_rect_alpha(ell, x0, y0, x1, y1);
    }
  }
  uint32_t* gcount = seg_count + (size_t)v * T;
  __shared__ WaveRects s_wr[NT / 64];
  const int lane = tid & 63;
  uint32_t* hist = lds_hist ? s_hist : gcount;
  TileEll oe = ell;
  for_each_rect_tile(s_wr[tid >> 6], lane, x0, y0, x1, y1, r > 0, gx, [&](int t, int, int tx, int ty) {
    if constexpr (EXACT) {
      if (!tile_reach(oe, tx, ty)) return;
    }
    atomicAdd(&hist[t], 1u);
  }, [&](int o) {
    if constexpr (EXACT) oe = tile_ell_of(ell, o);
  });
  if (lds_hist) {
    __syncthreads();
    for (int t = tid; t < T; t += NT) {
      const uint32_t c = s_hist[t];
      if (c) atomicAdd(&gcount[t], c);
    }
  }
}

// ------------------------------------------------------------------------------------
// K1+K3 fused (fixed-capacity binning): one workgroup per (256 Gaussians, view) projects
// them, counts the block's (view, tile) entries in an LDS histogram, reserves a contiguous
// range per touched tile with one global atomic, and writes the (depth, id) keys into
// segment (v, t), which starts at (v*T + t) * G (a Gaussian touches a tile at most once, so
// G slots suffice). No global scan is needed before the keys exist. The V workgroups of one
// Gaussian block run back to back on one XCD (xcd_pair), so the scene's 148 B per
// Gaussian come from HBM once and from that XCD's L2 for the other views (one workgroup per
// scene looping over its views would hold 3x fewer waves in flight to hide the load and
// atomic latencies).
// (70 VGPRs: 7 waves per SIMD; forcing 8 spills 860 B per lane and runs 6-8x slower)
constexpr int kProjectWPE = 1;
// pair cache of the count pass (kPairCapW (tile, rank, owner) words per wave in LDS)
constexpr int kPairCapW = 768;
// EXACT: a pair is kept only when tile_reach says the alpha >= 1/255 ellipse reaches the tile
// (the inference path by default, the stateful path with DSR_LAYOUT_EXACT_BINNING); else the
// reference's 3-sigma rect lists, which the oracle list tests follow.
template <int DEG, bool CAM, bool EXACT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(kProjectWPE))) void k_project_emit(int G, int V, int H, int W, int gx, int gy, int M,
                                                     const float* __restrict__ means,
                                                     const float* __restrict__ shs,
                                                     const float* __restrict__ colors,
                                                     const float* __restrict__ opac,
                                                     const float* __restrict__ cov6,
                                                     dsr_camera* __restrict__ cams,
                                                     float* __restrict__ geom, int32_t* __restrict__ radii,
                                                     long long* __restrict__ dzero,
                                                     uint32_t* __restrict__ seg_count,
                                                     uint64_t* __restrict__ keys, uint32_t cap, int layout,
                                                     CamIn ci) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];
  __shared__ WaveRects s_wr[NT / 64];
  __shared__ uint64_t s_key[NT];
  __shared__ dsr_camera s_cam[1];  // CAM only
  __shared__ float2 s_focal;       // CAM only
  __shared__ uint32_t s_pairs[NT / 64][kPairCapW];
  __shared__ uint32_t s_ovf;
  int v, blk;
  // DSR_LAYOUT_VIEWS_PER_SCENE (scene-major XCD placement; same-box A/B at 16 scenes: -2 %)
  if (!xcd_scene_major((G + NT - 1) / NT, V, (layout >> 16) & 0xFF, blk, v)) return;
  const dsr_camera* cam = cams + v;
  const int T = gx * gy;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = blk * NT + tid;
  WaveRects& wr = s_wr[w];
  const uint64_t* wkey = s_key + w * 64;
  for (int t = tid; t < T; t += NT) s_hist[t] = 0;
  int r = 0, x0 = 0, y0 = 0, x1 = 0, y1 = 0;
  uint64_t key = 0;
  TileEll ell{0.f, 0.f, 0.f, 0.f, 0.f, -1.f, 0.f, 0.f};
  GaussIn<DEG> in;
  if (g < G) load_gauss<DEG>(in, (size_t)(CAM ? ci.view_scene[v] : cam->scene) * G + g, means, opac, cov6, layout);
  if constexpr (CAM) {
    // every workgroup sets up its view's camera while its Gaussians load (no separate
    // launch); the first block of each view also stores it for the later kernels
    if (w == 0) make_camera_wave(v, ci, lane, s_cam[0], H, W, &s_focal);
    __syncthreads();
    if (blk == 0 && tid < (int)(sizeof(dsr_camera) / 4))
      reinterpret_cast<uint32_t*>(cams + v)[tid] = reinterpret_cast<const uint32_t*>(s_cam)[tid];
    cam = s_cam;
  }
  if (g < G) {
    float rec[GS];
    r = project_gauss<DEG>(in, cam, CAM ? s_focal : focal_of(cam, H, W), H, W, gx, gy, M, shs, colors, layout, rec,
                           x0, y0, x1, y1);
    store_geom(geom, radii, (size_t)v * G + g, rec, r, dzero);
    key = ((uint64_t)__float_as_uint(rec[9]) << 32) | (uint32_t)g;
    if constexpr (EXACT) {
      ell = tile_ell(rec, r);
      if (r > 0) tile_rect_alpha(ell, x0, y0, x1, y1);
    }
  }
  s_key[tid] = key;
  if (tid == 0) s_ovf = 0u;
  __syncthreads();
  TileEll oe = ell;  // the owner's ellipse terms for the current pair (EXACT)
  const auto fetch = [&](int o) {
    if constexpr (EXACT) oe = tile_ell_of(ell, o);
  };
  // count pass; each pair's rank among the workgroup's entries of its tile (the LDS atomic's
  // return value) is kept with the tile and the owner lane, so the emission pass below is a
  // plain walk over the kept pairs instead of a second rect expansion
  uint32_t* wp = s_pairs[w];
  uint32_t stp = 0;
  const uint32_t wtotal = for_each_rect_tile(wr, lane, x0, y0, x1, y1, r > 0, gx, [&](int t, int o, int tx, int ty) {
    const uint32_t j = stp++ * 64u + (uint32_t)lane;
    if constexpr (EXACT) {
      if (!tile_reach(oe, tx, ty)) {  // dropped pair: a hole in the list
        if (j < (uint32_t)kPairCapW) wp[j] = 0xFFFFFFFFu;
        return;
      }
    }
    const uint32_t rk = atomicAdd(&s_hist[t], 1u);
    if (j < (uint32_t)kPairCapW) wp[j] = (uint32_t)t | (rk << 16) | ((uint32_t)o << 24);
  }, fetch);
  if (lane == 0 && wtotal > (uint32_t)kPairCapW) s_ovf = 1u;
  __syncthreads();
  uint32_t* gcount = seg_count + (size_t)v * T;
  for (int t = tid; t < T; t += NT) {
    const uint32_t c = s_hist[t];
    if (c) s_hist[t] = atomicAdd(&gcount[t], c);
  }
  __syncthreads();
  // segment (v, t) = keys[(v T + t) cap ...]: cap = G holds every entry a tile can get; a
  // smaller capacity (bounded key memory) keeps the first cap arrivals, the count goes on,
  // and dsr_sort_render rebuilds such a segment from the geometry records
  uint64_t* vkeys = keys + (size_t)v * T * cap;
  if (!s_ovf) {  // workgroup-uniform
    for (uint32_t j = (uint32_t)lane; j < wtotal; j += 64u) {
      const uint32_t p = wp[j];
      if (EXACT && p == 0xFFFFFFFFu) continue;
      const uint32_t t = p & 0xFFFFu;
      const uint32_t off = s_hist[t] + ((p >> 16) & 0xFFu);
      if (off < cap) vkeys[(size_t)t * cap + off] = wkey[p >> 24];
    }
    return;
  }
  // a wave of this workgroup had more than kPairCapW pairs: re-expand the rects. The keep test
  // is the same inlined code on the same operands (oe from the same owner lane, same tile
  // coordinates) as in the count pass, so both passes keep exactly the same pairs and the
  // emission fills the ranges reserved above (tests: test_inference_emit_overflow).
  for_each_rect_tile(wr, lane, x0, y0, x1, y1, r > 0, gx, [&](int t, int o, int tx, int ty) {
    if constexpr (EXACT) {
      if (!tile_reach(oe, tx, ty)) return;
    }
    const uint32_t off = atomicAdd(&s_hist[t], 1u);
    if (off < cap) vkeys[(size_t)t * cap + off] = wkey[o];
  }, fetch);
}

// ------------------------------------------------------------------------------------
// Single-workgroup exclusive scan of the per-(view, tile) counts (V*T is small: 768 at
// 2x256^2 x 3 views, ~20K at 12x512x960 x 10 views). Each thread scans 16 consecutive counts
// (their loads issued together), so 16K counts take ONE pass of 3 barriers: round 5 walked
// 1024 per pass (config D's 10,752 counts: 11 dependent passes, ~20 us).
__global__ __launch_bounds__(1024) void k_scan(int n, const uint32_t* __restrict__ cnt,
                                               uint32_t* __restrict__ start,
                                               uint32_t* __restrict__ cursor,
                                               uint32_t* __restrict__ totals) {
  constexpr int PT = 16;
  __shared__ uint32_t s_w[16];
  __shared__ uint32_t s_max[16];
  __shared__ uint32_t s_carry, s_big;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) {
    s_carry = 0;
    s_big = 0;
  }
  __syncthreads();
  uint32_t my_max = 0;
  for (int base = 0; base < n; base += 1024 * PT) {
    uint32_t x[PT], tot = 0;
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int k = base + tid * PT + i;
      x[i] = k < n ? cnt[k] : 0u;
    }
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      tot += x[i];
      my_max = max(my_max, x[i]);
    }
    const uint32_t incl = dsplat::wave_incl_scan(tot, lane);
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    uint64_t chunk = 0;
    uint32_t off = s_carry + incl - tot;
    for (int k = 0; k < 16; ++k) {
      if (k < w) off += s_w[k];
      chunk += s_w[k];
    }
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int k = base + tid * PT + i;
      if (k < n) {
        start[k] = off;
        cursor[k] = off;
      }
      off += x[i];
    }
    __syncthreads();  // every thread has read s_carry / s_w
    if (tid == 0) {
      const uint64_t c = (uint64_t)s_carry + chunk;
      if (c >> 31) s_big = 1u;  // offsets past 2^31: the caller must split the batch
      s_carry = (uint32_t)c;
    }
    __syncthreads();
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) my_max = max(my_max, (uint32_t)__shfl_xor((int)my_max, off, 64));
  if (lane == 0) s_max[w] = my_max;
  __syncthreads();
  if (tid == 0) {
    uint32_t m = 0;
    for (int k = 0; k < 16; ++k) m = max(m, s_max[k]);
    start[n] = s_carry;
    totals[0] = s_carry;
    totals[1] = m;
    totals[2] = s_big;
  }
}

// ---- depth-cut binning (include/dsplat_hip.h: dsr_preprocess_cut / dsr_bin_cutoff /
// dsr_bin_scatter_cut). Depth bucket = 16 per octave of the view-space depth (in near units)
// from 0.25, read off the float bits; monotone in the depth, so a bucket range is a depth range.
constexpr int kCutBuckets = DSR_CUT_BUCKETS;
// count histogram + super-block depth histograms: 26 KiB, so that with k_preprocess_cut's 14 KiB
// of static LDS four 512-thread workgroups fit a CU (32 waves; its deferred-geometry instances
// use 60 VGPRs). Round 5: the budget was 96 KiB, which picked 4 x 4-tile super-blocks at
// 512 x 960 (69 KiB of histograms: ONE workgroup per CU, 8 waves, while the host sized the
// persistent grid for two); 8 x 8-tile super-blocks there took config E from 40.1 to 31.5 ms
// per scene and config D from 1.24 to 1.09 ms per step (same box, profiles/r05s_ab_cut_lds.log)
constexpr int kCutLdsWords = 6656;
constexpr int kCutLdsWordsMax = 24576;  // larger images: fewer resident workgroups, still a cut
constexpr int kCutMaxSB = kCutLdsWordsMax / kCutBuckets;
__device__ __forceinline__ int depth_bucket(uint32_t zbits) {
  return min(kCutBuckets - 1, max(0, (int)(zbits >> 19) - (125 << 4)));
}
__host__ __device__ inline int cut_superblock(int gx, int gy) {
  for (int sb = 4; sb <= 64; sb *= 2) {
    const int nsb = ((gx + sb - 1) / sb) * ((gy + sb - 1) / sb);
    if ((gx + 1) * (gy + 1) + nsb * kCutBuckets <= kCutLdsWords) return sb;
  }
  for (int sb = 4; sb <= 64; sb *= 2) {
    const int nsb = ((gx + sb - 1) / sb) * ((gy + sb - 1) / sb);
    if ((gx + 1) * (gy + 1) + nsb * kCutBuckets <= kCutLdsWordsMax) return sb;
  }
  return 0;
}

// K3: emit (depth, id) keys into their (view, tile) bucket. EXACT: keep the pairs
// k_preprocess<DEG, true> counted (same tile test on the stored record).
template <bool EXACT>
__global__ __launch_bounds__(NT) void k_scatter(int G, int V, int gx, int gy, const float* __restrict__ geom,
                                                uint32_t* __restrict__ cursor,
                                                uint64_t* __restrict__ keys, int lds_hist) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];
  int v, blk;
  if (!xcd_item((G + NT - 1) / NT, V, v, blk)) return;
  const int T = gx * gy;
  const int tid = threadIdx.x;
  if (lds_hist) {
    for (int t = tid; t < T; t += NT) s_hist[t] = 0;
    __syncthreads();
  }
  const int g = blk * NT + tid;
  int r = 0, x0 = 0, y0 = 0, x1 = 0, y1 = 0;
  uint64_t key = 0;
  TileEll ell{0.f, 0.f, 0.f, 0.f, 0.f, -1.f, 0.f, 0.f};
  if (g < G) {
    const float* rec = geom + ((size_t)v * G + g) * GS;
    r = __float_as_int(rec[10]);
    if (r > 0) {
      tile_rect(rec[0], rec[1], r, gx, gy, x0, y0, x1, y1);
      key = ((uint64_t)__float_as_uint(rec[9]) << 32) | (uint32_t)g;
      if constexpr (EXACT) {
        ell = tile_ell(rec, r);
        tile_rect_alpha(ell, x0, y0, x1, y1);
      }
    }
  }
  TileEll oe = ell;
  const auto fetch = [&](int o) {
    if constexpr (EXACT) oe = tile_ell_of(ell, o);
  };
  uint32_t* gcur = cursor + (size_t)v * T;
  __shared__ WaveRects s_wr[NT / 64];
  __shared__ uint64_t s_key[NT];
  const int lane = tid & 63, w = tid >> 6;
  s_key[tid] = key;
  WaveRects& wr = s_wr[w];
  const uint64_t* wkey = s_key + w * 64;
  const auto keep = [&](int tx, int ty) {
    if constexpr (EXACT) return tile_reach(oe, tx, ty);
    return true;
  };
  if (lds_hist) {
    for_each_rect_tile(wr, lane, x0, y0, x1, y1, r > 0, gx, [&](int t, int, int tx, int ty) {
      if (keep(tx, ty)) atomicAdd(&s_hist[t], 1u);
    }, fetch);
    __syncthreads();
    for (int t = tid; t < T; t += NT) {
      const uint32_t c = s_hist[t];
      if (c) s_hist[t] = atomicAdd(&gcur[t], c);
    }
    __syncthreads();
    for_each_rect_tile(wr, lane, x0, y0, x1, y1, r > 0, gx, [&](int t, int o, int tx, int ty) {
      if (keep(tx, ty)) keys[atomicAdd(&s_hist[t], 1u)] = wkey[o];
    }, fetch);
  } else {
    for_each_rect_tile(wr, lane, x0, y0, x1, y1, r > 0, gx, [&](int t, int o, int tx, int ty) {
      if (keep(tx, ty)) keys[atomicAdd(&gcur[t], 1u)] = wkey[o];
    }, fetch);
  }
}

// The depth-cut scatter's persistent grid: per_view workgroups of kScatterCutNTH threads per
// view, workgroup p taking blocks p, p + per_view, ... Its survivor list (deferred geometry) is
// its own slice of survivor_slice() entries with its own counter, so listing costs one LDS
// atomic per wave and no global atomic (a per-view global counter, hit once per wave by every
// workgroup of the view, serialised the scatter: 8x slower at 12x512x960).
constexpr int kScatterCutNTH = 256;
__host__ __device__ inline int scatter_cut_per_view(int G, int V) {
  return max(1, min((G + kScatterCutNTH - 1) / kScatterCutNTH, (256 * 8) / V));
}
__host__ __device__ inline size_t survivor_slice(int G, int V) {
  const int nblk = (G + kScatterCutNTH - 1) / kScatterCutNTH, pv = scatter_cut_per_view(G, V);
  return (size_t)((nblk + pv - 1) / pv) * kScatterCutNTH;
}

// K3 under the depth cut (dsr_bin_scatter_cut): only the entries the cut keeps (tail == 0:
// depth bits <= the threshold of the tile's super-block; tail == 1: the others, of flagged
// tiles only).
// Kept entries are few (~4-9 % at 6x448x768 and up), so there is no per-block LDS count /
// reservation round (whose zero + flush of T counters per 256 Gaussians dominated): each
// kept entry takes its slot with one global atomic on its segment cursor, and a persistent
// grid (one view and a run of blocks per workgroup, no workgroup barrier in the loop) walks
// the Gaussians. A whole-Gaussian pre-test over the super-blocks its rect touches skips the
// expansion of Gaussians no tile keeps (most of them) and clips the others' rects to the
// super-blocks that keep something.
template <int NTH>
__global__ __launch_bounds__(NTH) void k_scatter_cut(int G, int V, int gx, int gy, const float* __restrict__ geom,
                                                     uint32_t* __restrict__ cursor, uint64_t* __restrict__ keys,
                                                     const uint32_t* __restrict__ cut, int tail,
                                                     const uint32_t* __restrict__ seg_overflow,
                                                     const uint2* __restrict__ cut_rec, int per_view,
                                                     uint32_t* __restrict__ surv, uint32_t* __restrict__ surv_count,
                                                     const uint32_t* __restrict__ totals, uint64_t keys_cap) {
  constexpr int NW = NTH / 64;
  // launched before the host has read N (round 6): a key buffer smaller than N entries leaves
  // everything untouched (uniform early exit before any side effect) and the host re-runs the pass
  if (totals != nullptr && ((uint64_t)totals[0] > keys_cap || totals[2] != 0u)) return;  // (totals[2]: N >= 2^31)
  __shared__ uint32_t s_cut[kCutMaxSB];
  __shared__ WaveRects s_wr[NW];
  __shared__ uint64_t s_key[NTH];
  __shared__ uint32_t s_rx[NW][64], s_ry[NW][64];  // tile rect x0 | x1 << 16, y0 | y1 << 16
  __shared__ WaveRects s_wr2[NW];                   // inner expansion of the large rects
  __shared__ uint64_t s_k2[NW][64];
  const int T = gx * gy;
  if (tail && seg_overflow[(size_t)V * T] == 0u) return;  // no tile flagged (uniform)
  // one view's workgroups on one XCD (xcd_item): the 8-byte key stores to a tile's segment
  // frontier then merge in that XCD's L2 before write-back (spread over the 8 XCDs, each
  // frontier line came back as up to 8 partial writes: 3x the algorithmic bytes at config D)
  int v, p;
  if (!xcd_item(per_view, V, v, p)) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int sb = cut_superblock(gx, gy), sbl = __builtin_ctz((unsigned)sb);
  const int nsx = (gx + sb - 1) / sb, nsb = nsx * ((gy + sb - 1) / sb);
  const uint32_t* vov = seg_overflow ? seg_overflow + (size_t)v * T : nullptr;
  const uint32_t* sbov = seg_overflow ? seg_overflow + (size_t)V * T + 1 + (size_t)v * nsb : nullptr;
  // tail: the bounding box of the view's flagged super-blocks (a flagged tile is usually one
  // of a handful), so that the Gaussians whose rects miss it skip the per-super-block test
  __shared__ int s_fb[4];
  if (tail && tid == 0) {
    s_fb[0] = nsx;
    s_fb[1] = -1;
    s_fb[2] = nsb;
    s_fb[3] = -1;
  }
  if (tail) __syncthreads();
  for (int k = tid; k < nsb; k += NTH) {
    s_cut[k] = cut[(size_t)v * nsb + k];
    if (tail && sbov[k] != 0u) {
      const int sy = k / nsx, sx = k - sy * nsx;
      atomicMin(&s_fb[0], sx);
      atomicMax(&s_fb[1], sx);
      atomicMin(&s_fb[2], sy);
      atomicMax(&s_fb[3], sy);
    }
  }
  __syncthreads();
  const int fx0 = tail ? s_fb[0] : 0, fx1 = tail ? s_fb[1] : nsx, fy0 = tail ? s_fb[2] : 0, fy1 = tail ? s_fb[3] : nsb;
  if (fx1 < fx0) return;  // tail, nothing flagged in this view (workgroup-uniform; counters stay 0)
  __shared__ uint32_t s_nsurv;
  uint32_t* wsurv = surv ? surv + ((size_t)v * per_view + p) * survivor_slice(G, V) : nullptr;
  if (tid == 0) s_nsurv = 0u;
  __syncthreads();
  uint32_t* gcur = cursor + (size_t)v * T;
  const float* gv = geom + (size_t)v * G * GS;
  WaveRects& wr = s_wr[w];
  const uint64_t* wkey = s_key + w * 64;
  const int nblk = (G + NTH - 1) / NTH;
  // blocks dealt round-robin (p, p + per_view, ...): neighbouring blocks (context-image rows)
  // carry similar loads, so contiguous runs left some workgroups with several times the work
  // the next block's compact records are loaded one iteration ahead (software pipelining:
  // the loop is a chain of short dependent steps, each waiting on memory)
  const uint2* vrec = cut_rec ? cut_rec + (size_t)v * G : nullptr;
  uint2 cr_next = make_uint2(0u, 0u);
  if (vrec && p * NTH + tid < G) cr_next = vrec[p * NTH + tid];
  for (int blk = p; blk < nblk; blk += per_view) {
    const int g = blk * NTH + tid;
    const uint2 cr_cur = cr_next;
    if (vrec) {
      const int gn = (blk + per_view) * NTH + tid;
      cr_next = gn < G ? vrec[gn] : make_uint2(0u, 0u);
    }
    int r = 0, x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    int sx0 = 0, sx1 = 0, sy0 = 0, sy1 = 0;
    bool big = false;  // rect over more than 16 super-blocks: tested per (Gaussian, super-block) below
    uint64_t key = 0;
    if (g < G) {
      // whole-Gaussian pre-test over the super-blocks its rect touches, from the 8-byte compact
      // record when given (tile rect + depth: the 48-byte geometry record is never read, and
      // with deferred geometry it does not exist yet), else from the geometry record
      uint32_t zb = 0u;
      if (cut_rec) {
        const uint2 cr = cr_cur;
        x0 = (int)(cr.x & 0xFFu);
        x1 = (int)((cr.x >> 8) & 0xFFu);
        y0 = (int)((cr.x >> 16) & 0xFFu);
        y1 = (int)(cr.x >> 24);
        zb = cr.y;
        r = cr.x != 0u ? 1 : 0;
      } else {
        const float* rec = gv + (size_t)g * GS;
        r = __float_as_int(rec[10]);
        if (r > 0) {
          tile_rect(rec[0], rec[1], r, gx, gy, x0, y0, x1, y1);
          zb = __float_as_uint(rec[9]);
        }
      }
      if (r > 0) sx0 = x0 >> sbl, sx1 = ((x1 - 1) >> sbl) + 1, sy0 = y0 >> sbl, sy1 = ((y1 - 1) >> sbl) + 1;
      if (tail) {  // only flagged super-blocks can pass
        sx0 = max(sx0, fx0);
        sx1 = min(sx1, fx1 + 1);
        sy0 = max(sy0, fy0);
        sy1 = min(sy1, fy1 + 1);
        if (sx1 <= sx0 || sy1 <= sy0) r = 0;
      }
      // the super-blocks that pass: their bounding box (in super-blocks) clips the expansion,
      // since every tile outside it lies in a super-block whose tiles the keep test rejects
      int bx0 = sx1, bx1 = sx0 - 1, by0 = sy1, by1 = sy0 - 1;
      big = r > 0 && (sx1 - sx0) * (sy1 - sy0) > 16;
      if (r > 0 && !big) {
        for (int sy = sy0; sy < sy1; ++sy)
          for (int sx = sx0; sx < sx1; ++sx) {
            const bool nearer = zb <= s_cut[sy * nsx + sx];
            if (tail ? (!nearer && sbov[sy * nsx + sx] != 0u) : nearer) {
              bx0 = min(bx0, sx);
              bx1 = max(bx1, sx);
              by0 = min(by0, sy);
              by1 = max(by1, sy);
            }
          }
        if (bx1 < bx0) r = 0;
      }
      if (r > 0) {
        if (!big) {
          x0 = max(x0, bx0 << sbl);
          x1 = min(x1, (bx1 + 1) << sbl);
          y0 = max(y0, by0 << sbl);
          y1 = min(y1, (by1 + 1) << sbl);
        }
        key = ((uint64_t)zb << 32) | (uint32_t)g;
      }
    }
    if (wsurv) {  // deferred geometry: list the Gaussians that may emit (one LDS atomic per wave)
      const uint64_t m = __ballot(r > 0);
      if (m) {
        uint32_t base = 0u;
        if (lane == 0) base = atomicAdd(&s_nsurv, (uint32_t)__popcll(m));
        base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
        if (r > 0)
          wsurv[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
              (uint32_t)g;
      }
    }
    s_key[tid] = key;
    s_rx[w][lane] = (uint32_t)x0 | ((uint32_t)x1 << 16);
    s_ry[w][lane] = (uint32_t)y0 | ((uint32_t)y1 << 16);
    for_each_rect_tile(wr, lane, x0, y0, x1, y1, r > 0 && !big, gx, [&](int t, int o, int tx, int ty) {
      const uint64_t k = wkey[o];
      const bool nearer = (uint32_t)(k >> 32) <= s_cut[(ty >> sbl) * nsx + (tx >> sbl)];
      if (tail ? (!nearer && vov[t] != 0u) : nearer) keys[atomicAdd(&gcur[t], 1u)] = k;
    });
    // large rects (a few % of the Gaussians, but most of the rect tiles at 12x512x960):
    // (Gaussian, super-block) pairs balanced over the wave; the tiles of the pairs that pass (the
    // rect clipped to the super-block; the first pass keeps all of them) are then expanded
    // balanced again, 64 pairs at a time
    for_each_rect_window(wr, lane, sx0, sy0, sx1, sy1, big, nsx, [&](bool valid, int s, int o, int sx, int sy) {
      const uint64_t k = wkey[o];
      const bool nearer = (uint32_t)(k >> 32) <= s_cut[s];
      const bool pass = valid && (tail ? (!nearer && sbov[s] != 0u) : nearer);
      const uint32_t rx = s_rx[w][o], ry = s_ry[w][o];
      const int tx0 = max((int)(rx & 0xFFFFu), sx << sbl), tx1 = min((int)(rx >> 16), (sx + 1) << sbl);
      const int ty0 = max((int)(ry & 0xFFFFu), sy << sbl), ty1 = min((int)(ry >> 16), (sy + 1) << sbl);
      s_k2[w][lane] = k;
      for_each_rect_tile(s_wr2[w], lane, tx0, ty0, tx1, ty1, pass, gx, [&](int t, int o2, int, int) {
        if (!tail || vov[t] != 0u) keys[atomicAdd(&gcur[t], 1u)] = s_k2[w][o2];
      });
    });
  }
  if (wsurv) {
    __syncthreads();
    if (tid == 0) surv_count[(size_t)v * per_view + p] = s_nsurv;
  }
}

// Deferred geometry (dsr_project_survivors): the full projection (colour included) and the
// geometry record of every Gaussian listed by the scatter pass just before, for each view.
// A persistent grid: (view, run) workgroups walk the view's list. The same project_gauss as
// every other path, so the records are bit-identical to dsr_preprocess_fwd's.
template <int DEG>
__global__ __launch_bounds__(NT) void k_project_survivors(int G, int V, int H, int W, int gx, int gy, int M,
                                                          const float* __restrict__ means,
                                                          const float* __restrict__ shs,
                                                          const float* __restrict__ colors,
                                                          const float* __restrict__ opac,
                                                          const float* __restrict__ cov6,
                                                          const dsr_camera* __restrict__ cams,
                                                          const uint32_t* __restrict__ surv,
                                                          const uint32_t* __restrict__ surv_count,
                                                          float* __restrict__ geom, int32_t* __restrict__ radii,
                                                          long long* __restrict__ dzero,
                                                          uint8_t* __restrict__ row_live, int per_view, int layout) {
  // workgroup (v, p) projects the slice the scatter's workgroup (v, p) listed; a view's
  // workgroups on one XCD (its 48-byte records are scattered over the view's rows)
  int v, p;
  if (!xcd_item(per_view, V, v, p)) return;
  const dsr_camera* cam = cams + v;
  const size_t slice = survivor_slice(G, V);
  const uint32_t n = min(surv_count[(size_t)v * per_view + p], (uint32_t)slice);
  const uint32_t* ws = surv + ((size_t)v * per_view + p) * slice;
  const float2 focal = focal_of(cam, H, W);
  for (uint32_t i = threadIdx.x; i < n; i += NT) {
    const uint32_t g = ws[i];
    GaussIn<DEG> in;
    load_gauss<DEG>(in, (size_t)cam->scene * G + g, means, opac, cov6, layout);
    float rec[GS];
    int x0, y0, x1, y1;
    const int r = project_gauss<DEG>(in, cam, focal, H, W, gx, gy, M, shs, colors, layout, rec, x0, y0, x1, y1);
    const size_t vg = (size_t)v * G + g;
    store_geom(geom, radii, vg, rec, r, dzero);  // (training: the backward's row zeroed here too)
    if (row_live != nullptr && r > 0) row_live[vg] = 1u;  // the rows the backward reads
  }
}

// LDS add with same-address runs combined inside the wave first. Every lane of the wave calls
// it (act: this lane adds val to lds[addr]). Lanes whose (addr, val) equals the previous lane's
// extend that lane's run (the DPP wave shift: no LDS traffic), and the last lane of each run
// adds run length x val with one atomic. Pixel-aligned Gaussians of one context-image row sit
// in consecutive lanes with near-equal tile rects, so the difference-grid corners and the
// (super-block, depth bucket) counters they hit come in long runs: one LDS atomic per run
// instead of a same-address conflict chain per lane (round 4: 2.98 conflict cycles per LDS
// instruction in this kernel at 12x512x960).
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x138, 0xf, 0xf, false);  // wave_shr:1
}
// Lanes outside the exec mask (a divergent caller) neither extend nor end a run:
// the lane after an inactive lane is a run head, the lane before it a run end.
__device__ __forceinline__ void lds_add_runs(uint32_t* lds, uint32_t addr, uint32_t val, bool act, int lane) {
  const uint32_t a = act ? addr : 0xFFFFFFFFu - (uint32_t)lane;  // !act lanes start runs of their own
  const uint32_t v = act ? val : 0u;
  const uint32_t pa = wave_shr1(a), pv = wave_shr1(v);
  const uint64_t on = __ballot(true);  // the exec mask
  const bool prev_on = lane > 0 && ((on >> (lane - 1)) & 1ull);
  const bool head = !prev_on || a != pa || v != pv;
  const uint64_t hm = __ballot(head);
  const bool last = lane == 63 || !((on >> (lane + 1)) & 1ull) || ((hm >> (lane + 1)) & 1ull);
  if (act && last) {
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const int start = 63 - __clzll(hm & upto);
    atomicAdd(&lds[addr], (uint32_t)(lane - start + 1) * val);
  }
}

// K1 + depth histogram (dsr_preprocess_cut). NTH threads per workgroup; each workgroup owns
// one view and a contiguous run of NTH-Gaussian blocks (a persistent grid sized to the
// resident capacity), so its LDS count and depth histograms are flushed to HBM once for many
// blocks instead of once per block. Per-tile counts: each Gaussian adds its tile rect to a
// (gx+1) x (gy+1) difference grid (4 LDS atomics instead of one per touched tile: ~34 at
// 12x512x960); the flush turns it into counts with a 2D prefix sum. Depth histogram: per
// super-block of sb x sb tiles, each
// (Gaussian, touched super-block) adds the number of its tiles inside that super-block to
// the bucket of its depth (super-blocks, not tiles: at 6x448x768 a 16-tile super-block
// keeps the whole view's histogram in 43 KiB of LDS).
template <int DEG, int NTH, bool LAZY>
__global__ __launch_bounds__(NTH) void k_preprocess_cut(int G, int V, int H, int W, int gx, int gy, int M,
                                                        const float* __restrict__ means,
                                                        const float* __restrict__ shs,
                                                        const float* __restrict__ colors,
                                                        const float* __restrict__ opac,
                                                        const float* __restrict__ cov6,
                                                        const dsr_camera* __restrict__ cams,
                                                        float* __restrict__ geom, int32_t* __restrict__ radii,
                                                        long long* __restrict__ dzero,
                                                        uint32_t* __restrict__ seg_count,
                                                        uint32_t* __restrict__ depth_hist,
                                                        uint2* __restrict__ cut_rec, int per_view, int layout) {
  constexpr int NW = NTH / 64;
  extern __shared__ __attribute__((aligned(16))) uint32_t s_mem[];
  __shared__ WaveRects s_wr[NW];
  __shared__ uint32_t s_rx[NW][64], s_ry[NW][64], s_bk[NW][64];
  const int T = gx * gy;
  const int sb = cut_superblock(gx, gy), sbl = __builtin_ctz((unsigned)sb);
  const int nsx = (gx + sb - 1) / sb, nsb = nsx * ((gy + sb - 1) / sb);
  const int gxp = gx + 1, gyp = gy + 1;
  uint32_t* s_dif = s_mem;  // [gyp][gxp] difference grid of the tile rects
  uint32_t* s_dh = s_mem + gxp * gyp;
  // (run p, view v): the V workgroups of run p sit on one XCD (xcd_pair) and walk the same
  // blocks, so each block's inputs come from HBM once and from L2 for the other views
  int v, p;
  if (!xcd_pair(per_view, V, p, v)) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int k = tid; k < gxp * gyp + nsb * kCutBuckets; k += NTH) s_mem[k] = 0u;
  __syncthreads();
  const dsr_camera* cam = cams + v;
  const float2 focal = focal_of(cam, H, W);  // (two IEEE divisions, not re-done per block)
  const int nblk = (G + NTH - 1) / NTH;
  WaveRects& wr = s_wr[w];
  for (int blk = p; blk < nblk; blk += per_view) {  // round-robin blocks (see k_scatter_cut)
    const int g = blk * NTH + tid;
    int r = 0, x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    uint32_t zb = 0u;
    if (g < G) {
      GaussIn<DEG> in;
      load_gauss<DEG>(in, (size_t)cam->scene * G + g, means, opac, cov6, layout);
      float rec[GS];
      // LAZY (deferred geometry): no colour, no record; dsr_project_survivors writes the
      // records of the Gaussians the depth-cut scatter keeps (a few % of them)
      r = project_gauss<DEG, !LAZY>(in, cam, focal, H, W, gx, gy, M, shs, colors, layout, rec, x0, y0, x1, y1);
      if constexpr (LAZY)
        radii[(size_t)v * G + g] = r;
      else
        store_geom(geom, radii, (size_t)v * G + g, rec, r, dzero);
      zb = __float_as_uint(rec[9]);
    }
    // the rect's four difference-grid corners, same-address runs combined in the wave
    lds_add_runs(s_dif, (uint32_t)(y0 * gxp + x0), 1u, r > 0, lane);
    lds_add_runs(s_dif, (uint32_t)(y0 * gxp + x1), 0xFFFFFFFFu, r > 0, lane);
    lds_add_runs(s_dif, (uint32_t)(y1 * gxp + x0), 0xFFFFFFFFu, r > 0, lane);
    lds_add_runs(s_dif, (uint32_t)(y1 * gxp + x1), 1u, r > 0, lane);
    s_rx[w][lane] = (uint32_t)x0 | ((uint32_t)x1 << 16);
    s_ry[w][lane] = (uint32_t)y0 | ((uint32_t)y1 << 16);
    s_bk[w][lane] = (uint32_t)depth_bucket(zb);
    const int sx0 = x0 >> sbl, sy0 = y0 >> sbl;
    const int sx1 = r > 0 ? ((x1 - 1) >> sbl) + 1 : sx0, sy1 = r > 0 ? ((y1 - 1) >> sbl) + 1 : sy0;
    if (cut_rec && g < G)  // tile rect (non-zero: x1 >= 1 when visible) and depth bits
      cut_rec[(size_t)v * G + g] =
          make_uint2(r > 0 ? (uint32_t)x0 | ((uint32_t)x1 << 8) | ((uint32_t)y0 << 16) | ((uint32_t)y1 << 24) : 0u,
                     zb);
    // (Gaussian, super-block) pairs, every lane of each 64-pair window together: neighbouring
    // owners hit the same (super-block, depth bucket) counter, combined in the wave
    for_each_rect_window(wr, lane, sx0, sy0, sx1, sy1, r > 0, nsx, [&](bool valid, int s, int o, int sx, int sy) {
      uint32_t addr = 0u, val = 0u;
      if (valid) {
        const uint32_t rx = s_rx[w][o], ry = s_ry[w][o];
        const int ox = min((int)(rx >> 16), sx * sb + sb) - max((int)(rx & 0xFFFFu), sx * sb);
        const int oy = min((int)(ry >> 16), sy * sb + sb) - max((int)(ry & 0xFFFFu), sy * sb);
        addr = (uint32_t)(s * kCutBuckets) + s_bk[w][o];
        val = (uint32_t)(ox * oy);
      }
      lds_add_runs(s_dh, addr, val, valid, lane);
    });
  }
  __syncthreads();
  // 2D inclusive prefix sum of the difference grid: rows (odd stride gxp: no bank conflicts
  // when gx is even), then columns -> s_dif[ty][tx] = rects covering tile (tx, ty)
  for (int y = tid; y < gyp; y += NTH) {
    uint32_t acc = 0u;
    for (int x = 0; x < gxp; ++x) {
      acc += s_dif[y * gxp + x];
      s_dif[y * gxp + x] = acc;
    }
  }
  __syncthreads();
  for (int x = tid; x < gxp; x += NTH) {
    uint32_t acc = 0u;
    for (int y = 0; y < gyp; ++y) {
      acc += s_dif[y * gxp + x];
      s_dif[y * gxp + x] = acc;
    }
  }
  __syncthreads();
  uint32_t* gc = seg_count + (size_t)v * T;
  for (int t = tid; t < T; t += NTH) {
    const int ty = t / gx;
    const uint32_t c = s_dif[ty * gxp + (t - ty * gx)];
    if (c) atomicAdd(&gc[t], c);
  }
  uint32_t* gh = depth_hist + (size_t)v * nsb * kCutBuckets;
  for (int k = tid; k < nsb * kCutBuckets; k += NTH) {
    const uint32_t c = s_dh[k];
    if (c) atomicAdd(&gh[k], c);
  }
}

// One wave per (view, super-block): the depth (as float bits) at which the super-block's
// cumulative entry count reaches `prefix` per tile (0xffffffff, i.e. everything, if it never
// does).
__global__ __launch_bounds__(256) void k_bin_cutoff(int V, int gx, int gy, const uint32_t* __restrict__ hist,
                                                    uint32_t prefix, uint32_t* __restrict__ cut) {
  const int sb = cut_superblock(gx, gy);
  const int nsx = (gx + sb - 1) / sb, nsb = nsx * ((gy + sb - 1) / sb);
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (item >= V * nsb) return;
  const int s = item % nsb, sy = s / nsx, sx = s - sy * nsx;
  const uint32_t ntiles = (uint32_t)((min(gx, sx * sb + sb) - sx * sb) * (min(gy, sy * sb + sb) - sy * sb));
  const uint64_t target = (uint64_t)prefix * ntiles;
  static_assert(kCutBuckets == 128, "two buckets per lane");
  const uint32_t* h = hist + (size_t)item * kCutBuckets;
  const uint32_t a = h[2 * lane], b = h[2 * lane + 1];
  const uint32_t incl = dsplat::wave_incl_scan(a + b, lane);
  const uint32_t before = incl - (a + b);
  const uint64_t reach = __ballot((uint64_t)incl >= target);
  // the threshold: inside the reaching bucket, interpolated linearly in the depth bits by the
  // fraction of its count still needed (entries spread about evenly across one 1/16 octave),
  // so the written heads come out near `prefix` instead of a whole bucket above it
  uint32_t thr = 0xffffffffu;  // never reached (or the open last bucket): keep everything
  if (reach) {
    const int L = __ffsll((unsigned long long)reach) - 1;
    const uint32_t bL = (uint32_t)__shfl((int)before, L, 64);
    const uint32_t aL = (uint32_t)__shfl((int)a, L, 64);
    const uint32_t hL = (uint32_t)__shfl((int)b, L, 64);
    const bool first = (uint64_t)bL + aL >= target;
    const int c = 2 * L + (first ? 0 : 1);
    const uint32_t below = first ? bL : bL + aL, inb = first ? aL : hL;
    if (c < kCutBuckets - 1) {
      const float f = fminf(1.f, (float)(target - below) / (float)max(inb, 1u));
      thr = ((uint32_t)(c + (125 << 4)) << 19) + (uint32_t)(f * 524287.f);
      if (c == 0) thr = max(thr, 0x3E800000u);  // bucket 0 also holds everything nearer than 0.25
    }
  }
  if (lane == 0) cut[item] = thr;
}

// ------------------------------------------------------------------------------------
// K4: per-segment stable LSD radix sort (8-bit digits) with wave64 ballot ranking.
// Waves own contiguous, in-order ranges of the segment, so the pass is stable; keys are
// unique ((depth, id)), so the result equals upstream's stable sort order exactly.
__device__ __forceinline__ uint64_t match_digit(uint32_t d, uint64_t valid) {
  uint64_t m = valid;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t bb = __ballot(bit);
    m &= bit ? bb : ~bb;
  }
  return m;
}

// One pass src -> dst on digit (key >> shift) & 255. Returns false (and leaves dst
// untouched) when every key has the same digit. hist: LDS [NW][256]; wsum: LDS [4];
// flag: LDS word. Must be called by all NTH threads.
template <int NTH>
__device__ bool radix_pass(const uint64_t* src, uint64_t* dst, uint32_t n, int shift, uint32_t* hist,
                           uint32_t* wsum, uint32_t* flag) {
  constexpr int NW = NTH / kWave;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t chunk = (((n + NW - 1) / NW) + 63u) & ~63u;
  const uint32_t lo = min(n, (uint32_t)w * chunk), hi = min(n, lo + chunk);
  const uint64_t lt = dsplat::lanemask_lt(lane);
  for (int i = tid; i < NW * 256; i += NTH) hist[i] = 0;
  if (tid == 0) *flag = 0;
  __syncthreads();
  for (uint32_t base = lo; base < hi; base += 64) {
    const uint32_t i = base + lane;
    const bool valid = i < hi;
    const uint32_t d = valid ? (uint32_t)(src[i] >> shift) & 255u : 0u;
    const uint64_t peers = match_digit(d, __ballot(valid));
    if (valid && (peers & lt) == 0) hist[w * 256 + d] += (uint32_t)__popcll(peers);
  }
  __syncthreads();
  uint32_t tot = 0, incl = 0;
  if (tid < 256) {
    for (int ww = 0; ww < NW; ++ww) tot += hist[ww * 256 + tid];
    if (tot == n) *flag = 1;
    incl = dsplat::wave_incl_scan(tot, lane);
    if (lane == 63) wsum[w] = incl;
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t run = incl - tot;
    for (int ww = 0; ww < w; ++ww) run += wsum[ww];
    for (int ww = 0; ww < NW; ++ww) {
      const uint32_t c = hist[ww * 256 + tid];
      hist[ww * 256 + tid] = run;
      run += c;
    }
  }
  __syncthreads();
  if (*flag) return false;
  for (uint32_t base = lo; base < hi; base += 64) {
    const uint32_t i = base + lane;
    const bool valid = i < hi;
    const uint64_t key = valid ? src[i] : 0ull;
    const uint32_t d = (uint32_t)(key >> shift) & 255u;
    const uint64_t peers = match_digit(d, __ballot(valid));
    if (valid) {
      const uint32_t pos = hist[w * 256 + d] + (uint32_t)__popcll(peers & lt);
      dst[pos] = key;
      if ((peers & lt) == 0) hist[w * 256 + d] = pos + (uint32_t)__popcll(peers);
    }
  }
  __syncthreads();
  return true;
}

// Sort one segment by its 64-bit (depth << 32 | id) keys. Common case: 4 stable LSD
// passes over the depth bits only, then a tie check; pairs of equal depth (rare: random
// float depths) are put in id order by an insertion sort of each short run; segments with
// many ties (e.g. fronto-parallel planes) redo the full id-then-depth LSD (7 passes).
// Either way the result is the unique ascending order of the keys.
template <int NTH>
__device__ void sort_segment(uint64_t* A, uint64_t* B, uint32_t n, int id_bits, uint32_t* hist, uint32_t* wsum,
                             uint32_t* flag, uint64_t* home) {
  uint64_t* src = A;
  uint64_t* dst = B;
  for (int sh = 32; sh < 64; sh += 8)
    if (radix_pass<NTH>(src, dst, n, sh, hist, wsum, flag)) {
      uint64_t* t = src;
      src = dst;
      dst = t;
    }
  // tie check (flag reused as a counter)
  if (threadIdx.x == 0) *flag = 0;
  __syncthreads();
  uint32_t ties = 0;
  for (uint32_t i = threadIdx.x; i + 1 < n; i += NTH) ties += (uint32_t)((src[i] >> 32) == (src[i + 1] >> 32));
  if (ties) atomicAdd(flag, ties);
  __syncthreads();
  ties = *flag;
  __syncthreads();
  if (ties != 0 && ties <= 32) {
    // one thread per run of equal depth: insertion sort by the full key (= by id)
    for (uint32_t i = threadIdx.x; i + 1 < n; i += NTH) {
      const uint64_t d = src[i] >> 32;
      if ((src[i + 1] >> 32) != d || (i > 0 && (src[i - 1] >> 32) == d)) continue;
      uint32_t e = i + 1;
      while (e < n && (src[e] >> 32) == d) ++e;
      for (uint32_t k = i + 1; k < e; ++k) {
        const uint64_t x = src[k];
        uint32_t m = k;
        while (m > i && src[m - 1] > x) {
          src[m] = src[m - 1];
          --m;
        }
        src[m] = x;
      }
    }
    __syncthreads();
  } else if (ties > 32) {
    for (int sh = 0; sh < id_bits; sh += 8)
      if (radix_pass<NTH>(src, dst, n, sh, hist, wsum, flag)) {
        uint64_t* t = src;
        src = dst;
        dst = t;
      }
    for (int sh = 32; sh < 64; sh += 8)
      if (radix_pass<NTH>(src, dst, n, sh, hist, wsum, flag)) {
        uint64_t* t = src;
        src = dst;
        dst = t;
      }
  }
  if (src != home)
    for (uint32_t i = threadIdx.x; i < n; i += NTH) home[i] = src[i];
}

// The tail pass's sort (dsr_bin_sort with seg_filter): the flagged tiles are few (0-21 of
// 19,200 per config-E launch) and each is a whole list of 10-30 K keys. A persistent grid of
// 1024-thread workgroups walks the segments and sorts the flagged ones through HBM with 16
// waves each (sort_segment<1024>: 4x the threads of the LDS-sort workgroup); when no tile is
// flagged (the any-flag word filter[nseg] is 0) every workgroup leaves at once. It replaces one
// LDS-heavy workgroup per segment, whose dispatch alone took ~0.3 ms per config-E launch
// (round 5).
template <int NTH>
__global__ __launch_bounds__(NTH) void k_sort_flagged(int nseg, const uint32_t* __restrict__ seg_start,
                                                      const uint32_t* __restrict__ seg_count, uint32_t stride,
                                                      uint64_t* __restrict__ keys, uint64_t* __restrict__ scratch,
                                                      int id_bits, const uint32_t* __restrict__ filter,
                                                      uint32_t* __restrict__ seg_sorted) {
  __shared__ uint32_t hist[(NTH / kWave) * 256];
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t flag[4];
  if (filter[nseg] == 0u) return;  // no tile flagged (uniform)
  for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    if (filter[seg] == 0u) continue;  // uniform
    uint32_t b, e;
    seg_bounds(seg_start, seg_count, stride, seg, b, e);
    const uint32_t n = e - b;
    if (seg_sorted && threadIdx.x == 0) seg_sorted[seg] = n;
    if (n > 1) sort_segment<NTH>(keys + b, scratch + b, n, id_bits, hist, wsum, flag, keys + b);
    __syncthreads();  // LDS reused by the next flagged segment
  }
}

// ---- in-LDS segment sort (n <= 256 * KMAX) -------------------------------------------
// Keys live in LDS; each pass every thread loads its KMAX contiguous keys into registers,
// ranks them with per-thread packed 8-bit counters for a 4-bit digit (no ballots, no
// atomics, no serial dependency across threads), one block-wide scan of the 16 x 256
// counters (u16, digit-major) gives every (digit, thread) its output base, and keys are
// scattered to the other LDS buffer. Contiguous ownership + digit-major scan = stable.
// LDS index padding i + i / KMAX makes the per-thread row reads bank-conflict free.
template <int KMAX>
__device__ __forceinline__ uint32_t padi(uint32_t i) { return i + i / KMAX; }

// digit of a key: ((32-bit word at word_shift) - dbase) >> shift & 15
template <int KMAX>
__device__ __forceinline__ uint32_t key_digit(uint64_t k, int word_shift, uint32_t dbase, int shift) {
  return (((uint32_t)(k >> word_shift) - dbase) >> shift) & 15u;
}

template <int KMAX, int NTH = NT>
__device__ bool reg_pass(uint64_t* buf, uint32_t n, int word_shift, uint32_t dbase, int shift, uint16_t* cnt,
                         uint32_t* wsum) {
  // in place: every key of the pass is in registers before the first barrier, so the
  // scatter can overwrite the same LDS buffer (one buffer -> more workgroups per CU)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t base = (uint32_t)tid * KMAX;
  // registers: the keys, their within-thread ranks packed 4 per word (digits are recomputed
  // at the scatter), and the 16 per-thread digit counters packed 8 per 64-bit word
  uint64_t k[KMAX];
  uint32_t locp[(KMAX + 3) / 4];
#pragma unroll
  for (int i = 0; i < (KMAX + 3) / 4; ++i) locp[i] = 0u;
  uint64_t c_lo = 0, c_hi = 0;
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    const uint32_t idx = base + i;
    const bool valid = idx < n;
    k[i] = valid ? buf[padi<KMAX>(idx)] : 0ull;
    const uint32_t d = valid ? key_digit<KMAX>(k[i], word_shift, dbase, shift) : 16u;
    const uint32_t sh8 = 8u * (d & 7u);
    uint32_t loc;
    if (d < 8u) {
      loc = (uint32_t)(c_lo >> sh8) & 255u;
      c_lo += 1ull << sh8;
    } else {
      loc = (uint32_t)(c_hi >> sh8) & 255u;
      if (d < 16u) c_hi += 1ull << sh8;
    }
    locp[i / 4] |= loc << (8 * (i % 4));
  }
  const uint32_t d0 = key_digit<KMAX>(buf[0], word_shift, dbase, shift);  // digit of key 0 (broadcast read)
#pragma unroll
  for (int d = 0; d < 16; ++d) cnt[d * NTH + tid] = (uint16_t)(((d < 8 ? c_lo : c_hi) >> (8 * (d & 7))) & 255u);
  __syncthreads();
  // exclusive scan of the 4096 counters in (digit, thread) order; thread t owns [16t, 16t+16)
  uint32_t v[16];
  {
    const uint4* p = reinterpret_cast<const uint4*>(cnt + 16 * tid);
    const uint4 x = p[0], y = p[1];
    const uint32_t wds[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      v[2 * q] = wds[q] & 0xFFFFu;
      v[2 * q + 1] = wds[q] >> 16;
    }
  }
  uint32_t tot = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const uint32_t c = v[q];
    v[q] = tot;
    tot += c;
  }
  const uint32_t incl = dsplat::wave_incl_scan(tot, lane);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t off = incl - tot;
  for (int ww = 0; ww < w; ++ww) off += wsum[ww];
  {
    uint32_t wds[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) wds[q] = (v[2 * q] + off) | ((v[2 * q + 1] + off) << 16);
    uint4* p = reinterpret_cast<uint4*>(cnt + 16 * tid);
    p[0] = make_uint4(wds[0], wds[1], wds[2], wds[3]);
    p[1] = make_uint4(wds[4], wds[5], wds[6], wds[7]);
  }
  __syncthreads();
  // a digit holding every key makes the pass the identity (same decision in every thread)
  const uint32_t s0 = cnt[d0 * NTH];
  const uint32_t s1 = d0 < 15 ? (uint32_t)cnt[(d0 + 1) * NTH] : n;
  if (s1 - s0 == n) return false;  // nothing written; the next pass re-reads buf
#pragma unroll
  for (int i = 0; i < KMAX; ++i)
    if (base + i < n) {
      const uint32_t d = key_digit<KMAX>(k[i], word_shift, dbase, shift);
      const uint32_t loc = (locp[i / 4] >> (8 * (i % 4))) & 255u;
      buf[padi<KMAX>((uint32_t)cnt[d * NTH + tid] + loc)] = k[i];
    }
  __syncthreads();
  return true;
}

// Sort of one segment in LDS. Keys are (depth bits << 32 | id), all distinct. The passes
// only look at the 16 bits of (depth - min depth) below the highest bit in which the
// segment's depths differ (4 passes instead of 8); keys that agree on those bits form runs
// that are then put in full-key order by one thread each (insertion sort). Bits above the
// range are common to every key and bits below the window only order keys inside a run, so
// this is the full (depth, id) order. Runs longer than 32 (depths packed far tighter than the
// segment's range) fall back to full-width passes: ids, then all 32 depth bits (stable).
// Runs of keys that agree on ((depth - mn) >> shift) are put in full-key order: thread t
// walks the runs that start in its KMAX positions and insertion-sorts each (full 64-bit keys;
// runs may extend past its range). Runs longer than 32 (depths packed far tighter than the
// window resolves) fall back to full-width LSD passes: ids, then all 32 depth bits (stable).
template <int KMAX, int NTH = NT>
__device__ void fix_runs(uint64_t* A, uint32_t n, uint32_t mn, int shift, int id_bits, uint16_t* cnt, uint32_t* wsum,
                         uint32_t* flag) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NW = NTH / 64;
#define pref(i) ((((uint32_t)(A[padi<KMAX>(i)] >> 32)) - mn) >> shift)
  uint32_t longest = 0;
  {
    // prefixes of positions i0 - 1 .. i0 + KMAX (independent LDS reads, all in flight)
    const uint32_t i0 = (uint32_t)tid * KMAX;
    uint32_t pf[KMAX + 2];
#pragma unroll
    for (int j = 0; j < KMAX + 2; ++j) {
      const uint32_t i = i0 + (uint32_t)j - 1u;
      pf[j] = (j > 0 || i0 > 0) && i0 + j - 1 < n ? pref(i) : 0xffffffffu - (uint32_t)j;
    }
    uint32_t starts = 0;  // bit j: a run (>= 2 equal prefixes) starts at i0 + j
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
      if (i0 + j + 1 < n && pf[j + 1] != pf[j] && pf[j + 1] == pf[j + 2]) starts |= 1u << j;
    while (starts) {
      const int j = __builtin_ctz(starts);
      starts &= starts - 1;
      const uint32_t i = i0 + (uint32_t)j, p = pref(i);
      uint32_t e = i + 2;
      while (e < n && e - i <= 32 && pref(e) == p) ++e;
      longest = max(longest, e - i);
      if (e - i <= 32) {
        if (e - i == 2) {
          const uint64_t x0 = A[padi<KMAX>(i)], x1 = A[padi<KMAX>(i + 1)];
          if (x0 > x1) {
            A[padi<KMAX>(i)] = x1;
            A[padi<KMAX>(i + 1)] = x0;
          }
        } else {
          for (uint32_t k = i + 1; k < e; ++k) {
            const uint64_t x = A[padi<KMAX>(k)];
            uint32_t m = k;
            while (m > i && A[padi<KMAX>(m - 1)] > x) {
              A[padi<KMAX>(m)] = A[padi<KMAX>(m - 1)];
              --m;
            }
            A[padi<KMAX>(m)] = x;
          }
        }
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) longest = max(longest, (uint32_t)__shfl_xor((int)longest, off, 64));
  if (lane == 0) flag[w] = longest;
  __syncthreads();
  longest = flag[0];
#pragma unroll
  for (int k = 1; k < NW; ++k) longest = max(longest, flag[k]);
  __syncthreads();
  if (longest <= 32) return;
  {
    for (int sh = 0; sh < id_bits; sh += 4) reg_pass<KMAX, NTH>(A, n, 0, 0u, sh, cnt, wsum);
    for (int sh = 0; sh < 32; sh += 4) reg_pass<KMAX, NTH>(A, n, 32, 0u, sh, cnt, wsum);
  }
#undef pref
}

// block min / max of the keys' depth words (flag[0 .. 2 NW) scratch; two barriers)
template <int NTH>
__device__ __forceinline__ void block_minmax(uint32_t& mn, uint32_t& mx, uint32_t* flag) {
  constexpr int NW = NTH / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, off, 64));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
  }
  if (lane == 0) {
    flag[w] = mn;
    flag[NW + w] = mx;
  }
  __syncthreads();
  mn = flag[0];
  mx = flag[NW];
#pragma unroll
  for (int k = 1; k < NW; ++k) {
    mn = min(mn, flag[k]);
    mx = max(mx, flag[NW + k]);
  }
  __syncthreads();
}

// Sort of one segment in LDS. Keys are (depth bits << 32 | id), all distinct. The passes
// only look at the 16 bits of (depth - min depth) below the highest bit in which the
// segment's depths differ (4 passes instead of 8); fix_runs then orders keys equal on those bits.
template <int KMAX, int NTH = NT>
__device__ void reg_sort(uint64_t* A, uint32_t n, int id_bits, uint16_t* cnt, uint32_t* wsum, uint32_t* flag) {
  const int tid = threadIdx.x;
  uint32_t mn = 0xffffffffu, mx = 0u;
  for (uint32_t i = tid; i < n; i += NTH) {
    const uint32_t d = (uint32_t)(A[padi<KMAX>(i)] >> 32);
    mn = min(mn, d);
    mx = max(mx, d);
  }
  block_minmax<NTH>(mn, mx, flag);
  const uint32_t range = mx - mn;
  const int msb = range ? 31 - __clz(range) : -1;
  const int lo_shift = max(0, msb - 15);
  for (int sh = lo_shift; sh <= msb; sh += 4) reg_pass<KMAX, NTH>(A, n, 32, mn, sh, cnt, wsum);
  fix_runs<KMAX, NTH>(A, n, mn, lo_shift, id_bits, cnt, wsum, flag);
}

// One-pass alternative: a counting sort on the top 12 bits of (depth - min) — a 4096-bin
// histogram (u16 counts, two per LDS word), its scan, and one scatter — then every key ranks
// itself inside its bin. With ~3K keys over 4096 bins most bins hold 0-2 keys: 6 barriers
// and no serial insertion chains (the LSD passes + fix_runs took 35 us per launch at 2x256^2,
// 21 of them in fix_runs). The keys come in registers (thread t holds keys t + i NTH).
// Bin-pair word w of the counting sort lives at LDS word bin_word<R>(w): each thread's scan
// row of R words is read / written as R/4 16-byte chunks (ds_read_b128 / ds_write_b128) and
// the chunks are XOR-rotated by (thread / 4) mod (R/4), so the 16 lanes of one b128 lane
// group touch 16 different 4-bank slots. Unswizzled, rows of 16 words at a 64-byte lane
// stride put 4 lanes of a group on each slot (4-way conflicts in every scan access).
template <int R>
__device__ __forceinline__ uint32_t bin_word(uint32_t w) {
  static_assert(R >= 4 && (R & (R - 1)) == 0, "rows of whole 16-byte chunks");
  constexpr int RL = R == 4 ? 2 : R == 8 ? 3 : R == 16 ? 4 : R == 32 ? 5 : 6;
  return w ^ ((((w >> RL) >> 2) & (uint32_t)(R / 4 - 1)) << 2);
}

template <int KMAX, int NTH = NT, int NBL = kSortNBinLog2>
__device__ void count_sort(const uint64_t (&tmp)[KMAX], uint32_t n, uint64_t* A, int id_bits, uint16_t* cnt,
                           uint32_t* wsum, uint32_t* flag) {
  constexpr int NBIN = 1 << NBL, BPT = NBIN / NTH;  // bins per thread in the scan
  constexpr int R = BPT / 2;                                    // scan row: bin-pair words per thread
  constexpr uint32_t kBinMax = 16;  // larger bins (clustered / equal depths): LSD passes instead
  static_assert(BPT % 8 == 0 && NTH * KMAX < 65536 && NBIN / 2 <= sort_cnt_words<NTH, NBL>(), "u16 bin pairs in cnt");
  uint32_t* hw = reinterpret_cast<uint32_t*>(cnt);  // NBIN / 2 words (cnt holds NTH * 16 u16), 16-B aligned
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t mn = 0xffffffffu, mx = 0u;
#pragma unroll
  for (int i = 0; i < KMAX; ++i)
    if (tid + (uint32_t)i * NTH < n) {
      const uint32_t d = (uint32_t)(tmp[i] >> 32);
      mn = min(mn, d);
      mx = max(mx, d);
    }
  {
    uint4* h4 = reinterpret_cast<uint4*>(hw);
    for (int k = tid; k < NBIN / 8; k += NTH) h4[k] = make_uint4(0u, 0u, 0u, 0u);
  }
  block_minmax<NTH>(mn, mx, flag);
  const uint32_t range = mx - mn;
  const int shift = max(0, (range ? 31 - __clz(range) : 0) - (NBL - 1));
  // count pass: the atomic's return value is the key's rank among the keys of its bin that
  // got there first, so the scatter needs no second atomic pass (u16 halves never carry:
  // n < 65536)
  uint32_t rk[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    rk[i] = 0u;
    if (tid + (uint32_t)i * NTH < n) {
      const uint32_t bin = ((uint32_t)(tmp[i] >> 32) - mn) >> shift;
      const uint32_t s16 = (bin & 1u) * 16u;
      rk[i] = (atomicAdd(&hw[bin_word<R>(bin >> 1)], 1u << s16) >> s16) & 0xFFFFu;
    }
  }
  __syncthreads();
  {
    uint4* row = reinterpret_cast<uint4*>(hw) + tid * (R / 4);
    const int rot = (tid >> 2) & (R / 4 - 1);
    uint32_t wd[R], tot = 0;
#pragma unroll
    for (int c = 0; c < R / 4; ++c) {
      const uint4 x = row[c ^ rot];
      wd[4 * c] = x.x;
      wd[4 * c + 1] = x.y;
      wd[4 * c + 2] = x.z;
      wd[4 * c + 3] = x.w;
    }
#pragma unroll
    for (int q = 0; q < R; ++q) tot += (wd[q] & 0xFFFFu) + (wd[q] >> 16);
    const uint32_t incl = dsplat::wave_incl_add_dpp(tot);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t off = incl - tot;
    for (int k = 0; k < w; ++k) off += wsum[k];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const uint32_t lo = wd[q] & 0xFFFFu, hi = wd[q] >> 16;
      wd[q] = off | ((off + lo) << 16);  // start offsets of bins 2q, 2q + 1
      off += lo + hi;
    }
#pragma unroll
    for (int c = 0; c < R / 4; ++c) row[c ^ rot] = make_uint4(wd[4 * c], wd[4 * c + 1], wd[4 * c + 2], wd[4 * c + 3]);
  }
  __syncthreads();
  // bin b is [start(b), start(b + 1)), the last bin ending at n
  auto bin_start = [&](uint32_t b) -> uint32_t {
    if (b >= (uint32_t)NBIN) return n;
    const uint32_t wv = hw[bin_word<R>(b >> 1)];
    return (b & 1u) ? (wv >> 16) : (wv & 0xFFFFu);
  };
  uint32_t multi = 0u;  // bit i: key i shares its bin (its final place needs the in-bin rank)
  bool big = false;
#pragma unroll
  for (int i = 0; i < KMAX; ++i)
    if (tid + (uint32_t)i * NTH < n) {
      const uint32_t bin = ((uint32_t)(tmp[i] >> 32) - mn) >> shift;
      const uint32_t st = bin_start(bin), c = bin_start(bin + 1u) - st;
      A[padi<KMAX>(st + rk[i])] = tmp[i];
      big |= c > kBinMax;
      if (c > 1u) multi |= 1u << i;
      rk[i] = st | (c << 16);
    }
  if (__syncthreads_or(big)) {  // a clustered segment: A holds the keys grouped by bin, sort it outright
    reg_sort<KMAX, NTH>(A, n, id_bits, cnt, wsum, flag);
    return;
  }
  // order inside each shared bin (<= kBinMax keys): count the smaller keys of the bin (c
  // independent LDS reads, all lanes in parallel); single-key bins are already in place
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    if (multi & (1u << i)) {
      const uint32_t st = rk[i] & 0xFFFFu, e = st + (rk[i] >> 16);
      uint32_t r = 0;
      for (uint32_t j = st; j < e; ++j) r += A[padi<KMAX>(j)] < tmp[i] ? 1u : 0u;
      rk[i] = st + r;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < KMAX; ++i)
    if (multi & (1u << i)) A[padi<KMAX>(rk[i])] = tmp[i];
  __syncthreads();
}

// One workgroup per (view, tile) segment. n <= 256*KMAX: sort in LDS. Larger: when
// big_here, sort through HBM (keys <-> scratch) with the ballot-ranked passes; otherwise
// leave it to the MSD split (k_msd_split + k_sort_groups).
template <int KMAX, int NTH = NT>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(KMAX * NTH >= 8192 ? 1 : kSortWPE))) void k_sort_lds(const uint32_t* __restrict__ seg_start,
                                                 const uint32_t* __restrict__ seg_count, uint32_t stride,
                                                 uint64_t* __restrict__ keys, uint64_t* __restrict__ scratch,
                                                 int id_bits, int big_here, const uint32_t* __restrict__ filter,
                                                 uint32_t* __restrict__ seg_sorted) {
  constexpr uint32_t cap = NTH * KMAX;
  constexpr uint32_t padded = cap + cap / KMAX;
  extern __shared__ __attribute__((aligned(16))) uint64_t s_keys[];
  uint64_t* A = s_keys;
  uint32_t* aux = reinterpret_cast<uint32_t*>(A + padded);  // 8 KiB counters (u16) / HBM-path histogram
  uint16_t* cnt = reinterpret_cast<uint16_t*>(aux);
  uint32_t* wsum = aux + sort_cnt_words<NTH>();
  uint32_t* flag = wsum + 16;
  const int seg = blockIdx.x;
  if (filter && !filter[seg]) return;
  uint32_t b, e;
  seg_bounds(seg_start, seg_count, stride, seg, b, e);
  const uint32_t n = e - b;
  if (seg_sorted && threadIdx.x == 0 && (n <= cap || big_here)) seg_sorted[seg] = n;
  if (n <= 1) return;
  if (n > cap) {
    if (big_here) sort_segment<NTH>(keys + b, scratch + b, n, id_bits, aux, wsum, flag, keys + b);
    return;
  }
  // all KMAX global loads of a thread in flight at once (coalesced across the workgroup)
  {
    uint64_t tmp[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      const uint32_t idx = threadIdx.x + (uint32_t)i * NTH;
      tmp[i] = idx < n ? keys[b + idx] : 0ull;
    }
    count_sort<KMAX, NTH>(tmp, n, A, id_bits, cnt, wsum, flag);
  }
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    const uint32_t idx = threadIdx.x + (uint32_t)i * NTH;
    if (idx < n) keys[b + idx] = A[padi<KMAX>(idx)];
  }
}

template <int KMAX, int NTH = NT>
constexpr size_t sort_lds_bytes() {
  return (size_t)(NTH * KMAX + NTH) * 8 + (size_t)sort_cnt_words<NTH>() * 4 + 64 * 4;
}

// ---- segments larger than the LDS sort (6-view 448x768 and up: ~30-40K entries per tile) --
// One MSD pass splits each such segment by the top 12 bits of (depth - segment min) into
// 4096 buckets, written bucket-contiguous to `scratch` at the segment's own offsets; runs of
// consecutive buckets then form groups of at most ~kGroupCap keys (a group ends at the first
// bucket boundary past each multiple of kGroupCap/2), and every group is sorted by the full
// key in LDS (k_sort_groups) straight into `keys`. Buckets are ordered ranges of depth, so
// sorted groups concatenate into the sorted segment. Two HBM round trips per key instead of
// eight radix passes. A group still above the LDS capacity (one bucket holding > ~2K keys
// of near-equal depth) takes the HBM radix path inside k_sort_groups.
constexpr int kSplitNB = 4096;
constexpr uint32_t kGroupCap = NT * 16;  // k_sort_groups<16>
constexpr uint32_t kGroupHalf = kGroupCap / 2;
constexpr uint32_t kFromKeys = 0x80000000u;  // group flag: data still in keys (not split)

__host__ __device__ inline int split_groups(uint32_t max_count) { return (int)((max_count + kGroupHalf - 1) / kGroupHalf) + 1; }

__device__ __forceinline__ uint32_t split_bound(const uint32_t* hist, uint32_t target, uint32_t n) {
  // first bucket offset >= target (n if none); hist holds exclusive bucket offsets
  if (target == 0) return 0u;
  if (target >= n) return n;
  int lo = 0, hi = kSplitNB;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (hist[mid] >= target) hi = mid;
    else lo = mid + 1;
  }
  return lo < kSplitNB ? hist[lo] : n;
}

// Prefix mode (prefix > 0, for the segments longer than `prefix`): only the nearest part of
// the segment is sorted. The split's bucket offsets give P = the first bucket boundary at or
// past `prefix`; keys of the buckets below it go to scratch (bucket-contiguous) and are
// sorted into keys[0, P) by k_sort_groups, while the keys of the remaining buckets (all
// deeper than every prefix key) are left, unordered, in keys[P, n): those already there
// stay, and those that sat in [0, P) move into the holes left by prefix keys found in
// [P, n) (the two counts are equal). seg_sorted[seg] = P. The compositor only has to
// confirm that no tail key reaches a pixel that is still live (k_render_fwd).
constexpr int kSplitNT = 512;
constexpr int kSplitKPT = 82;         // depth words per thread kept in registers: segments up to 41984
constexpr uint32_t kStageCap = 5120;  // prefix keys assembled in LDS, then written out contiguously
constexpr uint32_t kHoleCap = 5120;
constexpr uint32_t kMinPrefix = 1024;
constexpr size_t split_lds_bytes() { return (size_t)kStageCap * 8 + (size_t)(kSplitNB + kHoleCap) * 4; }

// One workgroup per long segment (two per CU). The depth words of a segment of up to
// NTH*KPT keys are read once and held in registers for the min/max, histogram and
// classification passes; only the keys that move (the sorted prefix, and tail keys sitting
// inside [0, P)) are read again in full. Longer segments re-read per pass. The prefix is
// assembled in LDS and written to scratch with contiguous stores. In prefix mode P is the
// first bucket boundary at or past `prefix`, or, when that exceeds kStageCap, the last one
// below it (if at least kMinPrefix): a shorter prefix is still exact (the compositor's tail
// check catches what it misses) and keeps the work bounded.
template <int NTH, int KPT>
__global__ __launch_bounds__(NTH) void k_msd_split(const uint32_t* __restrict__ seg_start,
                                                   const uint32_t* __restrict__ seg_count, uint32_t stride,
                                                   uint64_t* __restrict__ keys, uint64_t* __restrict__ scratch,
                                                   uint32_t small_cap, uint32_t* __restrict__ groups, int gmax,
                                                   uint32_t prefix, uint32_t* __restrict__ seg_sorted) {
  constexpr int NW = NTH / 64;
  constexpr int BPT = kSplitNB / NTH;  // buckets per thread in the scan
  extern __shared__ __attribute__((aligned(16))) uint64_t s_stage[];  // kStageCap
  uint32_t* hist = reinterpret_cast<uint32_t*>(s_stage + kStageCap);
  uint32_t* holes = hist + kSplitNB;
  __shared__ uint32_t red[2 * NW + 2];
  const int seg = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t* gout = groups + (size_t)seg * gmax * 2;
  uint32_t b, e;
  seg_bounds(seg_start, seg_count, stride, seg, b, e);
  const uint32_t n = e - b;
  if (n <= small_cap) {  // sorted by k_sort_lds already
    for (int g = tid; g < gmax; g += NTH) gout[2 * g] = gout[2 * g + 1] = 0u;
    if (seg_sorted && tid == 0) seg_sorted[seg] = n;
    return;
  }
  const bool pfx = prefix != 0 && n > prefix;
  if (!pfx && (int)((n + kGroupHalf - 1) / kGroupHalf) + 1 > gmax) {  // larger than the launch was sized for
    for (int g = tid; g < gmax; g += NTH) {
      gout[2 * g] = g == 0 ? b : 0u;
      gout[2 * g + 1] = g == 0 ? (e | kFromKeys) : 0u;
    }
    if (seg_sorted && tid == 0) seg_sorted[seg] = n;
    return;
  }
  const bool inreg = n <= (uint32_t)(NTH * KPT);  // uniform
  uint32_t rd[KPT];
  if (inreg) {
#pragma unroll
    for (int q = 0; q < KPT; ++q) {
      const uint32_t i = tid + (uint32_t)q * NTH;
      rd[q] = i < n ? (uint32_t)(keys[b + i] >> 32) : 0u;
    }
  }
  // BODY sees the depth word d of key index i (valid lanes only)
#define SPLIT_VISIT(BODY)                                  \
  if (inreg) {                                             \
    _Pragma("unroll") for (int q = 0; q < KPT; ++q) {      \
      const uint32_t i = tid + (uint32_t)q * NTH;          \
      if (i < n) {                                         \
        const uint32_t d = rd[q];                          \
        BODY                                               \
      }                                                    \
    }                                                      \
  } else {                                                 \
    for (uint32_t i = tid; i < n; i += NTH) {              \
      const uint32_t d = (uint32_t)(keys[b + i] >> 32);    \
      BODY                                                 \
    }                                                      \
  }
  // segment min / max of the depth word
  uint32_t mn = 0xffffffffu, mx = 0u;
  SPLIT_VISIT({
    mn = min(mn, d);
    mx = max(mx, d);
  })
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, off, 64));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
  }
  if (lane == 0) {
    red[w] = mn;
    red[NW + w] = mx;
  }
  for (int k = tid; k < kSplitNB; k += NTH) hist[k] = 0u;
  if (tid == 0) red[2 * NW] = red[2 * NW + 1] = 0u;
  __syncthreads();
  mn = red[0];
  mx = red[NW];
  for (int k = 1; k < NW; ++k) {
    mn = min(mn, red[k]);
    mx = max(mx, red[NW + k]);
  }
  const uint32_t range = mx - mn;
  const int msb = range ? 31 - __clz(range) : 0;
  const int sh = max(0, msb - 11);
  __syncthreads();
  SPLIT_VISIT({ atomicAdd(&hist[(d - mn) >> sh], 1u); })
  __syncthreads();
  // exclusive scan: thread t owns buckets [BPT t, BPT t + BPT)
  uint32_t c[BPT], tot = 0;
#pragma unroll
  for (int k = 0; k < BPT; ++k) {
    c[k] = hist[BPT * tid + k];
    tot += c[k];
  }
  const uint32_t incl = dsplat::wave_incl_scan(tot, lane);
  if (lane == 63) red[w] = incl;
  __syncthreads();
  uint32_t off = incl - tot;
  for (int k = 0; k < w; ++k) off += red[k];
#pragma unroll
  for (int k = 0; k < BPT; ++k) {
    hist[BPT * tid + k] = off;
    off += c[k];
  }
  __syncthreads();
  // prefix cut: buckets >= kc (offsets >= P) stay unsorted in keys[P, n)
  uint32_t P = n;
  int kc = kSplitNB;
  if (pfx) {
    int lo = 0, hi = kSplitNB;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (hist[mid] >= prefix) hi = mid;
      else lo = mid + 1;
    }
    kc = lo;
    P = lo < kSplitNB ? hist[lo] : n;
    if (P > kStageCap && kc > 0 && hist[kc - 1] >= kMinPrefix) {  // shorter prefix, one bucket less
      --kc;
      P = hist[kc];
    }
    if (min(P, n - P) > kHoleCap) {  // pathological depth clustering: sort all of it
      P = n;
      kc = kSplitNB;
    }
    // groups [B_g, B_g+1) for g < prefix / kGroupHalf cover [0, P) whenever P <= bound(prefix);
    // only a full sort of a segment this long can need more than the launch has
    if (P == n && (int)((n + kGroupHalf - 1) / kGroupHalf) + 1 > gmax) {  // uniform across the workgroup
      for (int g = tid; g < gmax; g += NTH) {
        gout[2 * g] = g == 0 ? b : 0u;
        gout[2 * g + 1] = g == 0 ? (e | kFromKeys) : 0u;
      }
      if (seg_sorted && tid == 0) seg_sorted[seg] = n;
      return;
    }
  }
  if (seg_sorted && tid == 0) seg_sorted[seg] = P;
  // group g = [B_g, B_{g+1}) clipped to [0, P), B_g = first bucket offset >= g * kGroupHalf
  for (int g = tid; g < gmax; g += NTH) {
    const uint32_t g0 = min(split_bound(hist, (uint32_t)g * kGroupHalf, n), P);
    const uint32_t g1 = min(split_bound(hist, (uint32_t)(g + 1) * kGroupHalf, n), P);
    gout[2 * g] = b + g0;
    gout[2 * g + 1] = b + g1;
  }
  const bool stage = P <= kStageCap;
  __syncthreads();
  SPLIT_VISIT({
    const int bk = (int)((d - mn) >> sh);
    if (bk < kc) {
      const uint64_t k = keys[b + i];
      const uint32_t pos = atomicAdd(&hist[bk], 1u);
      if (stage) s_stage[pos] = k;
      else scratch[b + pos] = k;
      if (i >= P) holes[atomicAdd(&red[2 * NW], 1u)] = i;
    }
  })
  __syncthreads();
  if (stage)
    for (uint32_t i = tid; i < P; i += NTH) scratch[b + i] = s_stage[i];
  if (P < n) {
    SPLIT_VISIT({
      if (i < P && (int)((d - mn) >> sh) >= kc) keys[b + holes[atomicAdd(&red[2 * NW + 1], 1u)]] = keys[b + i];
    })
  }
#undef SPLIT_VISIT
}

// Sort every group produced by k_msd_split into `keys` (from scratch, or from keys when the
// segment was not split). grid = nseg * gmax.
template <int KMAX>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(kSortWPE))) void k_sort_groups(
    const uint32_t* __restrict__ groups, uint64_t* __restrict__ keys, uint64_t* __restrict__ scratch, int id_bits) {
  constexpr uint32_t cap = NT * KMAX;
  constexpr uint32_t padded = cap + cap / KMAX;
  extern __shared__ __attribute__((aligned(16))) uint64_t s_keys[];
  uint64_t* A = s_keys;
  uint32_t* aux = reinterpret_cast<uint32_t*>(A + padded);
  uint16_t* cnt = reinterpret_cast<uint16_t*>(aux);
  uint32_t* wsum = aux + 2048;
  uint32_t* flag = wsum + 16;
  const uint32_t b = groups[2 * blockIdx.x], ew = groups[2 * blockIdx.x + 1];
  const uint32_t e = ew & ~kFromKeys;
  if (e <= b) return;
  const uint32_t n = e - b;
  uint64_t* src = (ew & kFromKeys) ? keys : scratch;
  if (n > cap) {
    sort_segment<NT>(src + b, (src == keys ? scratch : keys) + b, n, id_bits, aux, wsum, flag, keys + b);
    return;
  }
  {
    uint64_t tmp[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      const uint32_t idx = threadIdx.x + (uint32_t)i * NT;
      tmp[i] = idx < n ? src[b + idx] : 0ull;
    }
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      const uint32_t idx = threadIdx.x + (uint32_t)i * NT;
      if (idx < n) A[padi<KMAX>(idx)] = tmp[i];
    }
  }
  __syncthreads();
  if (n > 1) reg_sort<KMAX>(A, n, id_bits, cnt, wsum, flag);
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    const uint32_t idx = threadIdx.x + (uint32_t)i * NT;
    if (idx < n) keys[b + idx] = A[padi<KMAX>(idx)];
  }
}


// ------------------------------------------------------------------------------------
// K6/K7 shared structure. A 16x16 tile = 4 waves; wave w owns the 8x8 sub-tile
// (w & 1, w >> 1), lane l its pixel (l & 7, l >> 3). The workgroup stages 256 list
// entries at a time in LDS (one coalesced key + record read per entry); every entry gets a
// 4-bit mask of the sub-tiles its alpha >= 1/255 ellipse can reach (conservative bounding
// box of {d : d^T Q d <= 2 ln(255 o)}, Q = conic), and each wave composites only the entries
// of its mask, in list order. Culled entries would have been skipped by the per-pixel test
// (power > 0 or alpha < 1/255) for every pixel of that sub-tile, so outputs are those of the
// uncull loop; positions in the list are kept so n_contrib keeps its meaning.
constexpr int SUB = 8;

__device__ __forceinline__ float gauss_weight(float power) { return __expf(power); }

// The compositing loops evaluate the Gaussian falloff in base 2 with the conic pre-scaled
// once per staged entry: p2 = log2(e) * power = A dx^2 + C dy^2 + B dx dy with
// A = -0.5 log2(e) a, C = -0.5 log2(e) c, B = -log2(e) b, and G = 2^p2 (one v_exp_f32),
// p2 itself as a polynomial in the pixel's sub-tile offset (fall_poly / fall_p2 below).
constexpr float kLog2e = 1.4426950408889634f;
__device__ __forceinline__ float4 scaled_conic_q(float4 q) {  // (x, y, a, b) -> (x, y, A, B)
  return make_float4(q.x, q.y, -0.5f * kLog2e * q.z, -kLog2e * q.w);
}

// Can the alpha >= 1/255 region of a Gaussian reach any pixel centre of the 8x8 sub-tile
// [x0, x0 + 7] x [y0, y0 + 7]? Exact for the continuous box (conservative for the pixel
// centres in it): with Q(d) = a dx^2 + 2b dx dy + c dy^2 (the conic; power = -Q/2) and
// alpha = min(.99, o e^power), alpha >= 1/255 needs Q(d) <= t2 = 2 ln(255 o). Q is convex,
// so its minimum over the box is 0 when the centre is inside, else on one of the 4 edges,
// where it is a clamped 1-D quadratic. The margin absorbs the rounding of the compositing
// arithmetic, so the entries dropped here are exactly ones the per-pixel test would skip.
// Degenerate / NaN conics are kept.
__device__ __forceinline__ bool rect_hit(float4 q, float4 r, float x0, float y0, float x1, float y1) {
  const float op = r.y;
  if (!(op >= 1.0f / 255.0f)) return false;
  const float a = q.z, b = q.w, c = r.x;
  const float t2 = 2.0f * __logf(255.0f * op) * 1.002f + 0.02f;
  const float lx = x0 - q.x, hx = x1 - q.x;  // box relative to the centre
  const float ly = y0 - q.y, hy = y1 - q.y;
  if (!(a > 0.f && c > 0.f && a * c - b * b > 0.f)) return true;
  if (lx <= 0.f && hx >= 0.f && ly <= 0.f && hy >= 0.f) return true;
  // the clamped 1-D minimiser only has to be a point of the edge: with the hardware
  // reciprocal (1 ulp) it moves by ~1e-7 relative, which changes Q there to second order
  const float ia = __builtin_amdgcn_rcpf(a), ic = __builtin_amdgcn_rcpf(c);
  float m = 3.4e38f;
  // edges x = const
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float dx = k ? hx : lx;
    const float dy = fminf(fmaxf(-b * dx * ic, ly), hy);
    m = fminf(m, a * dx * dx + 2.f * b * dx * dy + c * dy * dy);
  }
  // edges y = const
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float dy = k ? hy : ly;
    const float dx = fminf(fmaxf(-b * dy * ia, lx), hx);
    m = fminf(m, a * dx * dx + 2.f * b * dx * dy + c * dy * dy);
  }
  return !(m > t2);
}

// Bounding box (pixel centres) of the wave's still-live pixels (lane = 8 * row + col of the
// 8x8 sub-tile at (fx0, fy0)); live != 0. Entries that cannot reach it would only meet
// pixels that have stopped (or lie outside the image) and change nothing there.
__device__ __forceinline__ void live_rect(uint64_t live, float fx0, float fy0, float& x0, float& y0, float& x1,
                                          float& y1) {
  uint64_t cols = live | (live >> 32);
  cols |= cols >> 16;
  cols |= cols >> 8;
  const uint32_t cb = (uint32_t)cols & 0xFFu;
  y0 = fy0 + (float)(__builtin_ctzll(live) >> 3);
  y1 = fy0 + (float)((63 - __builtin_clzll(live)) >> 3);
  x0 = fx0 + (float)__builtin_ctz(cb);
  x1 = fx0 + (float)(31 - __builtin_clz(cb));
}

constexpr int CH = 64;  // list entries per chunk (one per lane)
// Chunks whose records a wave gathers in one batch before compositing. A record gather is a
// random read that mostly hits the MALL (the views' geometry does not fit one XCD's L2), and a
// wave walks ~160 entries (p99 ~280, 3-5 chunks) of its tile at config B, so with only the
// next chunk prefetched the walk was a chain of one memory round trip per chunk. Two chunks
// (then one ahead): the round-3 A/B at 16 scenes per launch measured PD = 4 / 3 / 2 / 1 at
// 0.307 / 0.296 / 0.291 / 0.294 ms per sort_render launch and config C 3.22 / 3.19 / 3.17 /
// 3.22 ms (fewer live registers at 5 waves per EU outweigh the deeper batch).
constexpr int PD = 2;
typedef float f2v __attribute__((ext_vector_type(2)));
// The falloff as a polynomial in the pixel's offset (u, v) from its 8x8 sub-tile's centre
// (cx, cy) = (x0 + 3.5, y0 + 3.5): with X = x - cx, Y = y - cy (the Gaussian's centre),
//   p2 = A dx^2 + C dy^2 + B dx dy  (dx = X - u, dy = Y - v)
//      = F + D u + E v + A u^2 + C v^2 + B u v,
//   F = A X^2 + C Y^2 + B X Y,  D = -2 A X - B Y,  E = -2 C Y - B X.
// A wave stages (F, D, E) once per entry; per pixel the falloff is then 5 FMAs on per-lane
// constants (u, v, u^2, v^2, u v are exact: halves in [-3.5, 3.5]) instead of 8 operations.
// The forward, the backward and the tail check all evaluate exactly this sequence, so their
// skip decisions agree; the culling tests (rect_hit, tile_reach) keep margins far above its
// rounding (|terms| of a reachable entry are O(10), so errors are ~1e-6 in p2).
struct PixUV {
  float u, v, uu, vv, uv;
};
__device__ __forceinline__ PixUV pix_uv(int px, int py, float fx0, float fy0) {
  PixUV p;
  p.u = (float)px - (fx0 + 3.5f);
  p.v = (float)py - (fy0 + 3.5f);
  p.uu = p.u * p.u;
  p.vv = p.v * p.v;
  p.uv = p.u * p.v;
  return p;
}
struct FallPoly {
  float F, D, E;
};
__device__ __forceinline__ FallPoly fall_poly(float x, float y, float A, float B, float C, float fx0, float fy0) {
  const float X = x - (fx0 + 3.5f), Y = y - (fy0 + 3.5f);
  FallPoly f;
  f.F = fmaf(A * X, X, fmaf(C * Y, Y, B * X * Y));
  f.D = fmaf(-2.0f * A, X, -(B * Y));
  f.E = fmaf(-2.0f * C, Y, -(B * X));
  return f;
}
// The reference skips a pixel when power > 0, which for a positive-definite conic happens only
// through its own rounding; the polynomial's absolute rounding near the centre is up to
// ~2e-5 (terms of magnitude <= ~100), so "power <= 0" is tested as p2 <= kP2Max: every
// positive-definite Gaussian still blends at its centre pixel (G = 2^p2 <= 1.00007 there).
constexpr float kP2Max = 1e-4f;
// Positive-definite scaled conic (p2 = A u^2 + B u v + C v^2 + ...: A < 0, 4 A C > B^2). For
// such an entry the true p2 is <= 0 everywhere, so "power > 0" can only come from rounding
// (of the polynomial form: needle Gaussians far from their centre) and the skip test is
// alpha >= 1/255 alone. Only an indefinite conic (from a covariance that is not PSD: the +0.3
// dilation makes every PSD input definite) keeps the p2 <= kP2Max test. Forward, backward
// and the tail check evaluate this same expression on the same staged floats, so their
// decisions agree.
__device__ __forceinline__ bool conic_pd(float A, float B, float C) { return A < 0.f && 4.f * A * C > B * B; }
__device__ __forceinline__ float fall_p2(const PixUV& p, float F, float D, float E, float A, float B, float C) {
  return fmaf(A, p.uu, fmaf(C, p.vv, fmaf(B, p.uv, fmaf(D, p.u, fmaf(E, p.v, F)))));
}
// Two consecutive list entries with their fields interleaved, so the falloff of both runs
// as packed FP32 (v_pk_fma/mul) with no operand shuffling; per-element results are the same
// IEEE operations as fall_p2 (the backward's decisions agree).
struct __align__(16) PairRec {
  f2v F, D, E, A, C, B;  // falloff fields of entries 0 and 1, interleaved (packed math); F holds
                         // F + lo, lo = log2(opacity) (pair_put)
  f2v b;
  f2v rg[2];             // (r, g) of entry j: one packed FMA into the pixel's (R, G)
  f2v o;                 // lo (the power test of an indefinite conic only): last, so the common
                         // loop reads the fields before it as whole 16-byte vectors
};
// A wave's staged chunk: up to CH kept entries + 8 pads as field-interleaved pairs (80 B: a
// 20-word stride, so the 32 lanes' stores of one field hit 2-way at most), and beside them
// each entry's list position (read once per chunk by a backward-bound forward: n_contrib).
struct __align__(16) WaveList {
  PairRec rec[(CH + 8) / 2];
  uint32_t pos[CH + 8];
};
// the pixel terms stay scalars; the packed FMAs broadcast them (op_sel), no duplicated registers
typedef PixUV PixUV2;
__device__ __forceinline__ PixUV2 pix_uv2(const PixUV& p) { return p; }
__device__ __forceinline__ f2v fall_p2x2(const PixUV2& p, const PairRec& P) {
  const f2v t0 = __builtin_elementwise_fma(P.E, f2v{p.v, p.v}, P.F);
  const f2v t1 = __builtin_elementwise_fma(P.D, f2v{p.u, p.u}, t0);
  const f2v t2 = __builtin_elementwise_fma(P.B, f2v{p.uv, p.uv}, t1);
  const f2v t3 = __builtin_elementwise_fma(P.C, f2v{p.vv, p.vv}, t2);
  return __builtin_elementwise_fma(P.A, f2v{p.uu, p.uu}, t3);
}
// The opacity folded into the falloff: with lo = log2(o), exp2(p2 + lo) = o G, so a pixel's
// o G is one v_exp of the polynomial whose constant term is F + lo (one multiply fewer per
// (pixel, entry)); o = 0 gives lo = -inf, o G = 0. The backward stages F + lo with the same
// two operations (fall_lo), so both evaluate the same alpha.
__device__ __forceinline__ float fall_lo(float o) { return o > 0.f ? __builtin_amdgcn_logf(o) : -__builtin_inff(); }
// stage one entry (centre x, y; scaled conic A, B, C) as element k of the wave's pair list
__device__ __forceinline__ void pair_put(WaveList* wl, int k, float x, float y, float A, float C, float B, float o,
                                         float r, float g, float b, uint32_t pos, float fx0, float fy0) {
  PairRec& d = wl->rec[k >> 1];
  const int j = k & 1;
  const FallPoly f = fall_poly(x, y, A, B, C, fx0, fy0);
  const float lo = fall_lo(o);
  d.F[j] = f.F + lo; d.D[j] = f.D; d.E[j] = f.E; d.A[j] = A; d.C[j] = C; d.B[j] = B; d.o[j] = lo;
  d.rg[j] = f2v{r, g}; d.b[j] = b;
  wl->pos[k] = pos;
}
__device__ __forceinline__ void pair_pad(WaveList* wl, int k) {  // opacity 0: alpha 0, never blends
  PairRec& d = wl->rec[k >> 1];
  const int j = k & 1;
  constexpr float ninf = -__builtin_inff();
  d.F[j] = ninf; d.D[j] = 0.f; d.E[j] = 0.f; d.A[j] = 0.f; d.C[j] = 0.f; d.B[j] = 0.f; d.o[j] = ninf;
  d.rg[j] = f2v{0.f, 0.f}; d.b[j] = 0.f;
}
// Front-to-back step over two entries. A pixel's state is its transmittance with the sign
// as the stop flag (Tr < 0: stopped or outside the image, |Tr| the final T), so the chain
// T -> test T -> stop -> T is vector compares and selects (VCC) only: no per-pixel lane mask
// round-trips through SALU ops at every entry. Per entry, as the reference: skip
// unless power <= 0 (conic_pd, or p2 <= kP2Max) and alpha = min(.99, o G) >= 1/255 (PD: a
// chunk whose entries all have definite conics tests alpha alone); test T = T (1 - alpha); stop
// (without blending) when test T < 1e-4; else colour += rgb alpha T, T = test T, last =
// position. A skipped entry gets alpha 0, which leaves T bit-identical (T * 1) and adds +0
// colour; a stopped pixel fails the stop test at every later entry (T (1 - alpha) <= 0).
// LAST: track the chunk index of the last blended entry (its list position, n_contrib, which
// only a backward reads, is looked up once per chunk).
template <bool LAST, bool PD>
__device__ __forceinline__ void composite_pair(const PairRec& P, const PixUV2& pp, float& Tr, f2v& C01, float& C2,
                                               int& lastk, int k0) {
  const f2v p2o = fall_p2x2(pp, P);  // p2 + lo
  f2v alpha;
  alpha.x = fminf(0.99f, __builtin_amdgcn_exp2f(p2o.x));
  alpha.y = fminf(0.99f, __builtin_amdgcn_exp2f(p2o.y));
  f2v a;
  if (PD) {
    a.x = alpha.x >= 1.0f / 255.0f ? alpha.x : 0.f;
    a.y = alpha.y >= 1.0f / 255.0f ? alpha.y : 0.f;
  } else {
    // ok <=> min(thr - p2o, alpha - 1/255) >= 0 with thr = kP2Max + lo (each difference has
    // the exact sign of its comparison); the power test only for an indefinite conic
    const f2v np2 = (f2v{kP2Max, kP2Max} + P.o) - p2o;
    const f2v over = alpha - f2v{1.0f / 255.0f, 1.0f / 255.0f};
    a.x = (conic_pd(P.A.x, P.B.x, P.C.x) ? over.x : fminf(np2.x, over.x)) >= 0.f ? alpha.x : 0.f;
    a.y = (conic_pd(P.A.y, P.B.y, P.C.y) ? over.y : fminf(np2.y, over.y)) >= 0.f ? alpha.y : 0.f;
  }
  const f2v om = f2v{1.f, 1.f} - a;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float testT = Tr * om[j];
    const bool stop = testT < 0.0001f;  // always once stopped (test T <= 0)
    const float wgt = stop ? 0.f : a[j] * Tr;
    const f2v rg = P.rg[j];
    f2v w2;
    w2.x = wgt;
    w2.y = wgt;
    C01 = __builtin_elementwise_fma(rg, w2, C01);
    C2 = fmaf(P.b[j], wgt, C2);
    Tr = stop ? -fabsf(Tr) : testT;
    if (LAST) lastk = wgt > 0.f ? k0 + j : lastk;  // blended <=> wgt > 0 (alpha >= 1/255, T >= 1e-4)
  }
}

// Tail check for prefix-sorted segments: the keys in [b, e) are all deeper than the sorted
// prefix but unordered. Compositing them in depth order changes a pixel only if one of them
// passes the per-pixel test (power <= 0, alpha >= 1/255) while the pixel is still live, so
// when none does the prefix alone gives the exact result. Returns (wave-uniform) whether
// one does.
__device__ bool tail_reaches_live(const float* __restrict__ gv, const uint64_t* __restrict__ keys, uint32_t b,
                                  uint32_t e, float fx0, float fy0, const PixUV2& pp, bool alive, WaveList* plist,
                                  uint64_t lt, int lane, uint32_t gmax) {
  uint32_t nid = b + lane < e ? min((uint32_t)keys[b + lane], gmax) : 0xffffffffu;
  for (uint32_t base = b; base < e; base += 64) {
    const uint64_t live = __ballot(alive);
    if (!live) break;
    float lx0, ly0, lx1, ly1;
    live_rect(live, fx0, fy0, lx0, ly0, lx1, ly1);
    const uint32_t id = nid;
    nid = base + 64 + lane < e ? min((uint32_t)keys[base + 64 + lane], gmax) : 0xffffffffu;
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f), r = q;
    if (id != 0xffffffffu) {
      const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)id * GS);
      q = rec[0];
      r = rec[1];
    }
    const bool mine = id != 0xffffffffu && rect_hit(q, r, lx0, ly0, lx1, ly1);
    const uint64_t bal = __ballot(mine);
    if (mine) {
      const float4 sq = scaled_conic_q(q);
      pair_put(plist, __popcll(bal & lt), sq.x, sq.y, sq.z, -0.5f * kLog2e * r.x, sq.w, r.y, 0.f, 0.f, 0.f, 0u, fx0,
               fy0);
    }
    const int cnt = __popcll(bal);
    if (lane < 2) pair_pad(plist, cnt + lane);
    __builtin_amdgcn_wave_barrier();
    bool hit = false;
    for (int k = 0; k < cnt; k += 2) {
      const PairRec& P = plist->rec[k >> 1];
      const f2v p2o = fall_p2x2(pp, P);  // p2 + lo (pair_put)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float alpha = fminf(0.99f, __builtin_amdgcn_exp2f(p2o[j]));
        hit |= (conic_pd(P.A[j], P.B[j], P.C[j]) || p2o[j] <= kP2Max + P.o[j]) && alpha >= 1.0f / 255.0f;
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (__any(hit && alive)) return true;
  }
  return false;
}

// One chunk of the walk: keep the entries of [base, base + CH) (this lane's record q, r, b)
// whose alpha >= 1/255 region reaches the live pixels' box in the wave's LDS list (ballot
// compaction, list order kept, entry pairs field-interleaved for packed math, 8 zero-opacity
// pad entries after the end), then composite that list four entries per step with the next
// four read ahead.
template <bool LAST>
__device__ __forceinline__ void composite_chunk(uint32_t base, uint32_t start, uint32_t end, float4 q, float4 r,
                                                float b, float lx0, float ly0, float lx1, float ly1, float fx0,
                                                float fy0, const PixUV2& pp, int lane, uint64_t lt, WaveList* plist,
                                                float& Tr, f2v& C01, float& C2, uint32_t& last) {
  const uint32_t e = base + lane;
  const bool mine = e < end && rect_hit(q, r, lx0, ly0, lx1, ly1);
  const uint64_t bal = __ballot(mine);
  bool indef = false;  // an indefinite conic in the chunk: the loop with the power test
  if (mine) {
    const float4 sq = scaled_conic_q(q);  // (x, y, A, B)
    const float C = -0.5f * kLog2e * r.x;
    indef = !conic_pd(sq.z, sq.w, C);
    pair_put(plist, __popcll(bal & lt), sq.x, sq.y, sq.z, C, sq.w, r.y, r.z, r.w, b, e - start + 1u, fx0, fy0);
  }
  const int cnt = __popcll(bal);
  if (lane < 8) pair_pad(plist, cnt + lane);  // pad up to 8 entries (never blend)
  __builtin_amdgcn_wave_barrier();
  const PairRec* pl = plist->rec;
  int lastk = -1;  // LAST: index of the chunk's last blended entry
  // four entries per step (the pads make pairs k/2, k/2 + 1 valid reads)
  if (!__any(indef)) {
    for (int k = 0; k < cnt; k += 4) {
      const PairRec a0 = pl[k >> 1], a1 = pl[(k >> 1) + 1];
      composite_pair<LAST, true>(a0, pp, Tr, C01, C2, lastk, k);
      composite_pair<LAST, true>(a1, pp, Tr, C01, C2, lastk, k + 2);
      if (!__any(Tr > 0.f)) break;
    }
  } else {
    for (int k = 0; k < cnt; k += 4) {
      const PairRec a0 = pl[k >> 1], a1 = pl[(k >> 1) + 1];
      composite_pair<LAST, false>(a0, pp, Tr, C01, C2, lastk, k);
      composite_pair<LAST, false>(a1, pp, Tr, C01, C2, lastk, k + 2);
      if (!__any(Tr > 0.f)) break;
    }
  }
  if (LAST && lastk >= 0) last = plist->pos[lastk];
  __builtin_amdgcn_wave_barrier();  // list reads of this chunk before the next chunk's writes
}

// K6 core: one wave composites its 8x8 sub-tile (pixel (px, py) per lane) front to back
// over the sorted entries [start, end) of its tile, key_at(e) giving entry e's Gaussian id
// (from HBM keys, or from the fused sort's LDS), CH entries at a time (composite_chunk), and
// returns as soon as its 64 pixels have terminated. The records of the first PD chunks are
// gathered up front in one batch (straight-line code, so each chunk waits only for its own
// loads); past them the walk keeps the next chunk's records and the keys of the chunk after
// in flight.
template <bool LAST, typename KeyAt>
__device__ __forceinline__ void composite_walk(KeyAt key_at, uint32_t start, uint32_t end, const float* __restrict__ gv,
                                               float fx0, float fy0, const PixUV2& pp, int lane, uint64_t lt,
                                               WaveList* plist, float& Tr, f2v& C01, float& C2, uint32_t& last) {
  if (start >= end) return;
  // unconditional key reads (clamped index), so HBM key loads need no wait each; entries past
  // the end read record 0 (a valid address) and are masked by the chunk's e < end test
  auto id_of = [&](uint32_t e) -> uint32_t {
    const uint32_t k = key_at(min(e, end - 1u));
    return e < end ? k : 0u;
  };
  float4 q[PD], r[PD];
  float b[PD];
  uint32_t ids[PD];
#pragma unroll
  for (int s = 0; s < PD; ++s) ids[s] = id_of(start + s * CH + lane);  // HBM keys: one batch too
#pragma unroll
  for (int s = 0; s < PD; ++s) {
    const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)ids[s] * GS);
    q[s] = rec[0];
    r[s] = rec[1];
    b[s] = rec[2].x;
  }
  uint32_t nid = id_of(start + PD * CH + lane);
#pragma unroll
  for (int s = 0; s < PD; ++s) {
    const uint32_t base = start + s * CH;
    if (base >= end) return;
    const uint64_t live = __ballot(Tr > 0.f);
    if (!live) return;
    float lx0, ly0, lx1, ly1;
    live_rect(live, fx0, fy0, lx0, ly0, lx1, ly1);
    composite_chunk<LAST>(base, start, end, q[s], r[s], b[s], lx0, ly0, lx1, ly1, fx0, fy0, pp, lane, lt, plist, Tr,
                          C01, C2, last);
  }
  float4 cq = make_float4(0.f, 0.f, 0.f, 0.f), cr = cq;
  float cb = 0.f;
  {
    const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)nid * GS);
    cq = rec[0];
    cr = rec[1];
    cb = rec[2].x;
  }
  nid = id_of(start + (PD + 1) * CH + lane);
  for (uint32_t base = start + PD * CH; base < end; base += CH) {
    const uint64_t live = __ballot(Tr > 0.f);
    if (!live) break;
    float lx0, ly0, lx1, ly1;
    live_rect(live, fx0, fy0, lx0, ly0, lx1, ly1);
    const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)nid * GS);
    const float4 nq = rec[0], nr = rec[1];
    const float nb = rec[2].x;
    nid = id_of(base + 2 * CH + lane);
    composite_chunk<LAST>(base, start, end, cq, cr, cb, lx0, ly0, lx1, ly1, fx0, fy0, pp, lane, lt, plist, Tr, C01, C2,
                          last);
    cq = nq;
    cr = nr;
    cb = nb;
  }
}

// composite_walk with the kernels' state: alive (the pixel lies in the image and has not
// stopped) and T = the pixel's transmittance (the final T once stopped).
template <bool LAST, typename KeyAt>
__device__ __forceinline__ void composite_tile(KeyAt key_at, uint32_t start, uint32_t end, const float* __restrict__ gv,
                                               float fx0, float fy0, const PixUV2& pp, int lane, uint64_t lt,
                                               WaveList* plist, float& Tr, f2v& C01, float& C2, uint32_t& last,
                                               bool& alive) {
  Tr = alive ? Tr : -Tr;
  composite_walk<LAST>(key_at, start, end, gv, fx0, fy0, pp, lane, lt, plist, Tr, C01, C2, last);
  alive = Tr > 0.f;
  Tr = fabsf(Tr);
}

__device__ __forceinline__ void store_pixel(float* __restrict__ out, float* __restrict__ finalT,
                                            uint32_t* __restrict__ ncontrib, const float* bg, int v, int H, int W,
                                            int px, int py, float Tr, f2v C01, float C2, uint32_t last) {
  const size_t HW = (size_t)H * W;
  const size_t pix = (size_t)py * W + px;
  finalT[v * HW + pix] = Tr;
  if (ncontrib) ncontrib[v * HW + pix] = last;
  out[(size_t)v * 3 * HW + pix] = C01.x + Tr * bg[0];
  out[(size_t)v * 3 * HW + HW + pix] = C01.y + Tr * bg[1];
  out[(size_t)v * 3 * HW + 2 * HW + pix] = C2 + Tr * bg[2];
}

// Tile of this compositing workgroup (grid = (gx, gy, V)). The dispatcher places workgroups
// L, L + 256, L + 512, ... (linear ids) on one CU (measured: round-robin over the 8 XCDs, then
// over an XCD's 32 CUs), i.e. at config B the same tile position of the 3 views, and centre
// tiles carry ~1.8x the entries of border ones. Shifting each view's tile grid by a third of
// it along both axes gives a CU tiles from different parts of the image, so the CUs' loads
// even out (tools/sr_timing.py: per-CU finish times).
__device__ __forceinline__ void tile_of(int gx, int gy, int& tx, int& ty) {
  const int v = blockIdx.z;
  tx = (int)((blockIdx.x + (unsigned)v * (unsigned)((gx + 2) / 3)) % (unsigned)gx);
  ty = (int)((blockIdx.y + (unsigned)v * (unsigned)((gy + 2) / 3)) % (unsigned)gy);
}

// XCD-contiguous tiles for grids of (gx, gy, V) workgroups: the dispatcher deals linear
// workgroup ids round-robin to the 8 XCDs, so XCD x takes ids x, x + 8, ...; they are given
// the contiguous range [x * per, (x + 1) * per) of (view, row, column) tiles, so a view's
// neighbouring tiles — which gather the same Gaussians' records — run on one XCD, close in
// time, and find them in its L2. Columns are skewed per row (an XCD deals its range over its
// 32 CUs in turn: without the skew CU c would get one column of every other row, centre
// columns carrying ~1.8x the entries of border ones). Needs V T % 8 == 0 (else the plain
// mapping); returns the view.
__device__ __forceinline__ int tile_xcd(int gx, int gy, int& tx, int& ty) {
  const int T = gx * gy, total = T * (int)gridDim.z;
  if (total & 7) {
    tile_of(gx, gy, tx, ty);
    return blockIdx.z;
  }
  const int L = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
  const int item = (L & 7) * (total >> 3) + (L >> 3);
  const int v = item / T, r = item - v * T;
  ty = r / gx;
  tx = (r - ty * gx + 3 * ty) % gx;
  return v;
}

// K6: front-to-back compositing. grid = (gx, gy, V), block = 256 = 4 independent waves;
// wave w owns the 8x8 sub-tile (w & 1, w >> 1) of the tile (composite_tile). There is no
// workgroup barrier; the waves of a workgroup share the tile's keys/records through L1. A
// stopped pixel keeps its final T (alive is a lane mask).
// One tile of K6 (k_render_fwd's body; also run by k_render_flagged). V: the launch's views.
__device__ __forceinline__ void render_fwd_tile(int v, int tx, int ty, int V, int G, int H, int W, int gx, int T,
                                                const dsr_camera* __restrict__ cams, const float* __restrict__ geom,
                                                const uint32_t* __restrict__ seg_start,
                                                const uint32_t* __restrict__ seg_count, uint32_t stride,
                                                const uint64_t* __restrict__ keys,
                                                const uint32_t* __restrict__ seg_sorted,
                                                uint32_t* __restrict__ seg_overflow, float* __restrict__ out,
                                                float* __restrict__ finalT, uint32_t* __restrict__ ncontrib,
                                                WaveList* l_pair) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int sx0 = tx * BX + (w & 1) * SUB, sy0 = ty * BY + (w >> 1) * SUB;
  const int px = sx0 + (lane & (SUB - 1));
  const int py = sy0 + (lane >> 3);
  const bool inside = px < W && py < H;
  const int seg = v * T + ty * gx + tx;
  uint32_t start, end;
  seg_bounds(seg_start, seg_count, stride, seg, start, end);
  const uint32_t tail_end = end;  // [end, tail_end): unsorted tail (prefix-sorted segments)
  if (seg_sorted) end = start + min(seg_sorted[seg], end - start);
  // depth-cut binning: entries past `end` were never written (all deeper than the written ones)
  const bool absent_tail = stride == kSegEnds && seg_overflow != nullptr && end < seg_start[seg + 1];
  const float fx0 = (float)sx0, fy0 = (float)sy0;
  const float* gv = geom + (size_t)v * G * GS;
  const uint64_t lt = dsplat::lanemask_lt(lane);
  WaveList* plist = &l_pair[w];
  const PixUV2 pp = pix_uv2(pix_uv(px, py, fx0, fy0));
  f2v C01 = {0.f, 0.f};
  float Tr = 1.0f, C2 = 0.f;
  bool alive = inside;
  uint32_t last = 0;
  const uint32_t gmax = (uint32_t)G - 1u;  // ids are clamped: a corrupt key reads a valid record, never faults
  composite_tile<true>([&](uint32_t e) { return min((uint32_t)keys[e], gmax); }, start, end, gv, fx0, fy0, pp, lane, lt, plist,
                       Tr, C01, C2, last, alive);
  bool void_tile = false;  // wave-uniform
  if (absent_tail)
    void_tile = __any(alive);  // a pixel still live at the end of the written part: the rest may blend
  else if (end < tail_end)
    void_tile = tail_reaches_live(gv, keys, end, tail_end, fx0, fy0, pp, alive, plist, lt, lane, gmax);
  if (void_tile && lane == 0) {  // the tile's output is void: completed, sorted and re-rendered by the caller
    seg_overflow[seg] = 1u;
    seg_overflow[(size_t)V * T] = 1u;  // any-flag
    if (absent_tail) {  // depth cut: also flag the tile's super-block (the tail scatter's pre-test)
      const int sb = cut_superblock(gx, T / gx), sbl = __builtin_ctz((unsigned)sb);
      const int nsx = (gx + sb - 1) / sb, nsb = nsx * ((T / gx + sb - 1) / sb);
      seg_overflow[(size_t)V * T + 1 + (size_t)v * nsb + (ty >> sbl) * nsx + (tx >> sbl)] = 1u;
    }
  }
  if (inside) store_pixel(out, finalT, ncontrib, cams[v].bg, v, H, W, px, py, Tr, C01, C2, last);
}

__global__ __launch_bounds__(NT) void k_render_fwd(int G, int H, int W, int gx, int T,
                                                   const dsr_camera* __restrict__ cams,
                                                   const float* __restrict__ geom,
                                                   const uint32_t* __restrict__ seg_start,
                                                   const uint32_t* __restrict__ seg_count, uint32_t stride,
                                                   const uint64_t* __restrict__ keys,
                                                   const uint32_t* __restrict__ seg_sorted,
                                                   uint32_t* __restrict__ seg_overflow,
                                                   float* __restrict__ out, float* __restrict__ finalT,
                                                   uint32_t* __restrict__ ncontrib) {
  __shared__ WaveList l_pair[4];
  int tx, ty;
  const int v = tile_xcd(gx, T / gx, tx, ty);  // kbench: 3 views -4..-6 %, 64 views level
  render_fwd_tile(v, tx, ty, gridDim.z, G, H, W, gx, T, cams, geom, seg_start, seg_count, stride, keys, seg_sorted,
                  seg_overflow, out, finalT, ncontrib, l_pair);
}
// The tail pass's re-render (dsr_render_fwd with seg_filter): a persistent grid walks the
// (view, tile) segments and renders the flagged ones; with nothing flagged (any-flag word
// seg_filter[V T] = 0) it leaves at once instead of dispatching a workgroup per tile (~49 us
// per config-E launch, round 5).
__global__ __launch_bounds__(NT) void k_render_flagged(int V, int G, int H, int W, int gx, int T,
                                                       const dsr_camera* __restrict__ cams,
                                                       const float* __restrict__ geom,
                                                       const uint32_t* __restrict__ seg_start,
                                                       const uint32_t* __restrict__ seg_count, uint32_t stride,
                                                       const uint64_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ seg_filter,
                                                       float* __restrict__ out, float* __restrict__ finalT,
                                                       uint32_t* __restrict__ ncontrib) {
  __shared__ WaveList l_pair[4];
  const int nseg = V * T;
  if (seg_filter[nseg] == 0u) return;  // uniform
  for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    if (seg_filter[seg] == 0u) continue;  // uniform
    const int v = seg / T, t = seg - v * T, ty = t / gx, tx = t - ty * gx;
    render_fwd_tile(v, tx, ty, V, G, H, W, gx, T, cams, geom, seg_start, seg_count, stride, keys, nullptr, nullptr,
                    out, finalT, ncontrib, l_pair);
    __syncthreads();  // the wave lists are reused by the next flagged tile
  }
}

// K4 + K6 fused: one workgroup per tile sorts the tile's keys in LDS (count_sort) and its 4
// waves composite straight from the sorted LDS copy (their pair lists reuse the sort's
// counter area). The sorted keys go back to HBM only when the backward needs them
// (write_keys), the render never re-reads keys from HBM, and the sort and compositing phases
// of different tiles overlap inside one launch. A segment above the LDS capacity is sorted
// through HBM (scratch) by the same workgroup and composited from there.
// LDS of k_sort_render<KMAX, ·, NBL>: the padded key array, then one area shared by the
// sort's counters (u16 bins / LSD counters / HBM-path histogram) and, after the sort, the 4
// waves' pair lists, then the wave sums and flag.
template <int NBL>
constexpr int sort_render_aux_words() {
  constexpr int pl = (int)(sizeof(WaveList) * 4 / 4);
  return sort_cnt_words<NT, NBL>() > pl ? sort_cnt_words<NT, NBL>() : pl;
}
template <int KMAX, int NBL>
constexpr size_t sort_render_lds_bytes() {
  return (size_t)(NT * KMAX + NT) * 8 + (size_t)sort_render_aux_words<NBL>() * 4 + 64 * 4;
}

// ---- bounded-capacity segments ---------------------------------------------------------
// dsr_project_bin_cameras with seg_capacity < G keeps only the first `capacity` entries a tile
// receives (the count goes on). Such a tile's list is rebuilt from the view's geometry records:
// the binning test is a function of one record, so evaluating it for every Gaussian of the
// view gives the tile's full entry set. record_hits_tile is k_project_emit's keep test (the
// 3-sigma rect; with EXACT the alpha >= 1/255 rect and tile_reach) on the stored fields.
__device__ __forceinline__ bool record_hits_tile(float4 q, float4 rr, float4 z, int gx, int gy, int tx, int ty,
                                                 bool exact) {
  const int r = __float_as_int(z.z);  // rec[10]
  if (r <= 0) return false;
  int x0, y0, x1, y1;
  tile_rect(q.x, q.y, r, gx, gy, x0, y0, x1, y1);
  if (!exact) return tx >= x0 && tx < x1 && ty >= y0 && ty < y1;
  const float rec[6] = {q.x, q.y, q.z, q.w, rr.x, rr.y};
  const TileEll e = tile_ell(rec, r);
  tile_rect_alpha(e, x0, y0, x1, y1);
  if (!(tx >= x0 && tx < x1 && ty >= y0 && ty < y1)) return false;
  return tile_reach(e, tx, ty);
}

// Rank selection over a per-digit histogram (NB u32 bins in LDS, NB / NT per thread): the
// digit d holding the r-th candidate (1-based) and the number of candidates in lower digits;
// d = 0xffffffff when fewer than r candidates exist. Block-uniform results (flag[0..1]).
template <int NB>
__device__ __forceinline__ void hist_select(const uint32_t* hist, uint32_t r, uint32_t* wsum, uint32_t* flag,
                                            uint32_t& d, uint32_t& below) {
  constexpr int BPT = NB / NT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t c[BPT], tot = 0;
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    c[i] = hist[tid * BPT + i];
    tot += c[i];
  }
  const uint32_t incl = dsplat::wave_incl_add_dpp(tot);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t off = incl - tot;
  for (int k = 0; k < w; ++k) off += wsum[k];
  if (r > off && r <= off + tot) {
    uint32_t acc = off;
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      if (r > acc && r <= acc + c[i]) {
        flag[0] = (uint32_t)(tid * BPT + i);
        flag[1] = acc;
      }
      acc += c[i];
    }
  }
  __syncthreads();
  d = flag[0];
  below = flag[1];
  __syncthreads();
}

// Composite a rebuilt tile: its entries (keys above `lo`, in key order) are taken in windows
// of at most the LDS capacity — the window's last key found by a radix select over 11-bit
// digits of the 64-bit keys (one pass over the view's records per digit; a pass stops the
// descent once half a window is certain) — each window sorted in LDS (count_sort) and
// composited before the next, until every pixel has stopped or the list is exhausted.
// Entries are blended in exactly the full list's order, so the image equals the unbounded
// layout's. LAST: n_contrib positions count from the list's start. spill (non-NULL): each
// window's sorted keys are stored at their list positions there — every position below the
// tile's last blended one, which is all the backward reads.
template <int KMAX, bool LAST, int NBL>
__device__ __attribute__((noinline)) void render_rebuilt(int G, int gx, int gy, int tx, int ty, bool exact, const float* __restrict__ gv,
                               uint64_t* A, uint16_t* cnt, uint32_t* wsum, uint32_t* flag, int id_bits, float fx0,
                               float fy0, const PixUV2& pp, int lane, uint64_t lt, WaveList* plist, float& Tr, f2v& C01,
                               float& C2, uint32_t& last, bool& alive, uint64_t* __restrict__ spill) {
  constexpr uint32_t capl = NT * KMAX;
  constexpr int kNB = 2048;  // 11-bit digits
  static_assert((NT * KMAX + NT) * 2 >= kNB, "digit histogram fits the key array");
  uint32_t* hist = reinterpret_cast<uint32_t*>(A);
  const int tid = threadIdx.x;
  auto key_of = [&](uint32_t g, uint64_t& key) -> bool {
    const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)g * GS);
    const float4 q = rec[0], rr = rec[1], z = rec[2];
    if (!record_hits_tile(q, rr, z, gx, gy, tx, ty, exact)) return false;
    key = ((uint64_t)__float_as_uint(z.y) << 32) | g;  // (depth rec[9], id): k_project_emit's key
    return true;
  };
  uint64_t lo = 0ull;  // exclusive: every key is > 0 (depth > 0.2)
  uint32_t base = 0;
  for (;;) {
    uint64_t hi = ~0ull;
    {
      uint64_t prefix = 0ull;
      int pbits = 0;
      uint32_t r = capl, taken = 0;
      for (int shift = 53;; shift = max(shift - 11, 0)) {
        const int width = 64 - pbits - shift;
        for (int i = tid; i < kNB; i += NT) hist[i] = 0u;
        if (tid == 0) flag[0] = 0xffffffffu;
        __syncthreads();
        for (uint32_t g = (uint32_t)tid; g < (uint32_t)G; g += NT) {
          uint64_t key;
          if (!key_of(g, key) || key <= lo) continue;
          if (pbits != 0 && (key >> (64 - pbits)) != prefix) continue;
          atomicAdd(&hist[(uint32_t)(key >> shift) & ((1u << width) - 1u)], 1u);
        }
        __syncthreads();
        uint32_t d, below;
        hist_select<kNB>(hist, r, wsum, flag, d, below);
        if (d == 0xffffffffu) break;  // (level 0 only) the rest of the list fits one window: hi = ~0
        taken += below;
        r -= below;
        const uint64_t cell = (prefix << width) | d;
        if (shift == 0) {  // digits exhausted: the r-th candidate itself closes the window
          hi = cell;
          break;
        }
        if (taken >= capl / 2 && cell != 0ull) {  // every key below digit d: at least half a window
          hi = (cell << shift) - 1ull;
          break;
        }
        prefix = cell;
        pbits += width;
      }
    }
    if (tid == 0) flag[2] = 0u;
    __syncthreads();
    for (uint32_t g = (uint32_t)tid; g < (uint32_t)G; g += NT) {
      uint64_t key;
      if (!key_of(g, key) || key <= lo || key > hi) continue;
      A[padi<KMAX>(atomicAdd(&flag[2], 1u))] = key;
    }
    __syncthreads();
    const uint32_t n = flag[2];
    uint64_t tmp[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      const uint32_t idx = tid + (uint32_t)i * NT;
      tmp[i] = idx < n ? A[padi<KMAX>(idx)] : 0ull;
    }
    __syncthreads();
    if (n > 1) count_sort<KMAX, NT, NBL>(tmp, n, A, id_bits, cnt, wsum, flag);
    if (spill)  // the window's sorted keys at their list positions, for the backward
      for (uint32_t i = tid; i < n; i += NT) spill[base + i] = A[padi<KMAX>(i)];
    uint32_t wl = 0;
    composite_tile<LAST>([&](uint32_t i) { return min((uint32_t)A[padi<KMAX>(i)], (uint32_t)G - 1u); }, 0u, n, gv, fx0,
                         fy0, pp, lane, lt, plist, Tr, C01, C2, wl, alive);
    if (LAST && wl) last = base + wl;
    const bool more = __syncthreads_or(alive);
    if (!more || hi == ~0ull) break;
    lo = hi;
    base += n;
  }
}

template <int KMAX, bool LAST, int NBL, int WPE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) void k_sort_render(
    int G, int H, int W, int gx, int T, const dsr_camera* __restrict__ cams, const float* __restrict__ geom,
    const uint32_t* __restrict__ seg_start, uint32_t* __restrict__ seg_count, uint32_t stride,
    uint64_t* __restrict__ keys, uint64_t* __restrict__ scratch, uint64_t* __restrict__ spill_keys, int id_bits,
    int write_keys, int clear_counts, int exact_rebuild, float* __restrict__ out, float* __restrict__ finalT, uint32_t* __restrict__ ncontrib,
    uint32_t* __restrict__ seg_overflow) {
  constexpr uint32_t cap = NT * KMAX;
  constexpr uint32_t padded = cap + cap / KMAX;
  extern __shared__ __attribute__((aligned(16))) uint64_t s_keys[];
  uint64_t* A = s_keys;
  uint32_t* aux = reinterpret_cast<uint32_t*>(A + padded);
  uint16_t* cnt = reinterpret_cast<uint16_t*>(aux);
  uint32_t* wsum = aux + sort_render_aux_words<NBL>();
  uint32_t* flag = wsum + 16;
  static_assert(NT * 4 <= sort_render_aux_words<NBL>(), "HBM-path radix histogram fits the aux area");
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  int tx, ty;
  const int v = tile_xcd(gx, T / gx, tx, ty);  // kbench: 3 views -4.7 %, 24 / 64 views -0.6 %
  const int seg = v * T + ty * gx + tx;
  if (stride != 0u && stride != kSegEnds && seg_count[seg] > stride) {  // bounded segment that overflowed
    const int sx0 = tx * BX + (w & 1) * SUB, sy0 = ty * BY + (w >> 1) * SUB;
    const int px = sx0 + (lane & (SUB - 1)), py = sy0 + (lane >> 3);
    const bool inside = px < W && py < H;
    const PixUV2 pp = pix_uv2(pix_uv(px, py, (float)sx0, (float)sy0));
    f2v C01 = {0.f, 0.f};
    float Tr = 1.0f, C2 = 0.f;
    bool alive = inside;
    uint32_t last = 0;
    render_rebuilt<KMAX, LAST, NBL>(G, gx, T / gx, tx, ty, exact_rebuild != 0, geom + (size_t)v * G * GS, s_keys,
                                    reinterpret_cast<uint16_t*>(reinterpret_cast<uint32_t*>(s_keys + padded)),
                                    reinterpret_cast<uint32_t*>(s_keys + padded) + sort_render_aux_words<NBL>(),
                                    reinterpret_cast<uint32_t*>(s_keys + padded) + sort_render_aux_words<NBL>() + 16,
                                    id_bits, (float)sx0, (float)sy0, pp, lane, dsplat::lanemask_lt(lane),
                                    reinterpret_cast<WaveList*>(reinterpret_cast<uint32_t*>(s_keys + padded)) + w, Tr,
                                    C01, C2, last, alive, spill_keys ? spill_keys + (size_t)seg * G : nullptr);
    if (inside) store_pixel(out, finalT, ncontrib, cams[v].bg, v, H, W, px, py, Tr, C01, C2, last);
    if (clear_counts && tid == 0) seg_count[seg] = 0u;
    return;
  }
  uint32_t b, e;
  seg_bounds(seg_start, seg_count, stride, seg, b, e);
  const uint32_t n = e - b;
  const bool in_lds = n <= cap;  // uniform
  if (in_lds) {
    uint64_t tmp[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      const uint32_t idx = tid + (uint32_t)i * NT;
      tmp[i] = idx < n ? keys[b + idx] : 0ull;
    }
    if (n > 1) {
      count_sort<KMAX, NT, NBL>(tmp, n, A, id_bits, cnt, wsum, flag);
    } else {
      if (tid == 0 && n == 1) A[0] = tmp[0];
      __syncthreads();
    }
    if (write_keys)
      for (uint32_t i = tid; i < n; i += NT) keys[b + i] = A[padi<KMAX>(i)];
  } else {
    sort_segment<NT>(keys + b, scratch + b, n, id_bits, aux, wsum, flag, keys + b);
    __syncthreads();
  }
  const int sx0 = tx * BX + (w & 1) * SUB, sy0 = ty * BY + (w >> 1) * SUB;
  const int px = sx0 + (lane & (SUB - 1));
  const int py = sy0 + (lane >> 3);
  const bool inside = px < W && py < H;
  const float* gv = geom + (size_t)v * G * GS;
  const uint64_t lt = dsplat::lanemask_lt(lane);
  WaveList* plist = reinterpret_cast<WaveList*>(aux) + w;
  const PixUV2 pp = pix_uv2(pix_uv(px, py, (float)sx0, (float)sy0));
  f2v C01 = {0.f, 0.f};
  float Tr = 1.0f, C2 = 0.f;
  bool alive = inside;
  uint32_t last = 0;
  // Gaussian ids come from LDS (or HBM) slots the sort filled; they are clamped to the view's
  // range so that a slot the sort did not write (a broken variant: r04 "noscat" read garbage
  // ids and faulted with hipErrorIllegalAddress) reads a valid record instead of faulting
  const uint32_t gmax = (uint32_t)G - 1u;
  if (in_lds)
    composite_tile<LAST>([&](uint32_t i) { return min((uint32_t)A[padi<KMAX>(i)], gmax); }, 0u, n, gv, (float)sx0,
                         (float)sy0, pp, lane, lt, plist, Tr, C01, C2, last, alive);
  else
    composite_tile<LAST>([&](uint32_t i) { return min((uint32_t)keys[i], gmax); }, b, e, gv, (float)sx0, (float)sy0, pp,
                         lane, lt, plist, Tr, C01, C2, last, alive);
  if (inside) store_pixel(out, finalT, ncontrib, cams[v].bg, v, H, W, px, py, Tr, C01, C2, last);
  // depth cut (seg_overflow given, DSR_SEG_ENDS): a pixel of this wave still live at the end
  // of the written part while the tile has omitted entries -> flag the tile, the any-flag and
  // the super-block, exactly as dsr_render_fwd does (the tail pass completes such tiles)
  if (seg_overflow != nullptr && e < seg_start[seg + 1] && __any(alive) && lane == 0) {
    seg_overflow[seg] = 1u;
    seg_overflow[(size_t)gridDim.z * T] = 1u;
    const int sb = cut_superblock(gx, T / gx), sbl = __builtin_ctz((unsigned)sb);
    const int nsx = (gx + sb - 1) / sb, nsb = nsx * ((T / gx + sb - 1) / sb);
    seg_overflow[(size_t)gridDim.z * T + 1 + (size_t)v * nsb + (ty >> sbl) * nsx + (tx >> sbl)] = 1u;
  }
  // counts handed back zeroed for the next call's binning (every thread read it before the
  // sort's first barrier)
  if (clear_counts && tid == 0) seg_count[seg] = 0u;
}

// ------------------------------------------------------------------------------------
// Sums of 4 entries x 9 gradient values over the wave (36 values, 90 instructions instead
// of 4 x 54): v_permlane32_swap pairs entries (0,1) and (2,3) across the wave halves,
// v_permlane16_swap pairs the results across rows, and a 4-step DPP row sum finishes:
// lane 15 of row 0 / 1 / 2 / 3 ends with the totals of entry 0 / 2 / 1 / 3.
__device__ __forceinline__ float swap32_add(float a, float b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap16_add(float a, float b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
#define DSR_ROW9(ctrl)                                                                              \
  asm volatile("v_add_f32_dpp %0, %0, %0 " ctrl "\n v_add_f32_dpp %1, %1, %1 " ctrl                \
               "\n v_add_f32_dpp %2, %2, %2 " ctrl "\n v_add_f32_dpp %3, %3, %3 " ctrl               \
               "\n v_add_f32_dpp %4, %4, %4 " ctrl "\n v_add_f32_dpp %5, %5, %5 " ctrl               \
               "\n v_add_f32_dpp %6, %6, %6 " ctrl "\n v_add_f32_dpp %7, %7, %7 " ctrl               \
               "\n v_add_f32_dpp %8, %8, %8 " ctrl                                                    \
               : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]), "+v"(R[4]), "+v"(R[5]), "+v"(R[6]), \
                 "+v"(R[7]), "+v"(R[8]))
__device__ __forceinline__ void reduce36(const float (&g)[4][9], float (&R)[9]) {
#pragma unroll
  for (int c = 0; c < 9; ++c) {
    const float P = swap32_add(g[0][c], g[1][c]);
    const float Q = swap32_add(g[2][c], g[3][c]);
    R[c] = swap16_add(P, Q);
  }
  asm volatile("s_nop 1" ::: "memory");
  DSR_ROW9("row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1");
  DSR_ROW9("row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1");
  DSR_ROW9("row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1");
  DSR_ROW9("row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1");
  asm volatile("s_nop 1" ::: "memory");
}

// ------------------------------------------------------------------------------------
// Deterministic gradient sums (include/dsplat_hip.h, DSR_GRAD_FRAC_BITS): partials are
// accumulated as int64 fixed point with a unit derived from m = max |dL_dpix|.
constexpr int kGradBlocks = DSR_GRAD_SCALE_BLOCKS;
static_assert(kGradBlocks % 64 == 0, "grad-scale blocks: whole waves");

// per-block maxima of |d| (non-finite values: +inf, so the unit derivation sees them)
__global__ __launch_bounds__(256) void k_grad_scale(size_t n, const float* __restrict__ d, float* __restrict__ out) {
  float m = 0.f;
  bool bad = false;
  const size_t n4 = n / 4, stride = (size_t)256 * gridDim.x;
  const float4* d4 = reinterpret_cast<const float4*>(d);
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    const float4 x = d4[i];
    const float a = fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
    bad = bad || !(fabsf(x.x) + fabsf(x.y) + fabsf(x.z) + fabsf(x.w) <= 3.0e38f);
    m = fmaxf(m, a);
  }
  for (size_t i = 4 * n4 + (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const float a = fabsf(d[i]);
    bad = bad || !(a <= 3.0e38f);
    m = fmaxf(m, a);
  }
  if (bad) m = __builtin_inff();
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}

// k with m <= 2^k from the per-block maxima (one wave; every wave of every kernel reading
// the same maxima gets the same k). Returns false when m is not finite.
__device__ __forceinline__ bool grad_fx_exp(const float* __restrict__ bm, int lane, int& k) {
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < kGradBlocks / 64; ++i) m = fmaxf(m, bm[i * 64 + lane]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  if (!(m <= 3.0e38f)) return false;
  int e = 0;
  frexpf(m, &e);  // m = f * 2^e, f in [0.5, 1); m == 0 -> e = 0
  k = max(e, -60);  // keeps 2^(32 - k) a normal float
  return true;
}
// partial -> fixed point (saturating far inside the int64 range)
__device__ __forceinline__ long long to_fx(float a, float unit_inv) {
  return (long long)rintf(fminf(fmaxf(a * unit_inv, -4.0e18f), 4.0e18f));
}
// fixed point -> float: high word (signed) and low word (unsigned) converted by the hardware
// and recombined with one FMA (within 1 ulp; the unit is a power of 2, so scaling is exact)
__device__ __forceinline__ float fx_to_float(long long q, float unit) {
  const int hi = (int)(q >> 32);
  const unsigned lo = (unsigned)(q & 0xffffffffll);
  return fmaf((float)hi, 4294967296.0f * unit, (float)lo * unit);
}

// one compacted backward list entry
struct __align__(16) BwdRec {
  float4 q;   // x, y, A, C (scaled conic, as in the forward)
  float4 r;   // B, opacity, red, green
  float4 s;   // blue, conic a, b, c
  float F, D, E;  // the forward's falloff polynomial of this wave's sub-tile (fall_poly)
  uint32_t id, pos, pad[3];  // pad[0]: power-test threshold (float); pad[1]: 1 / o (float)
};

// K7: back-to-front gradient of the compositing (upstream renderCUDA backward semantics).
// Same wave layout as K6: wave w owns sub-tile (w & 1, w >> 1), waves are independent. Each
// wave walks the tile list backwards from the largest n_contrib of its pixels, CH entries at a
// time: entries that can reach its sub-tile (same exact test as the forward) go to a
// wave-private LDS list; per entry the 64 pixel gradients (9 values) are summed with DPP and
// lane 63 parks the sums in LDS; at the end of the chunk the wave adds them to dgeom with
// one 64-bit fixed-point atomic per non-zero (entry, component): order-independent sums.
constexpr int BCH = 64;
#ifndef DSR_K7TW_WPE
#define DSR_K7TW_WPE 3
#endif
#ifndef DSR_K7TW_NS
#define DSR_K7TW_NS 4
#endif
#ifndef DSR_K7TW_PD
#define DSR_K7TW_PD 2
#endif
constexpr int kPDtw = DSR_K7TW_PD;  // chunks whose records the tile-wave K7 gathers up front
// WPE = 5 (96 VGPRs, small spills) pays only on wide grids (kbench at 64 views: -3 %; 16:
// level; 3: +12 %), so dsr_render_bwd picks it from the number of tiles.
template <int WPE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) void k_render_bwd(int G, int H, int W, int gx, int T,
                                                   const dsr_camera* __restrict__ cams,
                                                   const float* __restrict__ geom,
                                                   const uint32_t* __restrict__ seg_start,
                                                   const uint32_t* __restrict__ seg_count, uint32_t stride,
                                                   const uint64_t* __restrict__ keys,
                                                   const uint64_t* __restrict__ spill_keys,
                                                   const float* __restrict__ finalT,
                                                   const uint32_t* __restrict__ ncontrib,
                                                   const float* __restrict__ dpix,
                                                   const float* __restrict__ gscale,
                                                   long long* __restrict__ dgeom) {
  __shared__ BwdRec l_rec[4][BCH + 1];
  __shared__ float l_acc[4][BCH * 9];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  int tx, ty;
  const int v = tile_xcd(gx, T / gx, tx, ty);  // kbench: 3 views -4..-6 %, 64 views level
  const int sx0 = tx * BX + (w & 1) * SUB, sy0 = ty * BY + (w >> 1) * SUB;
  const int px = sx0 + (lane & (SUB - 1));
  const int py = sy0 + (lane >> 3);
  const bool inside = px < W && py < H;
  const int seg = v * T + ty * gx + tx;
  uint32_t start, end;
  seg_bounds(seg_start, seg_count, stride, seg, start, end);
  // a bounded segment that overflowed: dsr_sort_render stored its rebuilt list in the spill
  // area (G slots per segment) instead
  const bool spilled = spill_keys != nullptr && stride != 0u && stride != kSegEnds && end - start > stride;
  const uint64_t* __restrict__ kseg = spilled ? spill_keys + (size_t)seg * G : keys + start;
  const size_t HW = (size_t)H * W;
  const size_t pix = (size_t)py * W + px;
  const float pfx = (float)px, pfy = (float)py;
  const float fx0 = (float)sx0, fy0 = (float)sy0;
  const PixUV puv = pix_uv(px, py, fx0, fy0);
  const float* gv = geom + (size_t)v * G * GS;
  long long* dgv = dgeom + (size_t)v * G * DSR_DGEOM_WORDS;
  int fx_k = 0;
  const bool fx_ok = grad_fx_exp(gscale, lane, fx_k);
  const float fx_unit_inv = fx_ok ? ldexpf(1.f, DSR_GRAD_FRAC_BITS - fx_k) : 0.f;  // exact power of 2
  const float* bg = cams[v].bg;
  const uint64_t lt = dsplat::lanemask_lt(lane);
  BwdRec* list = l_rec[w];
  float* acc = l_acc[w];
  const float Tfin = inside ? finalT[v * HW + pix] : 0.f;
  const uint32_t lastc = inside ? ncontrib[v * HW + pix] : 0u;
  float dp0 = 0.f, dp1 = 0.f, dp2 = 0.f;
  if (inside) {
    dp0 = dpix[(size_t)v * 3 * HW + pix];
    dp1 = dpix[(size_t)v * 3 * HW + HW + pix];
    dp2 = dpix[(size_t)v * 3 * HW + 2 * HW + pix];
  }
  const float bg_dot = bg[0] * dp0 + bg[1] * dp1 + bg[2] * dp2;
  uint32_t wmax = lastc;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, off, 64));
  const uint32_t nproc = min(end - start, wmax);
  const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
  float Tr = Tfin;
  float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;
  float lc0 = 0.f, lc1 = 0.f, lc2 = 0.f, last_alpha = 0.f;
  // chunk c covers list positions [hi_c - BCH, hi_c), hi_c = nproc - c * BCH (back to front).
  // Entry ids and records of the first PD chunks are gathered in one batch up front, later
  // chunks one ahead (a wave walks ~3 chunks: one memory round trip instead of one per chunk).
  const int nch = (int)((nproc + BCH - 1) / BCH);
  auto id_at = [&](int c) -> uint32_t {  // unconditional key read (clamped), id 0 past the range
    const int pos = (int)nproc - (c + 1) * BCH + lane;
    const uint32_t k = min((uint32_t)kseg[(uint32_t)min(max(pos, 0), max((int)nproc - 1, 0))], (uint32_t)G - 1u);
    return (pos >= 0 && c < nch) ? k : 0u;
  };
  auto chunk = [&](int ch, uint32_t id, float4 q, float4 r, float bl) {
    const int p = (int)nproc - (ch + 1) * BCH + lane;  // this lane's list position (< 0: none)
    // pixels that can take a gradient from this chunk: last contributor past its lowest
    // position (walking back to front, few pixels are active in the first chunks); entries
    // whose alpha >= 1/255 region misses their box are skipped for the whole wave
    const uint32_t plo = (uint32_t)max((int)nproc - (ch + 1) * BCH, 0);
    const uint64_t act_px = __ballot(inside && lastc > plo);
    float lx0 = fx0, ly0 = fy0, lx1 = fx0 + (SUB - 1), ly1 = fy0 + (SUB - 1);
    if (act_px) live_rect(act_px, fx0, fy0, lx0, ly0, lx1, ly1);
    const bool mine = p >= 0 && act_px != 0ull && rect_hit(q, r, lx0, ly0, lx1, ly1);
    const uint64_t bal = __ballot(mine);
    if (mine) {
      BwdRec& d = list[__popcll(bal & lt)];
      const float4 sq = scaled_conic_q(q);
      d.q = make_float4(sq.x, sq.y, sq.z, -0.5f * kLog2e * r.x);
      d.r = make_float4(sq.w, r.y, r.z, r.w);
      d.s = make_float4(bl, q.z, q.w, r.x);
      const FallPoly f = fall_poly(sq.x, sq.y, sq.z, sq.w, d.q.w, fx0, fy0);
      const float lo = fall_lo(r.y);
      d.F = f.F + lo;  // as pair_put: the forward's o G = exp2(p2 + lo)
      d.D = f.D;
      d.E = f.E;
      d.id = id;
      d.pos = (uint32_t)p;
      // the forward's power test on the same floats: p2o <= thr (definite conic: always)
      d.pad[0] = __float_as_uint(conic_pd(d.q.z, d.r.x, d.q.w) ? __builtin_inff() : kP2Max + lo);
      // 1 / o for dL/do = S(h) / o; a subnormal o would give rcp = inf and 0 * inf = NaN (such an
      // entry never blends, S(h) = 0): its dL/do is 0, as the reference's S(G dL/dalpha) gives
      d.pad[1] = __float_as_uint(r.y >= 1.17549435e-38f ? __builtin_amdgcn_rcpf(r.y) : 0.f);
    }
    const int cnt = __popcll(bal);
    __builtin_amdgcn_wave_barrier();
    // four entries per step (back to front): the T chain runs entry by entry, then the 36
    // gradient values are summed over the wave together (reduce36)
    for (int k = cnt - 1; k >= 0; k -= 4) {
      float g[4][9];
      bool any = false;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = k - j;
        const BwdRec cur = list[max(kk, 0)];
#pragma unroll
        for (int c = 0; c < 9; ++c) g[j][c] = 0.f;
        const float dx = cur.q.x - pfx, dy = cur.q.y - pfy;
        // same falloff sequence as k_render_fwd (decisions must agree with the forward):
        // p2o = p2 + lo, o G = exp2(p2o)
        const float p2o = fall_p2(puv, cur.F, cur.D, cur.E, cur.q.z, cur.r.x, cur.q.w);
        const float oG = __builtin_amdgcn_exp2f(p2o);
        const float alpha = fminf(0.99f, oG);
        const bool act = kk >= 0 && cur.pos < lastc && p2o <= __uint_as_float(cur.pad[0]) && alpha >= 1.0f / 255.0f;
        any = any || act;
        if (act) {
          const float inv1ma = __builtin_amdgcn_rcpf(1.f - alpha);  // 1 ulp; the grads' tolerance is 2e-3
          Tr = Tr * inv1ma;
          const float dchannel_dcolor = alpha * Tr;
          const float c0 = cur.r.z, c1 = cur.r.w, c2 = cur.s.x;
          acc0 = last_alpha * lc0 + (1.f - last_alpha) * acc0;
          acc1 = last_alpha * lc1 + (1.f - last_alpha) * acc1;
          acc2 = last_alpha * lc2 + (1.f - last_alpha) * acc2;
          lc0 = c0;
          lc1 = c1;
          lc2 = c2;
          float dL_dalpha = (c0 - acc0) * dp0;
          dL_dalpha += (c1 - acc1) * dp1;
          dL_dalpha += (c2 - acc2) * dp2;
          g[j][6] = dchannel_dcolor * dp0;
          g[j][7] = dchannel_dcolor * dp1;
          g[j][8] = dchannel_dcolor * dp2;
          dL_dalpha *= Tr;
          last_alpha = alpha;
          dL_dalpha += (-Tfin * inv1ma) * bg_dot;
          // per pixel only the factors that vary over the pixels: with h = o G dL/dalpha the entry's sums are S(h dx), S(h dy), S(h dx^2), S(h dx dy),
          // S(h dy^2), S(h) = o S(G dL/dalpha); the conic and ndc factors (and 1 / o for
          // dL/do) multiply the sums once per entry
          const float h = oG * dL_dalpha;
          const float hx = h * dx, hy = h * dy;
          g[j][0] = hx;
          g[j][1] = hy;
          g[j][2] = hx * dx;
          g[j][3] = hx * dy;
          g[j][4] = hy * dy;
          g[j][5] = h;
        }
      }
      if (__ballot(any) != 0ull) {
        float R[9];
        reduce36(g, R);
        // lane 15 of row r holds the sums of entry k - {0, 2, 1, 3}[r]
        if ((lane & 15) == 15) {
          const int row = lane >> 4;
          const int kk = k - ((row & 1) * 2 + (row >> 1));
          if (kk >= 0) {
            // dL/dmean2D = S(o G dL/dalpha dG/dd / G) (ndc scale), dL/dconic = -1/2 S(h d d^T),
            // dL/do = S(h) / o (upstream renderCUDA backward, its per-pixel products regrouped)
            const float4 cs = list[kk].s;  // (blue, conic a, b, c)
            float* a9 = acc + kk * 9;
            a9[0] = -(cs.y * R[0] + cs.z * R[1]) * ddelx_dx;
            a9[1] = -(cs.w * R[1] + cs.z * R[0]) * ddely_dy;
            a9[2] = -0.5f * R[2];
            a9[3] = -0.5f * R[3];
            a9[4] = -0.5f * R[4];
            a9[5] = R[5] * __uint_as_float(list[kk].pad[1]);
#pragma unroll
            for (int c = 6; c < 9; ++c) a9[c] = R[c];
          }
        }
      } else if ((lane & 15) == 15) {
        const int row = lane >> 4;
        const int kk = k - ((row & 1) * 2 + (row >> 1));
        if (kk >= 0) {
          float* a9 = acc + kk * 9;
#pragma unroll
          for (int c = 0; c < 9; ++c) a9[c] = 0.f;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < cnt * 9; i += 64) {
      const float a = acc[i];
      const int k = i / 9;
      if (a != 0.f)
        atomicAdd(reinterpret_cast<unsigned long long*>(&dgv[(size_t)list[k].id * DSR_DGEOM_WORDS + (i - k * 9)]),
                  (unsigned long long)to_fx(a, fx_unit_inv));
    }
    __builtin_amdgcn_wave_barrier();
  };
  uint32_t ids[PD];
  float4 q[PD], r[PD];
  float bl[PD];
#pragma unroll
  for (int c = 0; c < PD; ++c) ids[c] = id_at(c);
#pragma unroll
  for (int c = 0; c < PD; ++c) {
    const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)ids[c] * GS);
    q[c] = rec[0];
    r[c] = rec[1];
    bl[c] = rec[2].x;
  }
  uint32_t nid = id_at(PD);
#pragma unroll
  for (int c = 0; c < PD; ++c)
    if (c < nch) chunk(c, ids[c], q[c], r[c], bl[c]);
  for (int c = PD; c < nch; ++c) {
    const uint32_t id = nid;
    const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)id * GS);
    const float4 cq = rec[0], cr = rec[1];
    const float cb = rec[2].x;
    nid = id_at(c + 1);
    chunk(c, id, cq, cr, cb);
  }
}

// K7, tile-wave form (round 6): ONE wave per 16x16 tile; lane l holds the pixel (l & 7, l >> 3)
// of each of the four 8x8 sub-tiles (all four share the sub-tile offset (u, v), so the falloff
// polynomial of an entry differs between them only in its constant terms F, D, E, staged per
// sub-tile exactly as the sub-tile waves of k_render_bwd stage theirs: the same alpha, the same
// skip decisions). Per entry the four pixels' gradient terms are added in the lane, then over
// the wave (reduce36): one dgeom row per (tile, entry) instead of one per (sub-tile, entry),
// and four independent transmittance chains per lane.
struct __align__(16) BwdRec4 {
  float4 q;        // x, y, A, C (scaled conic)
  float4 r;        // B, opacity, red, green
  float4 s;        // blue, conic a, b, c
  float4 F, D, E;  // per sub-tile falloff constants (F includes lo = log2 o)
  uint32_t id, pos, mask;  // mask: the sub-tiles the entry reaches (rect_hit on their live pixels)
  float thr, rcp_o;        // power-test threshold, 1 / o
  uint32_t pad[3];
};
// NS: sub-tiles per wave (4: one wave per tile; 2: two waves, the tile's top and bottom halves)
template <int WPE, int NS>
__global__ __launch_bounds__(64 * (4 / NS)) __attribute__((amdgpu_waves_per_eu(WPE))) void k_render_bwd_tw(
    int G, int H, int W, int gx, int T, const dsr_camera* __restrict__ cams, const float* __restrict__ geom,
    const uint32_t* __restrict__ seg_start, const uint32_t* __restrict__ seg_count, uint32_t stride,
    const uint64_t* __restrict__ keys, const uint64_t* __restrict__ spill_keys, const float* __restrict__ finalT,
    const uint32_t* __restrict__ ncontrib, const float* __restrict__ dpix, const float* __restrict__ gscale,
    long long* __restrict__ dgeom) {
  __shared__ BwdRec4 l_list[4 / NS][BCH + 1];
  __shared__ float l_acc[4 / NS][BCH * 9];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, kb = wv * NS;  // this wave's first sub-tile
  BwdRec4* list = l_list[wv];
  float* acc = l_acc[wv];
  int tx, ty;
  const int v = tile_xcd(gx, T / gx, tx, ty);
  const int sxl = lane & (SUB - 1), syl = lane >> 3;
  const float tfx0 = (float)(tx * BX), tfy0 = (float)(ty * BY);
  const int seg = v * T + ty * gx + tx;
  uint32_t start, end;
  seg_bounds(seg_start, seg_count, stride, seg, start, end);
  const bool spilled = spill_keys != nullptr && stride != 0u && stride != kSegEnds && end - start > stride;
  const uint64_t* __restrict__ kseg = spilled ? spill_keys + (size_t)seg * G : keys + start;
  const size_t HW = (size_t)H * W;
  const float* gv = geom + (size_t)v * G * GS;
  long long* dgv = dgeom + (size_t)v * G * DSR_DGEOM_WORDS;
  int fx_k = 0;
  const bool fx_ok = grad_fx_exp(gscale, lane, fx_k);
  const float fx_unit_inv = fx_ok ? ldexpf(1.f, DSR_GRAD_FRAC_BITS - fx_k) : 0.f;
  const float* bg = cams[v].bg;
  const uint64_t lt = dsplat::lanemask_lt(lane);
  // the lane's pixel in each sub-tile k = (k & 1, k >> 1); the same (u, v) offsets for all four
  const PixUV puv = pix_uv(sxl, syl, 0.f, 0.f);
  // per pixel (lastc = 0 off the image: no entry is active there), the background term
  // -T_final (bg . dL/dpix) folded once
  float dp0[NS], dp1[NS], dp2[NS], bgT[NS], Tr[NS], a0[NS], a1[NS], a2[NS], l0[NS], l1[NS], l2[NS], la[NS];
  uint32_t lastc[NS];
  uint32_t wmax = 0u;
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int st = kb + k;
    const int px = tx * BX + (st & 1) * SUB + sxl, py = ty * BY + (st >> 1) * SUB + syl;
    const bool inside = px < W && py < H;
    const size_t pix = (size_t)py * W + px;
    const float tf = inside ? finalT[v * HW + pix] : 0.f;
    lastc[k] = inside ? ncontrib[v * HW + pix] : 0u;
    dp0[k] = inside ? dpix[(size_t)v * 3 * HW + pix] : 0.f;
    dp1[k] = inside ? dpix[(size_t)v * 3 * HW + HW + pix] : 0.f;
    dp2[k] = inside ? dpix[(size_t)v * 3 * HW + 2 * HW + pix] : 0.f;
    bgT[k] = -tf * (bg[0] * dp0[k] + bg[1] * dp1[k] + bg[2] * dp2[k]);
    Tr[k] = tf;
    a0[k] = a1[k] = a2[k] = l0[k] = l1[k] = l2[k] = la[k] = 0.f;
    wmax = max(wmax, lastc[k]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, off, 64));
  const uint32_t nproc = min(end - start, wmax);
  const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
  const int nch = (int)((nproc + BCH - 1) / BCH);
  auto id_at = [&](int c) -> uint32_t {
    const int pos = (int)nproc - (c + 1) * BCH + lane;
    const uint32_t kk = min((uint32_t)kseg[(uint32_t)min(max(pos, 0), max((int)nproc - 1, 0))], (uint32_t)G - 1u);
    return (pos >= 0 && c < nch) ? kk : 0u;
  };
  auto chunk = [&](int ch, uint32_t id, float4 q, float4 r, float bl) {
    const int p = (int)nproc - (ch + 1) * BCH + lane;
    const uint32_t plo = (uint32_t)max((int)nproc - (ch + 1) * BCH, 0);
    uint32_t mk = 0u;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const float fx0 = tfx0 + (float)(((kb + k) & 1) * SUB), fy0 = tfy0 + (float)(((kb + k) >> 1) * SUB);
      const uint64_t act_px = __ballot(lastc[k] > plo);
      float lx0 = fx0, ly0 = fy0, lx1 = fx0 + (SUB - 1), ly1 = fy0 + (SUB - 1);
      if (act_px) live_rect(act_px, fx0, fy0, lx0, ly0, lx1, ly1);
      if (p >= 0 && act_px != 0ull && rect_hit(q, r, lx0, ly0, lx1, ly1)) mk |= 1u << k;
    }
    const uint64_t bal = __ballot(mk != 0u);
    if (mk) {
      BwdRec4& d = list[__popcll(bal & lt)];
      const float4 sq = scaled_conic_q(q);
      d.q = make_float4(sq.x, sq.y, sq.z, -0.5f * kLog2e * r.x);
      d.r = make_float4(sq.w, r.y, r.z, r.w);
      d.s = make_float4(bl, q.z, q.w, r.x);
      const float lo = fall_lo(r.y);
      float Fk[4] = {0.f, 0.f, 0.f, 0.f}, Dk[4] = {0.f, 0.f, 0.f, 0.f}, Ek[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const FallPoly f = fall_poly(sq.x, sq.y, sq.z, sq.w, d.q.w, tfx0 + (float)(((kb + k) & 1) * SUB),
                                     tfy0 + (float)(((kb + k) >> 1) * SUB));
        Fk[k] = f.F + lo;
        Dk[k] = f.D;
        Ek[k] = f.E;
      }
      d.F = make_float4(Fk[0], Fk[1], Fk[2], Fk[3]);
      d.D = make_float4(Dk[0], Dk[1], Dk[2], Dk[3]);
      d.E = make_float4(Ek[0], Ek[1], Ek[2], Ek[3]);
      d.id = id;
      d.pos = (uint32_t)p;
      d.mask = mk;
      d.thr = conic_pd(d.q.z, d.r.x, d.q.w) ? __builtin_inff() : kP2Max + lo;
      d.rcp_o = r.y >= 1.17549435e-38f ? __builtin_amdgcn_rcpf(r.y) : 0.f;
    }
    const int cnt = __popcll(bal);
    __builtin_amdgcn_wave_barrier();
    for (int k = cnt - 1; k >= 0; k -= 4) {
      float g[4][9];
      bool any = false;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = k - j;
        const BwdRec4 cur = list[max(kk, 0)];
#pragma unroll
        for (int c = 0; c < 9; ++c) g[j][c] = 0.f;
        const float c0 = cur.r.z, c1 = cur.r.w, c2 = cur.s.x;
        const float Fs[4] = {cur.F.x, cur.F.y, cur.F.z, cur.F.w};
        const float Ds[4] = {cur.D.x, cur.D.y, cur.D.z, cur.D.w};
        const float Es[4] = {cur.E.x, cur.E.y, cur.E.z, cur.E.w};
#pragma unroll
        for (int s4 = 0; s4 < NS; ++s4) {
          const int st = kb + s4;
          const float pfx = tfx0 + (float)((st & 1) * SUB + sxl), pfy = tfy0 + (float)((st >> 1) * SUB + syl);
          const float dx = cur.q.x - pfx, dy = cur.q.y - pfy;
          const float p2o = fall_p2(puv, Fs[s4], Ds[s4], Es[s4], cur.q.z, cur.r.x, cur.q.w);
          const float oG = __builtin_amdgcn_exp2f(p2o);
          const float alpha = fminf(0.99f, oG);
          const bool act = kk >= 0 && ((cur.mask >> s4) & 1u) && cur.pos < lastc[s4] && p2o <= cur.thr &&
                           alpha >= 1.0f / 255.0f;
          any = any || act;
          if (act) {
            const float inv1ma = __builtin_amdgcn_rcpf(1.f - alpha);
            Tr[s4] = Tr[s4] * inv1ma;
            const float dchannel_dcolor = alpha * Tr[s4];
            a0[s4] = la[s4] * l0[s4] + (1.f - la[s4]) * a0[s4];
            a1[s4] = la[s4] * l1[s4] + (1.f - la[s4]) * a1[s4];
            a2[s4] = la[s4] * l2[s4] + (1.f - la[s4]) * a2[s4];
            l0[s4] = c0;
            l1[s4] = c1;
            l2[s4] = c2;
            float dL_dalpha = (c0 - a0[s4]) * dp0[s4];
            dL_dalpha += (c1 - a1[s4]) * dp1[s4];
            dL_dalpha += (c2 - a2[s4]) * dp2[s4];
            g[j][6] += dchannel_dcolor * dp0[s4];
            g[j][7] += dchannel_dcolor * dp1[s4];
            g[j][8] += dchannel_dcolor * dp2[s4];
            dL_dalpha *= Tr[s4];
            la[s4] = alpha;
            dL_dalpha += bgT[s4] * inv1ma;
            const float h = oG * dL_dalpha;
            const float hx = h * dx, hy = h * dy;
            g[j][0] += hx;
            g[j][1] += hy;
            g[j][2] += hx * dx;
            g[j][3] += hx * dy;
            g[j][4] += hy * dy;
            g[j][5] += h;
          }
        }
      }
      if (__ballot(any) != 0ull) {
        float R[9];
        reduce36(g, R);
        if ((lane & 15) == 15) {
          const int row = lane >> 4;
          const int kk = k - ((row & 1) * 2 + (row >> 1));
          if (kk >= 0) {
            const float4 cs = list[kk].s;
            float* a9 = acc + kk * 9;
            a9[0] = -(cs.y * R[0] + cs.z * R[1]) * ddelx_dx;
            a9[1] = -(cs.w * R[1] + cs.z * R[0]) * ddely_dy;
            a9[2] = -0.5f * R[2];
            a9[3] = -0.5f * R[3];
            a9[4] = -0.5f * R[4];
            a9[5] = R[5] * list[kk].rcp_o;
#pragma unroll
            for (int c = 6; c < 9; ++c) a9[c] = R[c];
          }
        }
      } else if ((lane & 15) == 15) {
        const int row = lane >> 4;
        const int kk = k - ((row & 1) * 2 + (row >> 1));
        if (kk >= 0) {
          float* a9 = acc + kk * 9;
#pragma unroll
          for (int c = 0; c < 9; ++c) a9[c] = 0.f;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < cnt * 9; i += 64) {
      const float a = acc[i];
      const int k = i / 9;
      if (a != 0.f)
        atomicAdd(reinterpret_cast<unsigned long long*>(&dgv[(size_t)list[k].id * DSR_DGEOM_WORDS + (i - k * 9)]),
                  (unsigned long long)to_fx(a, fx_unit_inv));
    }
    __builtin_amdgcn_wave_barrier();
  };
  uint32_t ids[kPDtw];
  float4 q[kPDtw], r[kPDtw];
  float bl[kPDtw];
#pragma unroll
  for (int c = 0; c < kPDtw; ++c) ids[c] = id_at(c);
#pragma unroll
  for (int c = 0; c < kPDtw; ++c) {
    const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)ids[c] * GS);
    q[c] = rec[0];
    r[c] = rec[1];
    bl[c] = rec[2].x;
  }
  uint32_t nid = id_at(kPDtw);
#pragma unroll
  for (int c = 0; c < kPDtw; ++c)
    if (c < nch) chunk(c, ids[c], q[c], r[c], bl[c]);
  for (int c = kPDtw; c < nch; ++c) {
    const uint32_t id = nid;
    const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)id * GS);
    const float4 cq = rec[0], cr = rec[1];
    const float cb = rec[2].x;
    nid = id_at(c + 1);
    chunk(c, id, cq, cr, cb);
  }
}

// K8 + K9's per-Gaussian work: Gaussian g of scene s (valid: g < G), its view-independent
// inputs m0 (mean), c60 (covariance triu) and sh (coefficient-major), summed over the scene's
// views in view order from the fixed-point rows dgeom -> the gradients of the mean (dm), the
// covariance triu (dc), the opacity (dop), the SH (dsh) or precomputed colours (dcol).
// Shared by k_preprocess_bwd and the fused head backward (k_head_bwd): the same operations.
template <int DEG>
__device__ __forceinline__ void pbwd_views(int s, int g, bool valid, int G, int H, int W, F3 m0,
                                           const float (&c60)[6], const float* sh, const dsr_camera* __restrict__ cams,
                                           const float* __restrict__ geom, const long long* __restrict__ dgeom,
                                           float fx_unit, const int32_t* __restrict__ scene_view_start,
                                           const int32_t* __restrict__ scene_views,
                                           const uint8_t* __restrict__ row_live, float* __restrict__ dmean2D,
                                           float& dm0, float& dm1, float& dm2, float& dop, float (&dc)[6],
                                           float* dsh, float& dcol0, float& dcol1, float& dcol2) {
  // the view loop is workgroup-uniform (scene = blockIdx.y), so the view ids and every camera
  // field below are scalar loads; lanes past the scene's last Gaussian ride along masked off
  const int vb = scene_view_start[s], ve = scene_view_start[s + 1];
  for (int k = vb; k < ve; ++k) {
    const int v = scene_views[k];
    const size_t vg = (size_t)v * G + g;
    // deferred geometry (depth cut): only the rows of the Gaussians some written list refers to
    // have a record and a zeroed accumulator (row_live); the others are skipped unread
    const bool live = valid && (row_live == nullptr || row_live[vg] != 0u);
    const float4 rec2 = live ? reinterpret_cast<const float4*>(geom + vg * GS)[2]  // depth, radius, clamp bits
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    const int radius = __float_as_int(rec2.z);
    if (radius <= 0) {
      if (dmean2D && valid) {
        dmean2D[3 * vg] = 0.f;
        dmean2D[3 * vg + 1] = 0.f;
        dmean2D[3 * vg + 2] = 0.f;
      }
      continue;
    }
    const long long* dq = dgeom + vg * DSR_DGEOM_WORDS;
    float dg[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) dg[c] = fx_to_float(dq[c], fx_unit);
    const dsr_camera* cam = cams + v;
    // scale-invariant rescale of this view: forward used m*s and cov*s^2
    const float gsc = cam->scale, gsc2 = gsc * gsc;
    const F3 m = {m0.x * gsc, m0.y * gsc, m0.z * gsc};
    float c6[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) c6[q] = c60[q] * gsc2;
    const float g2x = dg[0], g2y = dg[1];
    const float ga = dg[2], gb = dg[3], gc = dg[4];
    dop += dg[5];
    const float drgb0 = dg[6], drgb1 = dg[7], drgb2 = dg[8];
    if (dmean2D) {
      dmean2D[3 * vg] = g2x;
      dmean2D[3 * vg + 1] = g2y;
      dmean2D[3 * vg + 2] = 0.f;
    }
    const float fx = W / (2.0f * cam->tanfovx);
    const float fy = H / (2.0f * cam->tanfovy);
    Cov2D w;
    cov2d(m, fx, fy, cam->tanfovx, cam->tanfovy, c6, cam->viewmatrix, w);
    // conic S = inverse(cov2D): dL/dcov2D = -S (dL/dS) S with the conic the forward stored
    // (no det(cov2D)^2: its a c - b^2 cancels for needle-shaped Gaussians and cost up to ~2e-3
    // of the largest dL/dmean3D in float); gb carries half the off-diagonal derivative, so
    // dL/db = 2 M01 (oracle/dsr_oracle.cpp, same formula).
    const float4 rec0 = reinterpret_cast<const float4*>(geom + vg * GS)[0];  // x, y, conic A, B
    const float SA = rec0.z, SB = rec0.w, SC = geom[vg * GS + 4];
    const float sg00 = SA * ga + SB * gb, sg01 = SA * gb + SB * gc;
    const float sg10 = SB * ga + SC * gb, sg11 = SB * gb + SC * gc;
    const float dL_da = -(sg00 * SA + sg01 * SB);
    const float dL_dc = -(sg10 * SB + sg11 * SC);
    const float dL_db = -2.f * (sg00 * SB + sg01 * SC);
    const auto& Tm = w.T;
    float dcv[6];
    dcv[0] = Tm[0][0] * Tm[0][0] * dL_da + Tm[0][0] * Tm[1][0] * dL_db + Tm[1][0] * Tm[1][0] * dL_dc;
    dcv[3] = Tm[0][1] * Tm[0][1] * dL_da + Tm[0][1] * Tm[1][1] * dL_db + Tm[1][1] * Tm[1][1] * dL_dc;
    dcv[5] = Tm[0][2] * Tm[0][2] * dL_da + Tm[0][2] * Tm[1][2] * dL_db + Tm[1][2] * Tm[1][2] * dL_dc;
    dcv[1] = 2 * Tm[0][0] * Tm[0][1] * dL_da + (Tm[0][0] * Tm[1][1] + Tm[0][1] * Tm[1][0]) * dL_db +
             2 * Tm[1][0] * Tm[1][1] * dL_dc;
    dcv[2] = 2 * Tm[0][0] * Tm[0][2] * dL_da + (Tm[0][0] * Tm[1][2] + Tm[0][2] * Tm[1][0]) * dL_db +
             2 * Tm[1][0] * Tm[1][2] * dL_dc;
    dcv[4] = 2 * Tm[0][2] * Tm[0][1] * dL_da + (Tm[0][1] * Tm[1][2] + Tm[0][2] * Tm[1][1]) * dL_db +
             2 * Tm[1][1] * Tm[1][2] * dL_dc;
#pragma unroll
    for (int q = 0; q < 6; ++q) dc[q] += dcv[q] * gsc2;
    const float V[3][3] = {{c6[0], c6[1], c6[2]}, {c6[1], c6[3], c6[4]}, {c6[2], c6[4], c6[5]}};
    float dT0[3], dT1[3];
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
      const float vt0 = V[rr][0] * Tm[0][0] + V[rr][1] * Tm[0][1] + V[rr][2] * Tm[0][2];
      const float vt1 = V[rr][0] * Tm[1][0] + V[rr][1] * Tm[1][1] + V[rr][2] * Tm[1][2];
      dT0[rr] = 2 * vt0 * dL_da + vt1 * dL_db;
      dT1[rr] = 2 * vt1 * dL_dc + vt0 * dL_db;
    }
    const float* vw = cam->viewmatrix;
    const float W00 = vw[0], W01 = vw[4], W02 = vw[8];
    const float W10 = vw[1], W11 = vw[5], W12 = vw[9];
    const float W20 = vw[2], W21 = vw[6], W22 = vw[10];
    const float dJ00 = dT0[0] * W00 + dT0[1] * W01 + dT0[2] * W02;
    const float dJ02 = dT0[0] * W20 + dT0[1] * W21 + dT0[2] * W22;
    const float dJ11 = dT1[0] * W10 + dT1[1] * W11 + dT1[2] * W12;
    const float dJ12 = dT1[0] * W20 + dT1[1] * W21 + dT1[2] * W22;
    const float tz = 1.f / w.tz, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dtx = w.xmul * -fx * tz2 * dJ02;
    const float dty = w.ymul * -fy * tz2 * dJ12;
    const float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2 * fx * w.tx) * tz3 * dJ02 +
                      (2 * fy * w.ty) * tz3 * dJ12;
    float e0 = W00 * dtx + W10 * dty + W20 * dtz;
    float e1 = W01 * dtx + W11 * dty + W21 * dtz;
    float e2 = W02 * dtx + W12 * dty + W22 * dtz;
    const float* proj = cam->projmatrix;
    const float mhx = proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12];
    const float mhy = proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13];
    const float mw = 1.0f / (proj[3] * m.x + proj[7] * m.y + proj[11] * m.z + proj[15] + 0.0000001f);
    const float mul1 = mhx * mw * mw, mul2 = mhy * mw * mw;
    e0 += (proj[0] * mw - proj[3] * mul1) * g2x + (proj[1] * mw - proj[3] * mul2) * g2y;
    e1 += (proj[4] * mw - proj[7] * mul1) * g2x + (proj[5] * mw - proj[7] * mul2) * g2y;
    e2 += (proj[8] * mw - proj[11] * mul1) * g2x + (proj[9] * mw - proj[11] * mul2) * g2y;
    if constexpr (DEG < 0) {
      dcol0 += drgb0;
      dcol1 += drgb1;
      dcol2 += drgb2;
    } else {
      const uint32_t cb = __float_as_uint(rec2.w);
      const float dR[3] = {(cb & 1u) ? 0.f : drgb0, (cb & 2u) ? 0.f : drgb1, (cb & 4u) ? 0.f : drgb2};
      const float dx0 = m.x - cam->campos[0], dy0 = m.y - cam->campos[1], dz0 = m.z - cam->campos[2];
      const float len = sqrtf(dx0 * dx0 + dy0 * dy0 + dz0 * dz0);
      const float x = dx0 / len, y = dy0 / len, z = dz0 / len;
      float gdx = 0.f, gdy = 0.f, gdz = 0.f;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        auto sv = [&](int k) { return sh[k * 3 + ch]; };
        const float gr = dR[ch];
        dsh[0 * 3 + ch] += SH_C0 * gr;
        float ddx = 0.f, ddy = 0.f, ddz = 0.f;
        if constexpr (DEG > 0) {
          dsh[1 * 3 + ch] += -SH_C1 * y * gr;
          dsh[2 * 3 + ch] += SH_C1 * z * gr;
          dsh[3 * 3 + ch] += -SH_C1 * x * gr;
          ddx = -SH_C1 * sv(3);
          ddy = -SH_C1 * sv(1);
          ddz = SH_C1 * sv(2);
          if constexpr (DEG > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            dsh[4 * 3 + ch] += SH_C2_0 * xy * gr;
            dsh[5 * 3 + ch] += SH_C2_1 * yz * gr;
            dsh[6 * 3 + ch] += SH_C2_2 * (2.f * zz - xx - yy) * gr;
            dsh[7 * 3 + ch] += SH_C2_3 * xz * gr;
            dsh[8 * 3 + ch] += SH_C2_4 * (xx - yy) * gr;
            ddx += SH_C2_0 * y * sv(4) + SH_C2_2 * 2.f * -x * sv(6) + SH_C2_3 * z * sv(7) + SH_C2_4 * 2.f * x * sv(8);
            ddy += SH_C2_0 * x * sv(4) + SH_C2_1 * z * sv(5) + SH_C2_2 * 2.f * -y * sv(6) + SH_C2_4 * 2.f * -y * sv(8);
            ddz += SH_C2_1 * y * sv(5) + SH_C2_2 * 2.f * 2.f * z * sv(6) + SH_C2_3 * x * sv(7);
            if constexpr (DEG > 2) {
              dsh[9 * 3 + ch] += SH_C3_0 * y * (3.f * xx - yy) * gr;
              dsh[10 * 3 + ch] += SH_C3_1 * xy * z * gr;
              dsh[11 * 3 + ch] += SH_C3_2 * y * (4.f * zz - xx - yy) * gr;
              dsh[12 * 3 + ch] += SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy) * gr;
              dsh[13 * 3 + ch] += SH_C3_4 * x * (4.f * zz - xx - yy) * gr;
              dsh[14 * 3 + ch] += SH_C3_5 * z * (xx - yy) * gr;
              dsh[15 * 3 + ch] += SH_C3_6 * x * (xx - 3.f * yy) * gr;
              ddx += SH_C3_0 * sv(9) * 3.f * 2.f * xy + SH_C3_1 * sv(10) * yz + SH_C3_2 * sv(11) * -2.f * xy +
                     SH_C3_3 * sv(12) * -3.f * 2.f * xz + SH_C3_4 * sv(13) * (-3.f * xx + 4.f * zz - yy) +
                     SH_C3_5 * sv(14) * 2.f * xz + SH_C3_6 * sv(15) * 3.f * (xx - yy);
              ddy += SH_C3_0 * sv(9) * 3.f * (xx - yy) + SH_C3_1 * sv(10) * xz +
                     SH_C3_2 * sv(11) * (-3.f * yy + 4.f * zz - xx) + SH_C3_3 * sv(12) * -3.f * 2.f * yz +
                     SH_C3_4 * sv(13) * -2.f * xy + SH_C3_5 * sv(14) * -2.f * yz + SH_C3_6 * sv(15) * -3.f * 2.f * xy;
              ddz += SH_C3_1 * sv(10) * xy + SH_C3_2 * sv(11) * 4.f * 2.f * yz +
                     SH_C3_3 * sv(12) * 3.f * (2.f * zz - xx - yy) + SH_C3_4 * sv(13) * 4.f * 2.f * xz +
                     SH_C3_5 * sv(14) * (xx - yy);
            }
          }
        }
        gdx += ddx * gr;
        gdy += ddy * gr;
        gdz += ddz * gr;
      }
      const float sum2 = dx0 * dx0 + dy0 * dy0 + dz0 * dz0;
      const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
      e0 += ((sum2 - dx0 * dx0) * gdx - dy0 * dx0 * gdy - dz0 * dx0 * gdz) * invsum32;
      e1 += (-dx0 * dy0 * gdx + (sum2 - dy0 * dy0) * gdy - dz0 * dy0 * gdz) * invsum32;
      e2 += (-dx0 * dz0 * gdx - dy0 * dz0 * gdy + (sum2 - dz0 * dz0) * gdz) * invsum32;
    }
    dm0 += e0 * gsc;
    dm1 += e1 * gsc;
    dm2 += e2 * gsc;
  }
}

// ------------------------------------------------------------------------------------
// K8 + K9: per (scene, Gaussian), summed over the scene's views in a fixed order.
template <int DEG>
__global__ __launch_bounds__(NT) void k_preprocess_bwd(
    int G, int H, int W, int M, const float* __restrict__ means, const float* __restrict__ shs,
    const float* __restrict__ cov6, const dsr_camera* __restrict__ cams,
    const float* __restrict__ geom, const long long* __restrict__ dgeom, const float* __restrict__ gscale,
    const int32_t* __restrict__ scene_view_start, const int32_t* __restrict__ scene_views,
    const uint8_t* __restrict__ row_live,
    float* __restrict__ dmeans, float* __restrict__ dshs, float* __restrict__ dcolors,
    float* __restrict__ dopac, float* __restrict__ dcov6, float* __restrict__ dmean2D, int layout) {
  constexpr int NC = DEG >= 0 ? (DEG + 1) * (DEG + 1) : 1;
  int fx_k = 0;  // fixed-point unit of dgeom (k_render_bwd); non-finite dL_dpix -> NaN gradients
  const float fx_unit = grad_fx_exp(gscale, threadIdx.x & 63, fx_k) ? ldexpf(1.f, fx_k - DSR_GRAD_FRAC_BITS)
                                                                     : __builtin_nanf("");
  extern __shared__ __attribute__((aligned(16))) float lds[];  // NT * max(3 M, 9) floats: row staging
  const int s = blockIdx.y;
  const int tid = threadIdx.x;
  const int g0 = blockIdx.x * NT;
  const int nrows = min(NT, G - g0);
  const int g = g0 + tid;
  const bool valid = tid < nrows;
  const size_t sg0 = (size_t)s * G + g0;
  const size_t sg = sg0 + tid;
  const int cw = (layout & kLayoutCovFull) ? 9 : 6;
  // scene inputs of the block's Gaussians: coalesced through LDS
  F3 m0 = {0.f, 0.f, 0.f};
  float c60[6];
  float sh[NC * 3];
  float dsh[NC * 3];
#pragma unroll
  for (int k = 0; k < NC * 3; ++k) {
    sh[k] = 0.f;
    dsh[k] = 0.f;
  }
  // the covariance and SH row blocks are requested into registers together with the means
  // (one memory round trip per workgroup instead of three) when the blocks are 16-byte aligned
  // and the SH rows hold exactly the evaluated coefficients; else staged one after the other
  constexpr int PS = DEG >= 0 ? (3 * NC + 3) / 4 : 1;
  const int rw = DEG >= 0 ? 3 * M : 0;
  const bool pf = dsplat::aligned16(cov6 + cw * sg0) &&
                  (DEG < 0 || (rw <= 4 * PS && dsplat::aligned16(shs + (size_t)rw * sg0)));
  float4 vc[3], vs[PS];
  if (pf) {
    dsplat::pref_get<NT>(cov6 + cw * sg0, (size_t)cw * nrows, vc);
    if constexpr (DEG >= 0) dsplat::pref_get<NT>(shs + (size_t)rw * sg0, (size_t)rw * nrows, vs);
  }
  dsplat::stage_in<NT>(means + 3 * sg0, (size_t)3 * nrows, lds);
  __syncthreads();
  if (valid) m0 = {lds[3 * tid], lds[3 * tid + 1], lds[3 * tid + 2]};
  __syncthreads();
  if (pf)
    dsplat::pref_put<NT>(cov6 + cw * sg0, (size_t)cw * nrows, vc, lds);
  else
    dsplat::stage_in<NT>(cov6 + cw * sg0, (size_t)cw * nrows, lds);
  __syncthreads();
  {
    constexpr int full_idx[6] = {0, 1, 2, 4, 5, 8};
#pragma unroll
    for (int k = 0; k < 6; ++k) c60[k] = valid ? lds[tid * cw + (cw == 9 ? full_idx[k] : k)] : 0.f;
  }
  __syncthreads();
  if constexpr (DEG >= 0) {
    if (pf)
      dsplat::pref_put<NT>(shs + (size_t)rw * sg0, (size_t)rw * nrows, vs, lds);
    else
      dsplat::stage_in<NT>(shs + (size_t)rw * sg0, (size_t)rw * nrows, lds);
    __syncthreads();
    if (valid) {
      const float* p = lds + tid * rw;
      if (layout & kLayoutShChannelMajor) {
#pragma unroll
        for (int k = 0; k < NC; ++k)
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) sh[k * 3 + ch] = p[ch * M + k];
      } else {
#pragma unroll
        for (int k = 0; k < NC * 3; ++k) sh[k] = p[k];
      }
    }
    __syncthreads();
  }
  float dm0 = 0.f, dm1 = 0.f, dm2 = 0.f, dop = 0.f, dcol0 = 0.f, dcol1 = 0.f, dcol2 = 0.f;
  float dc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  pbwd_views<DEG>(s, g, valid, G, H, W, m0, c60, sh, cams, geom, dgeom, fx_unit, scene_view_start, scene_views,
                  row_live, dmean2D, dm0, dm1, dm2, dop, dc, dsh, dcol0, dcol1, dcol2);
  // outputs: coalesced through LDS
  if (valid) {
    lds[3 * tid] = dm0;
    lds[3 * tid + 1] = dm1;
    lds[3 * tid + 2] = dm2;
  }
  __syncthreads();
  dsplat::stage_out<NT>(dmeans + 3 * sg0, (size_t)3 * nrows, lds);
  __syncthreads();
  if (valid) {
    float* o = lds + tid * cw;
    if (cw == 9) {  // gradient lands on the upper triangle only (triu gather)
      o[0] = dc[0]; o[1] = dc[1]; o[2] = dc[2];
      o[3] = 0.f;   o[4] = dc[3]; o[5] = dc[4];
      o[6] = 0.f;   o[7] = 0.f;   o[8] = dc[5];
    } else {
#pragma unroll
      for (int k = 0; k < 6; ++k) o[k] = dc[k];
    }
  }
  __syncthreads();
  dsplat::stage_out<NT>(dcov6 + cw * sg0, (size_t)cw * nrows, lds);
  if (valid) dopac[sg] = dop;
  if constexpr (DEG < 0) {
    if (valid) {
      dcolors[3 * sg] = dcol0;
      dcolors[3 * sg + 1] = dcol1;
      dcolors[3 * sg + 2] = dcol2;
    }
  } else {
    const int rw = 3 * M;
    __syncthreads();
    if (valid) {
      float* o = lds + tid * rw;
      if (layout & kLayoutShChannelMajor) {
#pragma unroll
        for (int k = 0; k < NC; ++k)
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) o[ch * M + k] = dsh[k * 3 + ch];
        for (int k = NC; k < M; ++k)
          for (int ch = 0; ch < 3; ++ch) o[ch * M + k] = 0.f;
      } else {
#pragma unroll
        for (int k = 0; k < NC * 3; ++k) o[k] = dsh[k];
        for (int k = NC * 3; k < rw; ++k) o[k] = 0.f;
      }
    }
    __syncthreads();
    dsplat::stage_out<NT>(dshs + (size_t)rw * sg0, (size_t)rw * nrows, lds);
  }
}

// ------------------------------------------------------------------------------------
// Fused head backward (round 6; dsr_head_bwd): K8 + K9 and the adapter's backward in ONE pass
// per (scene, Gaussian) = adapter row. The training step's Gaussians come from the head through
// the fused adapter (dga_adapter_fwd), so the Gaussian gradients K8 + K9 produce are consumed
// by exactly one reader, the adapter's backward; written to HBM and read back they were ~320 B
// per Gaussian (config C: 2.1 M Gaussians, ~0.67 GB). Here the adapter's forward is re-evaluated
// from the head row (dga::adapter_row_fwd: the same float operations, so mean, covariance and
// harmonics are the values the rasterizer's forward read), K8 + K9 run on them (pbwd_views: the
// same operations as k_preprocess_bwd), and their gradients feed dga::adapter_row_bwd in
// registers: dhead is bit-identical to the two-kernel path. The head rows stay staged in LDS
// across the view loop (re-read for the adapter's backward instead of held in registers).
// Rows are view-major inside a scene (G = V_ctx H W), and H W % NT == 0 (host check), so a
// workgroup's rows share one context view and one scene: camera blocks and the view loop are
// workgroup-uniform.
template <int DEG, int NSH>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(DEG <= 2 ? 4 : 1))) void k_head_bwd(dga::AdIn a, int G, int Ht, int Wt, const dsr_camera* __restrict__ cams,
                                                 const float* __restrict__ geom, const long long* __restrict__ dgeom,
                                                 const float* __restrict__ gscale,
                                                 const int32_t* __restrict__ scene_view_start,
                                                 const int32_t* __restrict__ scene_views,
                                                 const uint8_t* __restrict__ row_live, float* __restrict__ drows,
                                                 float* __restrict__ ddepth) {
  constexpr int NC = (DEG + 1) * (DEG + 1);
  static_assert(NC <= NSH, "the harmonics hold the evaluated coefficients");
  constexpr int KH = dga::Rows<NSH, true>::kHead;
  int fx_k = 0;
  const float fx_unit = grad_fx_exp(gscale, threadIdx.x & 63, fx_k) ? ldexpf(1.f, fx_k - DSR_GRAD_FRAC_BITS)
                                                                     : __builtin_nanf("");
  extern __shared__ __attribute__((aligned(16))) float lds[];  // NT * C floats: the head rows
  const size_t total = (size_t)a.BV * a.H * a.W;
  const size_t n0 = (size_t)blockIdx.x * NT;
  const int nrows = (int)min((size_t)NT, total - n0);
  const int tid = threadIdx.x, C = a.C;
  dga::Pix px{};
  const bool valid = dga::pixel_of(n0 + tid, a, px);
  const int s = (int)(n0 / (size_t)G);  // workgroup-uniform
  const int g = (int)(n0 + tid - (size_t)s * G);
  const float* cam = a.cams + n0 / ((size_t)a.H * a.W) * dga::kCamFloats;
  dsplat::stage_in<NT>(a.rows + n0 * C, (size_t)nrows * C, lds);
  __syncthreads();
  float mo[3], Cw[9], ho[3 * NSH], sc[3], q[4];
  {
    float h[KH];
#pragma unroll
    for (int k = 0; k < KH; ++k) h[k] = valid ? lds[tid * C + k] : 0.f;
    if (valid) dga::adapter_row_fwd<NSH, true>(a, px, cam, h, nullptr, mo, Cw, ho, sc, q);
  }
  // the rasterizer's inputs as it read them: mean, covariance triu, SH coefficient-major
  const F3 m0 = valid ? F3{mo[0], mo[1], mo[2]} : F3{0.f, 0.f, 0.f};
  float c60[6];
  float sh[NC * 3], dsh[NC * 3];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    constexpr int full_idx[6] = {0, 1, 2, 4, 5, 8};
    c60[k] = valid ? Cw[full_idx[k]] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < NC; ++k)
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      sh[k * 3 + ch] = valid ? ho[ch * NSH + k] : 0.f;
      dsh[k * 3 + ch] = 0.f;
    }
  float dm0 = 0.f, dm1 = 0.f, dm2 = 0.f, dop = 0.f, dcol0 = 0.f, dcol1 = 0.f, dcol2 = 0.f;
  float dc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  pbwd_views<DEG>(s, g, valid, G, Ht, Wt, m0, c60, sh, cams, geom, dgeom, fx_unit, scene_view_start, scene_views,
                  row_live, nullptr, dm0, dm1, dm2, dop, dc, dsh, dcol0, dcol1, dcol2);
  // the adapter's backward from those gradients (the values k_preprocess_bwd would have stored:
  // covariance gradient on the upper triangle, harmonics channel-major, zeros past NC)
  const float gm[3] = {dm0, dm1, dm2};
  const float gCw[9] = {dc[0], dc[1], dc[2], 0.f, dc[3], dc[4], 0.f, 0.f, dc[5]};
  float gh[3 * NSH];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch)
#pragma unroll
    for (int k = 0; k < NSH; ++k) gh[ch * NSH + k] = k < NC ? dsh[k * 3 + ch] : 0.f;
  const float z0[3] = {0.f, 0.f, 0.f}, z1[4] = {0.f, 0.f, 0.f, 0.f};
  float dh[KH];
#pragma unroll
  for (int k = 0; k < KH; ++k) dh[k] = 0.f;
  float gxy[2] = {0.f, 0.f};
  __syncthreads();  // (the head rows are read again below, not kept live across the view loop)
  if (valid) {
    float h[KH];
#pragma unroll
    for (int k = 0; k < KH; ++k) h[k] = lds[tid * C + k];
    const float z = a.depths[px.n];
    dga::adapter_row_bwd<NSH, true>(a, px, cam, h, z, gm, gCw, gh, dop, true, z0, z1, dh, gxy, ddepth);
  }
  __syncthreads();
  if (valid) {
#pragma unroll
    for (int k = 0; k < KH; ++k) lds[tid * C + k] = dh[k];
    for (int k = KH; k < C; ++k) lds[tid * C + k] = 0.f;
  }
  __syncthreads();
  dsplat::stage_out<NT>(drows + n0 * C, (size_t)nrows * C, lds);
}

// dgeom_fx -> float [rows, GS] (diagnostics / tests): the values k_preprocess_bwd consumes
// (rows of culled Gaussians: zero; their accumulator rows are never written or zeroed)
__global__ __launch_bounds__(NT) void k_dgeom_to_float(size_t rows, const float* __restrict__ geom,
                                                       const long long* __restrict__ dq,
                                                       const float* __restrict__ gscale,
                                                       const uint8_t* __restrict__ row_live, float* __restrict__ out) {
  int k = 0;
  const float unit = grad_fx_exp(gscale, threadIdx.x & 63, k) ? ldexpf(1.f, k - DSR_GRAD_FRAC_BITS) : __builtin_nanf("");
  const size_t r = (size_t)blockIdx.x * NT + threadIdx.x;
  if (r >= rows) return;
  const bool vis = (row_live == nullptr || row_live[r] != 0u) && __float_as_int(geom[r * GS + 10]) > 0;
#pragma unroll
  for (int c = 0; c < GS; ++c) out[r * GS + c] = (c < 9 && vis) ? fx_to_float(dq[r * DSR_DGEOM_WORDS + c], unit) : 0.f;
}

// pointers a segment layout needs (seg_bounds): ENDS both, fixed capacity the counts, prefix the starts
inline bool seg_ptrs_ok(const uint32_t* start, const uint32_t* count, uint32_t stride) {
  return stride == kSegEnds ? (start != nullptr && count != nullptr) : stride ? count != nullptr : start != nullptr;
}
int lds_hist_bytes(int T) { return T <= kHistLdsMax ? T * 4 : 0; }

}  // namespace

// =====================================================================================
// C ABI
// =====================================================================================
extern "C" {

uint32_t dsr_sort_lds_capacity(void) { return kSortCap; }

int dsr_preprocess_fwd(int S, int G, int V, int H, int W, int sh_degree, int M, const float* means,
                       const float* shs, const float* colors, const float* opacities,
                       const float* cov6, const dsr_camera* cams, float* geom, int32_t* radii,
                       int64_t* dgeom_zero, uint32_t* seg_count, int layout, void* stream) {
  long long* dzero = reinterpret_cast<long long*>(dgeom_zero);
  DSPLAT_REQUIRE(S > 0 && G > 0 && V > 0 && H > 0 && W > 0, "dsr_preprocess_fwd: bad sizes S=%d G=%d V=%d H=%d W=%d", S, G, V, H, W);
  DSPLAT_REQUIRE((shs != nullptr) != (colors != nullptr), "dsr_preprocess_fwd: exactly one of shs/colors must be given");
  DSPLAT_REQUIRE(shs == nullptr || (sh_degree >= 0 && sh_degree <= 3 && M >= (sh_degree + 1) * (sh_degree + 1)),
                 "dsr_preprocess_fwd: sh_degree=%d M=%d unsupported (degree 0..3, M >= (deg+1)^2)", sh_degree, M);
  DSPLAT_REQUIRE(means && opacities && cov6 && cams && geom && radii && seg_count, "dsr_preprocess_fwd: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int gx = dsplat::tiles_x(W), gy = dsplat::tiles_y(H), T = gx * gy;
  if (!(layout & kLayoutCountsZeroed))
    if (int e = dsplat::zero_async(seg_count, (size_t)V * T * 4, st, "zero seg_count")) return e;
  const int lds = lds_hist_bytes(T);
  const unsigned grid = xcd_grid((G + NT - 1) / NT, V);
  const int deg = shs ? sh_degree : -1;
#define DSR_PRE(D)                                                                                              \
  do {                                                                                                         \
    if (layout & kLayoutExactBinning)                                                                          \
      k_preprocess<D, true><<<grid, NT, lds, st>>>(G, V, H, W, gx, gy, M, means, shs, colors, opacities, cov6, \
                                                   cams, geom, radii, dzero, seg_count, lds > 0, layout);      \
    else                                                                                                       \
      k_preprocess<D, false><<<grid, NT, lds, st>>>(G, V, H, W, gx, gy, M, means, shs, colors, opacities,      \
                                                    cov6, cams, geom, radii, dzero, seg_count, lds > 0, layout); \
  } while (0)
  switch (deg) {
    case -1: DSR_PRE(-1); break;
    case 0: DSR_PRE(0); break;
    case 1: DSR_PRE(1); break;
    case 2: DSR_PRE(2); break;
    default: DSR_PRE(3); break;
  }
#undef DSR_PRE
  return dsplat::check_launch("k_preprocess");
}

}  // extern "C"
namespace {
int project_bin_impl(const char* who, int S, int G, int V, int H, int W, int sh_degree, int M, const float* means,
                     const float* shs, const float* colors, const float* opacities, const float* cov6,
                     dsr_camera* cams, const CamIn* ci, float* geom, int32_t* radii, long long* dzero,
                     uint32_t* seg_count, uint64_t* keys, uint32_t cap, int layout, void* stream) {
  DSPLAT_REQUIRE(S > 0 && G > 0 && V > 0 && H > 0 && W > 0, "%s: bad sizes S=%d G=%d V=%d H=%d W=%d", who, S, G, V, H, W);
  DSPLAT_REQUIRE((shs != nullptr) != (colors != nullptr), "%s: exactly one of shs/colors must be given", who);
  DSPLAT_REQUIRE(shs == nullptr || (sh_degree >= 0 && sh_degree <= 3 && M >= (sh_degree + 1) * (sh_degree + 1)),
                 "%s: sh_degree=%d M=%d unsupported (degree 0..3, M >= (deg+1)^2)", who, sh_degree, M);
  DSPLAT_REQUIRE(means && opacities && cov6 && cams && geom && radii && seg_count && keys, "%s: null pointer", who);
  const int gx = dsplat::tiles_x(W), gy = dsplat::tiles_y(H), T = gx * gy;
  DSPLAT_REQUIRE(T <= kHistLdsMax, "%s: %d tiles per view exceed the LDS histogram (%d)", who, T, kHistLdsMax);
  if (cap == 0) cap = (uint32_t)G;
  DSPLAT_REQUIRE(cap <= (uint32_t)G, "%s: segment capacity %u above G = %d", who, cap, G);
  DSPLAT_REQUIRE((uint64_t)V * T * cap < (1ull << 32), "%s: V*tiles*capacity must fit 32-bit key offsets", who);
  hipStream_t st = (hipStream_t)stream;
  if (!(layout & kLayoutCountsZeroed))
    if (int e = dsplat::zero_async(seg_count, (size_t)V * T * 4, st, "zero seg_count")) return e;
  const unsigned grid = xcd_grid((G + NT - 1) / NT, V);
  const int deg = shs ? sh_degree : -1;
#define DSR_PB(D)                                                                                              \
  do {                                                                                                         \
    if (ci && !(layout & kLayoutRectBinning))                                                                  \
      k_project_emit<D, true, true><<<grid, NT, T * 4, st>>>(G, V, H, W, gx, gy, M, means, shs, colors,         \
                                                             opacities, cov6, cams, geom, radii, dzero, seg_count,     \
                                                             keys, cap, layout, *ci);                                \
    else if (ci)                                                                                               \
      k_project_emit<D, true, false><<<grid, NT, T * 4, st>>>(G, V, H, W, gx, gy, M, means, shs, colors,        \
                                                              opacities, cov6, cams, geom, radii, dzero, seg_count,    \
                                                              keys, cap, layout, *ci);                               \
    else if (layout & kLayoutExactBinning)                                                                     \
      k_project_emit<D, false, true><<<grid, NT, T * 4, st>>>(G, V, H, W, gx, gy, M, means, shs, colors,        \
                                                              opacities, cov6, cams, geom, radii, dzero, seg_count,    \
                                                              keys, cap, layout, CamIn{});                           \
    else                                                                                                       \
      k_project_emit<D, false, false><<<grid, NT, T * 4, st>>>(G, V, H, W, gx, gy, M, means, shs, colors,       \
                                                               opacities, cov6, cams, geom, radii, dzero, seg_count,   \
                                                               keys, cap, layout, CamIn{});                          \
  } while (0)
  switch (deg) {
    case -1: DSR_PB(-1); break;
    case 0: DSR_PB(0); break;
    case 1: DSR_PB(1); break;
    case 2: DSR_PB(2); break;
    default: DSR_PB(3); break;
  }
#undef DSR_PB
  return dsplat::check_launch("k_project_emit");
}
}  // namespace
extern "C" {

int dsr_project_bin(int S, int G, int V, int H, int W, int sh_degree, int M, const float* means, const float* shs,
                    const float* colors, const float* opacities, const float* cov6, const dsr_camera* cams,
                    float* geom, int32_t* radii, int64_t* dgeom_zero, uint32_t* seg_count, uint64_t* keys, int layout,
                    void* stream) {
  return project_bin_impl("dsr_project_bin", S, G, V, H, W, sh_degree, M, means, shs, colors, opacities, cov6,
                          const_cast<dsr_camera*>(cams), nullptr, geom, radii,
                          reinterpret_cast<long long*>(dgeom_zero), seg_count, keys, (uint32_t)G, layout, stream);
}

int dsr_project_bin_cameras(int S, int G, int V, int H, int W, int sh_degree, int M, const float* means,
                            const float* shs, const float* colors, const float* opacities, const float* cov6,
                            const float* extrinsics, const float* intrinsics, const float* near, const float* far,
                            const float* bg, const int32_t* view_scene, int scale_invariant, dsr_camera* cams,
                            float* geom, int32_t* radii, int64_t* dgeom_zero, uint32_t* seg_count, uint64_t* keys,
                            uint32_t seg_capacity, int layout, void* stream) {
  if (extrinsics == nullptr) {
    // caller-supplied camera block: cams [V] is an input (e.g. the reference wrapper's own
    // settings packed by the caller); the same kernel without its in-kernel camera set-up,
    // binning exact unless DSR_LAYOUT_RECT_BINNING (as with the set-up)
    const int lay = (layout & kLayoutRectBinning) ? (layout & ~kLayoutExactBinning) : (layout | kLayoutExactBinning);
    return project_bin_impl("dsr_project_bin_cameras(camera block)", S, G, V, H, W, sh_degree, M, means, shs, colors,
                            opacities, cov6, cams, nullptr, geom, radii, reinterpret_cast<long long*>(dgeom_zero),
                            seg_count, keys, seg_capacity, lay, stream);
  }
  DSPLAT_REQUIRE(intrinsics && near && far && bg && view_scene, "dsr_project_bin_cameras: null camera input");
  const CamIn ci{extrinsics, intrinsics, near, far, bg, view_scene, scale_invariant};
  return project_bin_impl("dsr_project_bin_cameras", S, G, V, H, W, sh_degree, M, means, shs, colors, opacities,
                          cov6, cams, &ci, geom, radii, reinterpret_cast<long long*>(dgeom_zero), seg_count, keys,
                          seg_capacity, layout, stream);
}

int dsr_bin_scan(int V, int H, int W, const uint32_t* seg_count, uint32_t* seg_start, uint32_t* seg_cursor,
                 uint32_t* totals, void* stream) {
  DSPLAT_REQUIRE(V > 0 && H > 0 && W > 0, "dsr_bin_scan: bad sizes");
  DSPLAT_REQUIRE(seg_count && seg_start && seg_cursor && totals, "dsr_bin_scan: null pointer");
  const int n = V * dsplat::tiles_x(W) * dsplat::tiles_y(H);
  k_scan<<<1, 1024, 0, (hipStream_t)stream>>>(n, seg_count, seg_start, seg_cursor, totals);
  return dsplat::check_launch("k_scan");
}

int dsr_bin_scatter(int G, int V, int H, int W, const float* geom, uint32_t* seg_cursor, uint64_t* keys,
                    int layout, void* stream) {
  DSPLAT_REQUIRE(G > 0 && V > 0 && H > 0 && W > 0, "dsr_bin_scatter: bad sizes");
  DSPLAT_REQUIRE(geom && seg_cursor, "dsr_bin_scatter: null pointer");
  const int gx = dsplat::tiles_x(W), gy = dsplat::tiles_y(H);
  const int lds = lds_hist_bytes(gx * gy);
  const unsigned grid = xcd_grid((G + NT - 1) / NT, V);
  if (layout & kLayoutExactBinning)
    k_scatter<true><<<grid, NT, lds, (hipStream_t)stream>>>(G, V, gx, gy, geom, seg_cursor, keys, lds > 0);
  else
    k_scatter<false><<<grid, NT, lds, (hipStream_t)stream>>>(G, V, gx, gy, geom, seg_cursor, keys, lds > 0);
  return dsplat::check_launch("k_scatter");
}

int dsr_cut_superblock(int H, int W) {
  if (H <= 0 || W <= 0) return 0;
  return cut_superblock(dsplat::tiles_x(W), dsplat::tiles_y(H));
}

int dsr_preprocess_cut(int S, int G, int V, int H, int W, int sh_degree, int M, const float* means,
                       const float* shs, const float* colors, const float* opacities, const float* cov6,
                       const dsr_camera* cams, float* geom, int32_t* radii, int64_t* dgeom_zero,
                       uint32_t* seg_count, uint32_t* depth_hist, uint32_t* cut_rec, int layout, void* stream) {
  long long* dzero = reinterpret_cast<long long*>(dgeom_zero);
  DSPLAT_REQUIRE(S > 0 && G > 0 && V > 0 && H > 0 && W > 0, "dsr_preprocess_cut: bad sizes S=%d G=%d V=%d H=%d W=%d", S, G, V, H, W);
  DSPLAT_REQUIRE((shs != nullptr) != (colors != nullptr), "dsr_preprocess_cut: exactly one of shs/colors must be given");
  DSPLAT_REQUIRE(shs == nullptr || (sh_degree >= 0 && sh_degree <= 3 && M >= (sh_degree + 1) * (sh_degree + 1)),
                 "dsr_preprocess_cut: sh_degree=%d M=%d unsupported (degree 0..3, M >= (deg+1)^2)", sh_degree, M);
  DSPLAT_REQUIRE(means && opacities && cov6 && cams && geom && radii && seg_count && depth_hist,
                 "dsr_preprocess_cut: null pointer");
  const int gx = dsplat::tiles_x(W), gy = dsplat::tiles_y(H), T = gx * gy;
  const int sb = cut_superblock(gx, gy);
  DSPLAT_REQUIRE(sb > 0, "dsr_preprocess_cut: %dx%d tiles exceed the LDS histograms", gx, gy);
  const int nsb = ((gx + sb - 1) / sb) * ((gy + sb - 1) / sb);
  DSPLAT_REQUIRE(cut_rec == nullptr || (gx <= 255 && gy <= 255),
                 "dsr_preprocess_cut: cut_rec needs at most 255 tiles per axis");
  const bool lazy = (layout & kLayoutDeferGeom) != 0;
  DSPLAT_REQUIRE(!lazy || (cut_rec != nullptr && dgeom_zero == nullptr),
                 "dsr_preprocess_cut: DSR_LAYOUT_DEFER_GEOM needs cut_rec and no dgeom_zero");
  hipStream_t st = (hipStream_t)stream;
  if (!(layout & kLayoutCountsZeroed))
    if (int e = dsplat::zero_async(seg_count, (size_t)V * T * 4, st, "zero seg_count")) return e;
  if (int e = dsplat::zero_async(depth_hist, (size_t)V * nsb * kCutBuckets * 4, st, "zero depth_hist")) return e;
  constexpr int kNTH = 512;
  const size_t lds = (size_t)((gx + 1) * (gy + 1) + nsb * kCutBuckets) * 4;
  // persistent grid: about the resident workgroup count (LDS-limited: the histograms plus the
  // kernel's static arrays), split evenly over views
  constexpr size_t kStatic = (size_t)(kNTH / 64) * (sizeof(WaveRects) + 3 * 64 * sizeof(uint32_t));
  const int per_cu = max(1, min(4, (int)((160 * 1024) / (lds + kStatic))));
  const int nblk = (G + kNTH - 1) / kNTH;
  const int per_view = max(1, min(nblk, (256 * per_cu) / V));
  const int deg = shs ? sh_degree : -1;
#define DSR_PC(D, L)                                                                                         \
  do {                                                                                                       \
    if (int e = dsplat::ensure_dyn_lds((const void*)k_preprocess_cut<D, kNTH, L>, kCutLdsWordsMax * 4,           \
                                       "hipFuncSetAttribute(k_preprocess_cut)"))                             \
      return e;                                                                                              \
    k_preprocess_cut<D, kNTH, L><<<xcd_grid(per_view, V), kNTH, lds, st>>>(                                  \
        G, V, H, W, gx, gy, M, means, shs, colors, opacities, cov6, cams, geom, radii, dzero, seg_count,      \
        depth_hist,                                                                                          \
        reinterpret_cast<uint2*>(cut_rec), per_view, layout);                                                \
  } while (0)
#define DSR_PC2(D)          \
  do {                      \
    if (lazy)               \
      DSR_PC(D, true);      \
    else                    \
      DSR_PC(D, false);     \
  } while (0)
  switch (deg) {
    case -1: DSR_PC2(-1); break;
    case 0: DSR_PC2(0); break;
    case 1: DSR_PC2(1); break;
    case 2: DSR_PC2(2); break;
    default: DSR_PC2(3); break;
  }
#undef DSR_PC2
#undef DSR_PC
  return dsplat::check_launch("k_preprocess_cut");
}

int dsr_bin_cutoff(int V, int H, int W, const uint32_t* depth_hist, uint32_t prefix, uint32_t* cut, void* stream) {
  DSPLAT_REQUIRE(V > 0 && H > 0 && W > 0, "dsr_bin_cutoff: bad sizes");
  DSPLAT_REQUIRE(depth_hist && cut, "dsr_bin_cutoff: null pointer");
  const int gx = dsplat::tiles_x(W), gy = dsplat::tiles_y(H);
  const int sb = cut_superblock(gx, gy);
  DSPLAT_REQUIRE(sb > 0, "dsr_bin_cutoff: %dx%d tiles exceed the LDS histograms", gx, gy);
  const int items = V * ((gx + sb - 1) / sb) * ((gy + sb - 1) / sb);
  k_bin_cutoff<<<(unsigned)((items + 3) / 4), 256, 0, (hipStream_t)stream>>>(V, gx, gy, depth_hist, prefix, cut);
  return dsplat::check_launch("k_bin_cutoff");
}

int dsr_bin_scatter_cut(int G, int V, int H, int W, const float* geom, uint32_t* seg_cursor, uint64_t* keys,
                        const uint32_t* cut, int tail, const uint32_t* seg_overflow, const uint32_t* cut_rec,
                        uint32_t* survivors, uint32_t* survivor_count, const uint32_t* totals, uint64_t keys_capacity,
                        void* stream) {
  DSPLAT_REQUIRE(G > 0 && V > 0 && H > 0 && W > 0, "dsr_bin_scatter_cut: bad sizes");
  DSPLAT_REQUIRE(geom && seg_cursor && keys && cut && (!tail || seg_overflow), "dsr_bin_scatter_cut: null pointer");
  DSPLAT_REQUIRE((survivors == nullptr) == (survivor_count == nullptr) && (survivors == nullptr || cut_rec),
                 "dsr_bin_scatter_cut: survivors and survivor_count go together and need cut_rec");
  const int gx = dsplat::tiles_x(W), gy = dsplat::tiles_y(H);
  DSPLAT_REQUIRE(cut_superblock(gx, gy) > 0, "dsr_bin_scatter_cut: %dx%d tiles exceed the LDS histograms", gx, gy);
  constexpr int kNTH = kScatterCutNTH;
  const int per_view = scatter_cut_per_view(G, V);
  k_scatter_cut<kNTH><<<xcd_grid(per_view, V), kNTH, 0, (hipStream_t)stream>>>(G, V, gx, gy, geom, seg_cursor,
                                                                                  keys, cut, tail, seg_overflow,
                                                                                  reinterpret_cast<const uint2*>(cut_rec),
                                                                                  per_view, survivors, survivor_count,
                                                                                  totals, keys_capacity);
  return dsplat::check_launch("k_scatter_cut");
}

int dsr_survivor_layout(int G, int V, int64_t* slots, int* counters) {
  DSPLAT_REQUIRE(G > 0 && V > 0 && slots && counters, "dsr_survivor_layout: bad arguments");
  const int pv = scatter_cut_per_view(G, V);
  *counters = V * pv;
  *slots = (int64_t)V * pv * (int64_t)survivor_slice(G, V);
  return 0;
}

int dsr_project_survivors(int S, int G, int V, int H, int W, int sh_degree, int M, const float* means,
                          const float* shs, const float* colors, const float* opacities, const float* cov6,
                          const dsr_camera* cams, const uint32_t* survivors, const uint32_t* survivor_count,
                          float* geom, int32_t* radii, int64_t* dgeom_zero, uint8_t* row_live, int layout,
                          void* stream) {
  DSPLAT_REQUIRE(S > 0 && G > 0 && V > 0 && H > 0 && W > 0, "dsr_project_survivors: bad sizes S=%d G=%d V=%d H=%d W=%d", S, G, V, H, W);
  DSPLAT_REQUIRE((shs != nullptr) != (colors != nullptr), "dsr_project_survivors: exactly one of shs/colors must be given");
  DSPLAT_REQUIRE(shs == nullptr || (sh_degree >= 0 && sh_degree <= 3 && M >= (sh_degree + 1) * (sh_degree + 1)),
                 "dsr_project_survivors: sh_degree=%d M=%d unsupported (degree 0..3, M >= (deg+1)^2)", sh_degree, M);
  DSPLAT_REQUIRE(means && opacities && cov6 && cams && survivors && survivor_count && geom && radii,
                 "dsr_project_survivors: null pointer");
  const int gx = dsplat::tiles_x(W), gy = dsplat::tiles_y(H);
  static_assert(NT == kScatterCutNTH, "one survivor slice per scatter workgroup");
  const int per_view = scatter_cut_per_view(G, V);
  const int deg = shs ? sh_degree : -1;
  hipStream_t st = (hipStream_t)stream;
#define DSR_PS(D)                                                                                            \
  k_project_survivors<D><<<xcd_grid(per_view, V), NT, 0, st>>>(G, V, H, W, gx, gy, M, means, shs, colors, \
                                                                   opacities, cov6, cams, survivors,         \
                                                                   survivor_count, geom, radii,              \
                                                                   reinterpret_cast<long long*>(dgeom_zero), \
                                                                   row_live, per_view, layout)
  switch (deg) {
    case -1: DSR_PS(-1); break;
    case 0: DSR_PS(0); break;
    case 1: DSR_PS(1); break;
    case 2: DSR_PS(2); break;
    default: DSR_PS(3); break;
  }
#undef DSR_PS
  return dsplat::check_launch("k_project_survivors");
}

size_t dsr_bin_sort_workspace_size(int V, int H, int W, uint32_t max_count) {
  if (max_count <= kSortCap) return 0;
  const size_t nseg = (size_t)V * dsplat::tiles_x(W) * dsplat::tiles_y(H);
  return nseg * (size_t)split_groups(max_count) * 2 * sizeof(uint32_t);
}

int dsr_workspace_size(int G, int H, int W, int n_views, uint64_t key_budget, dsr_workspace* out) {
  DSPLAT_REQUIRE(G > 0 && H > 0 && W > 0 && n_views > 0 && out, "dsr_workspace_size: bad arguments");
  const uint64_t V = (uint64_t)n_views, T = (uint64_t)dsplat::tiles_x(W) * dsplat::tiles_y(H);
  const uint64_t HW = (uint64_t)H * W;
  dsr_workspace ws{};
  ws.tiles = (int32_t)T;
  ws.cams_bytes = V * sizeof(dsr_camera);
  ws.geom_bytes = V * G * GS * 4;
  ws.radii_bytes = V * G * 4;
  ws.seg_count_bytes = V * T * 4;
  ws.seg_start_bytes = (V * T + 1) * 4;
  // the same test as the Python layer (raster.forward_raw): worst case V*T*G keys + as much
  // scratch within the budget, tiles within the LDS histogram, offsets within 32 bits
  const uint64_t worst = V * T * (uint64_t)G;
  ws.fixed_capacity = (worst * 16 <= key_budget && T <= (uint64_t)kHistLdsMax && worst < (1ull << 32)) ? 1 : 0;
  ws.keys_bytes = ws.fixed_capacity ? worst * 8 : 0;
  ws.scratch_bytes = ws.keys_bytes;
  ws.sort_ws_bytes = dsr_bin_sort_workspace_size(n_views, H, W, (uint32_t)G);
  ws.color_bytes = V * 3 * HW * 4;
  ws.final_T_bytes = V * HW * 4;
  ws.n_contrib_bytes = V * HW * 4;
  ws.dgeom_bytes = (uint64_t)V * G * DSR_DGEOM_WORDS * 8;  // int64 fixed point
  ws.total_bytes = ws.cams_bytes + ws.geom_bytes + ws.radii_bytes + ws.seg_count_bytes + ws.seg_start_bytes +
                   ws.keys_bytes + ws.scratch_bytes + ws.sort_ws_bytes + ws.color_bytes + ws.final_T_bytes +
                   ws.n_contrib_bytes + ws.dgeom_bytes;
  *out = ws;
  return 0;
}

}  // extern "C"
namespace {
// dynamic LDS above 64 KiB must be opted into, per kernel instantiation and device
template <int KM, int NTH_>
int sort_lds_attr() {
  if (sort_lds_bytes<KM, NTH_>() <= 65536) return 0;
  return dsplat::ensure_dyn_lds((const void*)k_sort_lds<KM, NTH_>, sort_lds_bytes<KM, NTH_>(),
                                "hipFuncSetAttribute(k_sort_lds)");
}
}  // namespace
extern "C" {

int dsr_bin_sort(int G, int V, int H, int W, const uint32_t* seg_start, const uint32_t* seg_count,
                 uint32_t seg_stride, uint64_t* keys, uint64_t* scratch, uint32_t max_count, void* workspace,
                 uint32_t prefix, uint32_t* seg_sorted, const uint32_t* seg_filter, void* stream) {
  DSPLAT_REQUIRE(G > 0 && V > 0 && H > 0 && W > 0, "dsr_bin_sort: bad sizes");
  DSPLAT_REQUIRE(keys != nullptr && seg_ptrs_ok(seg_start, seg_count, seg_stride),
                 "dsr_bin_sort: null pointer");
  DSPLAT_REQUIRE(scratch != nullptr || (max_count > 0 && max_count <= kSortCap),
                 "dsr_bin_sort: without scratch, max_count (%u) must bound every segment and be <= %u", max_count,
                 kSortCap);
  DSPLAT_REQUIRE(prefix == 0 || seg_sorted != nullptr, "dsr_bin_sort: prefix mode needs seg_sorted");
  DSPLAT_REQUIRE(seg_filter == nullptr || scratch != nullptr, "dsr_bin_sort: seg_filter needs scratch");
  hipStream_t st = (hipStream_t)stream;
  const int nseg = V * dsplat::tiles_x(W) * dsplat::tiles_y(H);
  int id_bits = 0;
  while (id_bits < 32 && ((uint64_t)1 << id_bits) < (uint64_t)G) ++id_bits;
  const uint32_t want = max_count ? max_count : kSortCap;
  // segments above the LDS capacity: sorted in this launch through HBM unless they are
  // known to be large (max_count > kSortCap): then the MSD split + grouped LDS sort take them
  const bool big_known = scratch != nullptr && max_count > kSortCap && seg_filter == nullptr;
  const int big_here = scratch != nullptr && !big_known;
  DSPLAT_REQUIRE(!big_known || workspace != nullptr,
                 "dsr_bin_sort: max_count %u > %u needs workspace (dsr_bin_sort_workspace_size)", max_count, kSortCap);
  // dynamic LDS above 64 KiB must be opted into (per device; remembered by ensure_dyn_lds)
  for (const auto& a : {std::make_pair((const void*)k_sort_lds<32>, sort_lds_bytes<32>()),
                        std::make_pair((const void*)k_sort_lds<16>, sort_lds_bytes<16>()),
                        std::make_pair((const void*)k_sort_lds<kSortCap / kSortNT, kSortNT>,
                                       sort_lds_bytes<kSortCap / kSortNT, kSortNT>()),
                        std::make_pair((const void*)k_msd_split<kSplitNT, kSplitKPT>, split_lds_bytes())})
    if (int e = dsplat::ensure_dyn_lds(a.first, a.second, "hipFuncSetAttribute(k_sort_lds / k_msd_split)")) return e;
  uint32_t cap;
#define DSR_SORT_LDS(KM, NTH_, FILT)                                                                        \
  do {                                                                                                      \
    if (int e = sort_lds_attr<KM, NTH_>()) return e;                                                        \
    cap = (uint32_t)(KM) * (NTH_);                                                                          \
    k_sort_lds<KM, NTH_><<<nseg, NTH_, sort_lds_bytes<KM, NTH_>(), st>>>(seg_start, seg_count, seg_stride,   \
                                                                          keys, scratch, id_bits, big_here, \
                                                                          FILT, seg_sorted);                \
  } while (0)
  if (seg_filter) {  // the tail pass: the few flagged segments, in full (k_sort_flagged)
    constexpr int kFlagNT = 1024;
    k_sort_flagged<kFlagNT><<<(unsigned)min(nseg, 512), kFlagNT, 0, st>>>(nseg, seg_start, seg_count, seg_stride, keys,
                                                                       scratch, id_bits, seg_filter, seg_sorted);
    return dsplat::check_launch("k_sort_flagged");
  }
  if (big_known) {  // small segments in LDS now, the rest split below
    DSR_SORT_LDS(16, NT, nullptr);
  } else if (want <= kSortNT * 4) {
    DSR_SORT_LDS(4, kSortNT, nullptr);
  } else if (want <= kSortNT * 8) {
    DSR_SORT_LDS(8, kSortNT, nullptr);
  } else if (want <= kSortNT * 16 && kSortNT * 16 < kSortCap) {
    DSR_SORT_LDS(16, kSortNT, nullptr);
  } else {
    DSR_SORT_LDS(kSortCap / kSortNT, kSortNT, nullptr);
  }
#undef DSR_SORT_LDS
  if (int e = dsplat::check_launch("k_sort_lds")) return e;
  if (big_known) {
    uint32_t pfx = 0;
    int gmax = split_groups(max_count);
    if (prefix) {  // a multiple of the group half-size, at least the LDS capacity
      pfx = max(cap, (prefix + kGroupHalf - 1) / kGroupHalf * kGroupHalf);
      if (pfx < max_count) gmax = min(gmax, (int)(pfx / kGroupHalf) + 1);
      else pfx = 0;
    }
    uint32_t* groups = static_cast<uint32_t*>(workspace);
    k_msd_split<kSplitNT, kSplitKPT><<<nseg, kSplitNT, split_lds_bytes(), st>>>(
        seg_start, seg_count, seg_stride, keys, scratch, cap, groups, gmax, pfx, seg_sorted);
    if (int e = dsplat::check_launch("k_msd_split")) return e;
    k_sort_groups<16><<<(unsigned)(nseg * gmax), NT, sort_lds_bytes<16>(), st>>>(groups, keys, scratch, id_bits);
    if (int e = dsplat::check_launch("k_sort_groups")) return e;
  }
  return 0;
}

int dsr_render_fwd(int G, int V, int H, int W, const dsr_camera* cams, const float* geom,
                   const uint32_t* seg_start, const uint32_t* seg_count, uint32_t seg_stride, const uint64_t* keys,
                   const uint32_t* seg_sorted, uint32_t* seg_overflow, const uint32_t* seg_filter, float* out_color,
                   float* final_T, uint32_t* n_contrib, void* stream) {
  DSPLAT_REQUIRE(seg_sorted == nullptr || seg_overflow != nullptr, "dsr_render_fwd: seg_sorted needs seg_overflow");
  DSPLAT_REQUIRE(G > 0 && V > 0 && H > 0 && W > 0, "dsr_render_fwd: bad sizes");
  DSPLAT_REQUIRE(cams && geom && seg_ptrs_ok(seg_start, seg_count, seg_stride) && out_color && final_T &&
                     n_contrib,
                 "dsr_render_fwd: null pointer");
  const int gx = dsplat::tiles_x(W), gy = dsplat::tiles_y(H);
  if (seg_filter) {  // the tail pass: only the flagged tiles (their lists complete and sorted)
    DSPLAT_REQUIRE(seg_sorted == nullptr && seg_overflow == nullptr,
                   "dsr_render_fwd: seg_filter goes without seg_sorted / seg_overflow");
    const int nseg = V * gx * gy;
    k_render_flagged<<<(unsigned)min(nseg, 2048), NT, 0, (hipStream_t)stream>>>(
        V, G, H, W, gx, gx * gy, cams, geom, seg_start, seg_count, seg_stride, keys, seg_filter, out_color, final_T,
        n_contrib);
    return dsplat::check_launch("k_render_flagged");
  }
  dim3 grid(gx, gy, V);
  k_render_fwd<<<grid, NT, 0, (hipStream_t)stream>>>(G, H, W, gx, gx * gy, cams, geom, seg_start, seg_count,
                                                     seg_stride, keys, seg_sorted, seg_overflow, out_color, final_T,
                                                     n_contrib);
  return dsplat::check_launch("k_render_fwd");
}

int dsr_sort_render(int G, int V, int H, int W, const dsr_camera* cams, const float* geom,
                    const uint32_t* seg_start, uint32_t* seg_count, uint32_t seg_stride, uint64_t* keys,
                    uint64_t* scratch, uint64_t* spill_keys, int write_keys, int clear_counts,
                    uint32_t max_count_hint, int binning_layout, float* out_color, float* final_T,
                    uint32_t* n_contrib, uint32_t* seg_overflow, void* stream) {
  DSPLAT_REQUIRE(!clear_counts || seg_stride > 0, "dsr_sort_render: clear_counts needs the fixed-capacity layout");
  DSPLAT_REQUIRE(seg_overflow == nullptr || (seg_stride == kSegEnds && seg_start != nullptr),
                 "dsr_sort_render: seg_overflow needs the DSR_SEG_ENDS layout (depth cut)");
  // write_keys with bounded segments (seg_stride < G): a tile whose count exceeds the stride is
  // rebuilt; its sorted list goes to spill_keys (G slots per segment) when given
  DSPLAT_REQUIRE(spill_keys == nullptr || (write_keys && seg_stride != 0u && seg_stride != kSegEnds),
                 "dsr_sort_render: spill_keys needs write_keys and the fixed-capacity layout");
  DSPLAT_REQUIRE(G > 0 && V > 0 && H > 0 && W > 0, "dsr_sort_render: bad sizes");
  DSPLAT_REQUIRE(cams && geom && keys && scratch && seg_ptrs_ok(seg_start, seg_count, seg_stride) && out_color &&
                     final_T,
                 "dsr_sort_render: null pointer");
  // LDS size class from the caller's hint of the largest segment (earlier calls' counts):
  // smaller key arrays leave room for more resident workgroups (16: 3 per CU, 12 and 8: 4 per
  // CU at <= 128 VGPRs). A segment above the chosen class is still sorted exactly, through
  // `scratch` (slower), so the hint only affects speed.
  struct Cls {
    uint32_t cap;
    const void* k[2];  // LAST = false, true
    size_t lds;
  };
  static const Cls cls[3] = {
      {NT * 8u, {(const void*)k_sort_render<8, false, 12, 4>, (const void*)k_sort_render<8, true, 12, 4>},
       sort_render_lds_bytes<8, 12>()},
      {NT * 12u, {(const void*)k_sort_render<12, false, 12, 4>, (const void*)k_sort_render<12, true, 12, 4>},
       sort_render_lds_bytes<12, 12>()},
      {NT * 16u, {(const void*)k_sort_render<16, false, 13, 3>, (const void*)k_sort_render<16, true, 13, 3>},
       sort_render_lds_bytes<16, 13>()}};
  // 2048-key class at 5 waves per EU (31 KB: 5 WGs per CU at <= 96 VGPRs, some spills): wins
  // once the grid fills the chip several times over (kbench, inference at 12 / 24 views: -2 /
  // -3 %; with n_contrib at 16 / 64 views: -5 / -6 %), loses on one scene's 768 tiles (+5 %)
  constexpr int kWide = 2048;  // (view, tile) segments from which the 5-wave kernels are used
  const void* k8w5[2] = {(const void*)k_sort_render<8, false, 12, 5>, (const void*)k_sort_render<8, true, 12, 5>};
  for (const Cls& c : cls)
    for (const void* f : c.k)
      if (int e = dsplat::ensure_dyn_lds(f, c.lds, "hipFuncSetAttribute(k_sort_render)")) return e;
  for (const void* f : k8w5)
    if (int e = dsplat::ensure_dyn_lds(f, cls[0].lds, "hipFuncSetAttribute(k_sort_render)")) return e;
  int ci = 0;
  while (ci < 2 && (max_count_hint == 0 || max_count_hint > cls[ci].cap)) ++ci;
  int id_bits = 0;
  while (id_bits < 32 && ((uint64_t)1 << id_bits) < (uint64_t)G) ++id_bits;
  const int gx = dsplat::tiles_x(W), gy = dsplat::tiles_y(H);
  dim3 grid(gx, gy, V);
  const int T = gx * gy;
  size_t lds = cls[ci].lds;
  // A/B timing knob (DSPLAT_SR_LDS: dynamic LDS bytes of the launch, at least the class's): a
  // larger request caps the resident sort workgroups per CU and leaves room for another
  // kernel's workgroups (round-6 overlap experiment)
  static const size_t lds_req = [] {
    const char* e = getenv("DSPLAT_SR_LDS");
    return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)0;
  }();
  if (lds_req > lds && lds_req <= 64 * 1024) {
    lds = lds_req;
    for (const Cls& c : cls)
      for (const void* f : c.k)
        if (int e = dsplat::ensure_dyn_lds(f, lds, "hipFuncSetAttribute(k_sort_render)")) return e;
    for (const void* f : k8w5)
      if (int e = dsplat::ensure_dyn_lds(f, lds, "hipFuncSetAttribute(k_sort_render)")) return e;
  }
  hipStream_t st = (hipStream_t)stream;
#define DSR_SR_LAUNCH(K, L, NB, WP)                                                                          \
  k_sort_render<K, L, NB, WP><<<grid, NT, lds, st>>>(G, H, W, gx, T, cams, geom, seg_start, seg_count, seg_stride, \
                                                     keys, scratch, spill_keys, id_bits, write_keys, clear_counts, \
                                                     !(binning_layout & kLayoutRectBinning), out_color, final_T,   \
                                                     n_contrib, seg_overflow)
  // n_contrib is optional (inference: LAST = false)
  const bool wide = (int64_t)V * T >= kWide;
  switch (ci * 2 + (n_contrib ? 1 : 0)) {
    case 0:
      if (wide)
        DSR_SR_LAUNCH(8, false, 12, 5);
      else
        DSR_SR_LAUNCH(8, false, 12, 4);
      break;
    case 1:
      if (wide)
        DSR_SR_LAUNCH(8, true, 12, 5);
      else
        DSR_SR_LAUNCH(8, true, 12, 4);
      break;
    case 2: DSR_SR_LAUNCH(12, false, 12, 4); break;
    case 3: DSR_SR_LAUNCH(12, true, 12, 4); break;
    case 4: DSR_SR_LAUNCH(16, false, 13, 3); break;
    default: DSR_SR_LAUNCH(16, true, 13, 3); break;
  }
#undef DSR_SR_LAUNCH
  return dsplat::check_launch("k_sort_render");
}

int dsr_grad_scale(int V, int H, int W, const float* dL_dpix, float* grad_scale, void* stream) {
  DSPLAT_REQUIRE(V > 0 && H > 0 && W > 0, "dsr_grad_scale: bad sizes");
  DSPLAT_REQUIRE(dL_dpix && grad_scale, "dsr_grad_scale: null pointer");
  DSPLAT_REQUIRE(((uintptr_t)dL_dpix & 15) == 0, "dsr_grad_scale: dL_dpix must be 16-byte aligned");
  k_grad_scale<<<kGradBlocks, 256, 0, (hipStream_t)stream>>>((size_t)V * 3 * H * W, dL_dpix, grad_scale);
  return dsplat::check_launch("k_grad_scale");
}

int dsr_render_bwd(int G, int V, int H, int W, const dsr_camera* cams, const float* geom,
                   const uint32_t* seg_start, const uint32_t* seg_count, uint32_t seg_stride, const uint64_t* keys,
                   const uint64_t* spill_keys, const float* final_T, const uint32_t* n_contrib,
                   const float* dL_dpix, const float* grad_scale, int64_t* dgeom_fx, void* stream) {
  DSPLAT_REQUIRE(G > 0 && V > 0 && H > 0 && W > 0, "dsr_render_bwd: bad sizes");
  DSPLAT_REQUIRE(cams && geom && seg_ptrs_ok(seg_start, seg_count, seg_stride) && final_T && n_contrib &&
                     dL_dpix && grad_scale && dgeom_fx,
                 "dsr_render_bwd: null pointer");
  DSPLAT_REQUIRE(spill_keys == nullptr || (seg_stride != 0u && seg_stride != kSegEnds),
                 "dsr_render_bwd: spill_keys needs the fixed-capacity layout");
  long long* dgeom = reinterpret_cast<long long*>(dgeom_fx);
  const int gx = dsplat::tiles_x(W), gy = dsplat::tiles_y(H);
  dim3 grid(gx, gy, V);
  constexpr int64_t kWideBwd = 8192;  // (view, tile) segments from which WPE = 5 pays
  // DSPLAT_K7_SUBTILE=1: the sub-tile-wave kernel (A/B timing, and the test that checks the two
  // forms against each other; read per call)
  const char* e7 = getenv("DSPLAT_K7_SUBTILE");
  const bool tile_wave = !(e7 && e7[0] && e7[0] != '0');
  if (tile_wave) {
    k_render_bwd_tw<DSR_K7TW_WPE, DSR_K7TW_NS><<<grid, 64 * (4 / DSR_K7TW_NS), 0, (hipStream_t)stream>>>(G, H, W, gx, gx * gy, cams, geom, seg_start,
                                                                         seg_count, seg_stride, keys, spill_keys,
                                                                         final_T, n_contrib, dL_dpix, grad_scale, dgeom);
    return dsplat::check_launch("k_render_bwd_tw");
  }
  auto kern = (int64_t)V * gx * gy >= kWideBwd ? k_render_bwd<5> : k_render_bwd<1>;
  kern<<<grid, NT, 0, (hipStream_t)stream>>>(G, H, W, gx, gx * gy, cams, geom, seg_start, seg_count, seg_stride, keys,
                                             spill_keys, final_T, n_contrib, dL_dpix, grad_scale, dgeom);
  return dsplat::check_launch("k_render_bwd");
}

int dsr_dgeom_to_float(int G, int V, const float* geom, const int64_t* dgeom_fx, const float* grad_scale,
                       const uint8_t* row_live, float* dgeom, void* stream) {
  DSPLAT_REQUIRE(G > 0 && V > 0, "dsr_dgeom_to_float: bad sizes");
  DSPLAT_REQUIRE(geom && dgeom_fx && grad_scale && dgeom, "dsr_dgeom_to_float: null pointer");
  const size_t rows = (size_t)G * V;
  k_dgeom_to_float<<<(unsigned)((rows + NT - 1) / NT), NT, 0, (hipStream_t)stream>>>(
      rows, geom, reinterpret_cast<const long long*>(dgeom_fx), grad_scale, row_live, dgeom);
  return dsplat::check_launch("k_dgeom_to_float");
}

int dsr_preprocess_bwd(int S, int G, int V, int H, int W, int sh_degree, int M, const float* means,
                       const float* shs, const float* cov6, const dsr_camera* cams, const float* geom,
                       const int64_t* dgeom_fx, const float* grad_scale, const int32_t* scene_view_start,
                       const int32_t* scene_views, const uint8_t* row_live,
                       float* dmeans, float* dshs, float* dcolors, float* dopac, float* dcov6, float* dmean2D,
                       int layout, void* stream) {
  DSPLAT_REQUIRE(S > 0 && G > 0 && V > 0 && H > 0 && W > 0, "dsr_preprocess_bwd: bad sizes");
  DSPLAT_REQUIRE((shs != nullptr) == (dshs != nullptr), "dsr_preprocess_bwd: shs and dshs must both be given or both NULL");
  DSPLAT_REQUIRE(shs != nullptr || dcolors != nullptr, "dsr_preprocess_bwd: colors path needs dcolors");
  DSPLAT_REQUIRE(shs == nullptr || (sh_degree >= 0 && sh_degree <= 3 && M >= (sh_degree + 1) * (sh_degree + 1)),
                 "dsr_preprocess_bwd: sh_degree=%d M=%d unsupported", sh_degree, M);
  DSPLAT_REQUIRE(means && cov6 && cams && geom && dgeom_fx && grad_scale && scene_view_start && scene_views && dmeans &&
                     dopac && dcov6,
                 "dsr_preprocess_bwd: null pointer");
  const long long* dgeom = reinterpret_cast<const long long*>(dgeom_fx);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((G + NT - 1) / NT, S);
  const int deg = shs ? sh_degree : -1;
  const size_t lds = (size_t)NT * (size_t)max(shs ? 3 * M : 0, 9) * sizeof(float);
  DSPLAT_REQUIRE(lds <= 64 * 1024, "dsr_preprocess_bwd: M=%d SH coefficients exceed the LDS row staging", M);
#define DSR_PREB(D)                                                                                              \
  k_preprocess_bwd<D><<<grid, NT, lds, st>>>(G, H, W, M, means, shs, cov6, cams, geom, dgeom, grad_scale,          \
                                           scene_view_start,                                                     \
                                           scene_views, row_live, dmeans, dshs, dcolors, dopac, dcov6, dmean2D,  \
                                           layout)
  switch (deg) {
    case -1: DSR_PREB(-1); break;
    case 0: DSR_PREB(0); break;
    case 1: DSR_PREB(1); break;
    case 2: DSR_PREB(2); break;
    default: DSR_PREB(3); break;
  }
#undef DSR_PREB
  return dsplat::check_launch("k_preprocess_bwd");
}

int dsr_head_bwd(int B, int V, int H, int W, int d_sh, int C, const float* head, const float* depths,
                 const float* images, const float* adapter_cams, float scale_min, float scale_max, const float* sh_mask, int Ht, int Wt,
                 const dsr_camera* cams, const float* geom, const int64_t* dgeom_fx, const float* grad_scale,
                 const int32_t* scene_view_start, const int32_t* scene_views, const uint8_t* row_live, float* dhead,
                 float* ddepths, void* stream) {
  DSPLAT_REQUIRE(B > 0 && V > 0 && H > 0 && W > 0 && Ht > 0 && Wt > 0, "dsr_head_bwd: bad sizes");
  DSPLAT_REQUIRE(d_sh == 1 || d_sh == 4 || d_sh == 9 || d_sh == 16, "dsr_head_bwd: d_sh=%d (1, 4, 9, 16)", d_sh);
  DSPLAT_REQUIRE(C >= 10 + 3 * d_sh, "dsr_head_bwd: %d head channels < 10 + 3*d_sh", C);
  DSPLAT_REQUIRE((size_t)H * W % NT == 0, "dsr_head_bwd: H*W=%d must be a multiple of %d (use dsr_preprocess_bwd + "
                 "dga_adapter_bwd)", H * W, NT);
  DSPLAT_REQUIRE(head && depths && images && adapter_cams && sh_mask && cams && geom && dgeom_fx && grad_scale &&
                     scene_view_start && scene_views && dhead,
                 "dsr_head_bwd: null pointer");
  const size_t lds = (size_t)NT * C * sizeof(float);
  DSPLAT_REQUIRE(lds <= 160 * 1024, "dsr_head_bwd: %d head channels exceed the LDS row staging", C);
  const dga::AdIn a{head, nullptr, depths, images, adapter_cams, sh_mask, scale_min, scale_max, 1e-8f, C, B * V, H, W, 1};
  const int G = V * H * W;
  const long long* dgeom = reinterpret_cast<const long long*>(dgeom_fx);
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)(((size_t)B * G + NT - 1) / NT);
#define DSR_HEADB(D, NS)                                                                                          \
  do {                                                                                                            \
    if (int e = dsplat::ensure_dyn_lds((const void*)k_head_bwd<D, NS>, lds, "hipFuncSetAttribute(k_head_bwd)"))  \
      return e;                                                                                                   \
    k_head_bwd<D, NS><<<grid, NT, lds, st>>>(a, G, Ht, Wt, cams, geom, dgeom, grad_scale, scene_view_start,       \
                                             scene_views, row_live, dhead, ddepths);                               \
  } while (0)
  switch (d_sh) {  // the rasterizer's SH degree follows the harmonics: (degree + 1)^2 = d_sh
    case 1: DSR_HEADB(0, 1); break;
    case 4: DSR_HEADB(1, 4); break;
    case 9: DSR_HEADB(2, 9); break;
    default: DSR_HEADB(3, 16); break;
  }
#undef DSR_HEADB
  return dsplat::check_launch("k_head_bwd");
}

}  // extern "C"

// =====================================================================================
// Camera set-up on the device: replaces ~40 small torch ops per render call
// (scale-invariant rescale, get_fov, get_projection_matrix, inverse/transposes;
// cuda_splatting.py:62-86, projection.py:233-247). One thread per view, double internally.
// =====================================================================================
namespace {


__global__ void k_cameras(int V, const float* __restrict__ ext, const float* __restrict__ intr,
                          const float* __restrict__ near, const float* __restrict__ far,
                          const float* __restrict__ bg, const int32_t* __restrict__ view_scene,
                          int scale_invariant, dsr_camera* __restrict__ cams, uint32_t* __restrict__ zero,
                          uint32_t n_zero) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  // the next kernels' per-(view, tile) counters, zeroed here to save them a launch
  for (uint32_t i = (uint32_t)v; i < n_zero; i += gridDim.x * blockDim.x) zero[i] = 0u;
  if (v >= V) return;
  make_camera<double>(v, ext, intr, near, far, bg, view_scene, scale_invariant, cams[v]);
}
}  // namespace

extern "C" int dsr_build_cameras(int V, const float* extrinsics, const float* intrinsics, const float* near,
                                 const float* far, const float* bg, const int32_t* view_scene,
                                 int scale_invariant, dsr_camera* cams, uint32_t* zero_counts,
                                 uint32_t n_zero, void* stream) {
  DSPLAT_REQUIRE(V > 0, "dsr_build_cameras: V=%d", V);
  DSPLAT_REQUIRE(extrinsics && intrinsics && near && far && bg && view_scene && cams, "dsr_build_cameras: null pointer");
  DSPLAT_REQUIRE(n_zero == 0 || zero_counts != nullptr, "dsr_build_cameras: n_zero without zero_counts");
  const unsigned blocks = (unsigned)max((V + 255) / 256, min((int)((n_zero + 255) / 256), 64));
  k_cameras<<<blocks, 256, 0, (hipStream_t)stream>>>(V, extrinsics, intrinsics, near, far, bg, view_scene,
                                                     scale_invariant, cams, zero_counts, n_zero);
  return dsplat::check_launch("k_cameras");
}
