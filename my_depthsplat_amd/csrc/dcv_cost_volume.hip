// dcv_cost_volume.hip — fused plane-sweep warp + correlation for gfx950 (wave64).
//
// Replaces, in one pass and without materialising the [B, C, D, H, W] warped tensor,
//   warp_with_pose_depth_candidates   src/model/encoder/unimatch/matching.py:24-90
//   cost = mean_j(sum_c ref * warped_j) / sqrt(C)   src/model/encoder/unimatch/mv_unimatch.py:494-505
//
// C = 16 / 32 / 64 / 128 run on the matrix cores: reference pixels grouped by epipolar line,
// each group correlated with the band of target pixels its samples tap as one exact-f32 GEMM
// (the k_epi_* grouping passes + k_cost_epi / k_cost_epi_bwd below). Other channel counts: the
// target features are copied channel-last ([B,J,H,W,C]) so every bilinear tap is one
// contiguous C-float row; a wave owns one reference pixel with its 64 lanes over channels
// and finishes 64 depths' partial dot products with a transpose reduction (k_cost_fwd).
// Geometry per (pixel, depth, view) is wave-uniform and follows the reference's
// operation order: p_rot = R K^-1 [x, y, 1]; X = p_rot * depth + t; x = K X;
// uv = x.xy / max(x.z, clamp); grid = 2 uv / (size - 1) - 1; grid_sample unnormalise
// ((g + 1) / 2) * (size - 1), bilinear, zeros padding (align_corners=True).

#include "dsplat_common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace {

constexpr int DG = 16;  // depth hypotheses per register group

struct Cam {
  float Kinv[9], R[9], t[3], K[9];
};

__device__ __forceinline__ void load_cam(const float* intr, const float* pose, Cam& c) {
  // intr: 3x3 row-major K; pose: 4x4 row-major [R | t].
  const float* k = intr;
  for (int i = 0; i < 9; ++i) c.K[i] = k[i];
  // explicit 3x3 inverse (adjugate / det), row-major
  const float a = k[0], b = k[1], cc = k[2], d = k[3], e = k[4], f = k[5], g = k[6], h = k[7], i = k[8];
  const float A = e * i - f * h, Bc = -(d * i - f * g), C = d * h - e * g;
  const float det = a * A + b * Bc + cc * C;
  const float id = 1.0f / det;
  c.Kinv[0] = A * id;
  c.Kinv[1] = -(b * i - cc * h) * id;
  c.Kinv[2] = (b * f - cc * e) * id;
  c.Kinv[3] = Bc * id;
  c.Kinv[4] = (a * i - cc * g) * id;
  c.Kinv[5] = -(a * f - cc * d) * id;
  c.Kinv[6] = C * id;
  c.Kinv[7] = -(a * h - b * g) * id;
  c.Kinv[8] = (a * e - b * d) * id;
  for (int r = 0; r < 3; ++r) {
    for (int q = 0; q < 3; ++q) c.R[r * 3 + q] = pose[r * 4 + q];
    c.t[r] = pose[r * 4 + 3];
  }
}

struct Taps {
  int idx[4];   // flattened y*W + x of nw, ne, sw, se (or -1 when outside)
  float w[4];
};

__device__ __forceinline__ void taps_at(const Cam& c, float prx, float pry, float prz, float depth,
                                        float clampz, int H, int W, Taps& tp) {
  const float X = prx * depth + c.t[0];
  const float Y = pry * depth + c.t[1];
  const float Z = prz * depth + c.t[2];
  const float x = c.K[0] * X + c.K[1] * Y + c.K[2] * Z;
  const float y = c.K[3] * X + c.K[4] * Y + c.K[5] * Z;
  const float z = fmaxf(c.K[6] * X + c.K[7] * Y + c.K[8] * Z, clampz);
  const float u = x / z, v = y / z;
  const float gxn = 2 * u / (W - 1) - 1;
  const float gyn = 2 * v / (H - 1) - 1;
  const float ix = ((gxn + 1) / 2) * (W - 1);
  const float iy = ((gyn + 1) / 2) * (H - 1);
  if (!(ix > -2.f && ix < (float)W + 1.f && iy > -2.f && iy < (float)H + 1.f)) {  // also NaN
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      tp.idx[k] = -1;
      tp.w[k] = 0.f;
    }
    return;
  }
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
  // weights in grid_sample's form: nw = (x1 - ix)(y1 - iy) etc.
  const float wx0 = (float)x1 - ix, wx1 = ix - fx0, wy0 = (float)y1 - iy, wy1 = iy - fy0;
  const bool vx0 = x0 >= 0 && x0 < W, vx1 = x1 >= 0 && x1 < W;
  const bool vy0 = y0 >= 0 && y0 < H, vy1 = y1 >= 0 && y1 < H;
  // out-of-range sample positions (e.g. inf/nan) fall outside every tap
  tp.idx[0] = (vx0 && vy0) ? y0 * W + x0 : -1;
  tp.idx[1] = (vx1 && vy0) ? y0 * W + x1 : -1;
  tp.idx[2] = (vx0 && vy1) ? y1 * W + x0 : -1;
  tp.idx[3] = (vx1 && vy1) ? y1 * W + x1 : -1;
  tp.w[0] = wx0 * wy0;
  tp.w[1] = wx1 * wy0;
  tp.w[2] = wx0 * wy1;
  tp.w[3] = wx1 * wy1;
}

// [B,J,C,H,W] -> [B,J,H,W,C] through a 64x64 LDS tile.
// [n][C][HW] -> [n][rows][C] with rows >= HW; rows past HW (the zero padding row) are zeroed.
__global__ __launch_bounds__(256) void k_to_hwc(int C, int HW, int rows, const float* __restrict__ src,
                                                float* __restrict__ dst) {
  __shared__ float tile[64][65];
  const int bj = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const float* s = src + (size_t)bj * C * HW;
  float* d = dst + (size_t)bj * rows * C;
  if (blockIdx.x == 0 && (int)threadIdx.x < 64 && c0 + (int)threadIdx.x < C)
    for (int p = HW; p < rows; ++p) d[(size_t)p * C + c0 + threadIdx.x] = 0.f;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, p = p0 + tx;
    tile[r][tx] = (c < C && p < HW) ? s[(size_t)c * HW + p] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int p = p0 + r, c = c0 + tx;
    if (p < HW && c < C) d[(size_t)p * C + c] = tile[tx][r];
  }
}

// The same transpose with 16-byte accesses (C % 4 == 0, HW % 4 == 0): each thread reads 4
// consecutive pixels of one channel and writes 4 consecutive channels of one pixel (the
// 4-byte version moved ~4.2 TB/s at config D's 24 x 2 x 128 x 5376 floats).
// Two copies in one launch: planes z < nz1 from (src, dst), the rest from (src2, dst2).
struct HwcJob {
  int C, HW, rows, nz1;
  const float* src;
  float* dst;
  const float* src2;
  float* dst2;
};
// (tid: the thread's index among the tile's 256; every thread of the workgroup reaches the one
// barrier, valid or not)
__device__ __forceinline__ void hwc4_tile(const HwcJob& jb, int bx, int by, int bz, float (*tile)[65], int tid,
                                          bool valid = true) {
  const int C = valid ? jb.C : 0, HW = jb.HW;
  const float* src = jb.src;
  float* dst = jb.dst;
  int bj = bz;
  if (bj >= jb.nz1) {
    bj -= jb.nz1;
    src = jb.src2;
    dst = jb.dst2;
  }
  const int p0 = bx * 64, c0 = by * 64;
  const float* s = src + (size_t)bj * C * HW;
  float* d = dst + (size_t)bj * jb.rows * C;
  if (bx == 0 && tid < 64 && c0 + tid < C)
    for (int p = HW; p < jb.rows; ++p) d[(size_t)p * C + c0 + tid] = 0.f;
  const int q = tid & 15, rr = tid >> 4;  // 16 float4 per 64-float run, 16 runs per pass
  float4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + rr + 16 * k, p = p0 + 4 * q;
    v[k] = (c < C && p < HW) ? *reinterpret_cast<const float4*>(s + (size_t)c * HW + p) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float* t = &tile[rr + 16 * k][4 * q];
    t[0] = v[k].x;
    t[1] = v[k].y;
    t[2] = v[k].z;
    t[3] = v[k].w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = p0 + rr + 16 * k, c = c0 + 4 * q;
    if (p < HW && c < C)
      *reinterpret_cast<float4*>(d + (size_t)p * C + c) =
          make_float4(tile[4 * q][rr + 16 * k], tile[4 * q + 1][rr + 16 * k], tile[4 * q + 2][rr + 16 * k],
                      tile[4 * q + 3][rr + 16 * k]);
  }
}
__global__ __launch_bounds__(256) void k_to_hwc4(HwcJob jb) {
  __shared__ float tile[64][65];
  hwc4_tile(jb, blockIdx.x, blockIdx.y, blockIdx.z, tile, threadIdx.x);
}
__host__ __device__ inline int hwc4_blocks(const HwcJob& jb, int nz) {
  return ((jb.HW + 63) / 64) * ((jb.C + 63) / 64) * nz;
}

// [n][rows][C] (the first HW rows) -> [n][C][HW]
__global__ __launch_bounds__(256) void k_to_chw(int C, int HW, int rows, const float* __restrict__ src,
                                                float* __restrict__ dst) {
  __shared__ float tile[64][65];
  const int bj = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const float* s = src + (size_t)bj * rows * C;
  float* d = dst + (size_t)bj * C * HW;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int p = p0 + r, c = c0 + tx;
    tile[r][tx] = (p < HW && c < C) ? s[(size_t)p * C + c] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, p = p0 + tx;
    if (c < C && p < HW) d[(size_t)c * HW + p] = tile[tx][r];
  }
}

// k_to_chw with 16-byte accesses (C % 4 == 0, HW % 4 == 0).
__global__ __launch_bounds__(256) void k_to_chw4(int C, int HW, int rows, const float* __restrict__ src,
                                                 float* __restrict__ dst) {
  __shared__ float tile[64][65];
  const int bj = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const float* s = src + (size_t)bj * rows * C;
  float* d = dst + (size_t)bj * C * HW;
  const int q = threadIdx.x & 15, rr = threadIdx.x >> 4;
  float4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = p0 + rr + 16 * k, c = c0 + 4 * q;
    v[k] = (p < HW && c < C) ? *reinterpret_cast<const float4*>(s + (size_t)p * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float* t = &tile[rr + 16 * k][4 * q];  // tile[p - p0][c - c0]
    t[0] = v[k].x;
    t[1] = v[k].y;
    t[2] = v[k].z;
    t[3] = v[k].w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + rr + 16 * k, p = p0 + 4 * q;
    if (c < C && p < HW)
      *reinterpret_cast<float4*>(d + (size_t)c * HW + p) =
          make_float4(tile[4 * q][rr + 16 * k], tile[4 * q + 1][rr + 16 * k], tile[4 * q + 2][rr + 16 * k],
                      tile[4 * q + 3][rr + 16 * k]);
  }
}

// Transpose-reduce of DG=16 per-lane partials over the wave: 4 halving exchange stages
// (lane bits 32, 16, 8, 4) then a butterfly over lane bits 2, 1 -> 17 shuffles for 16
// sums; lane l ends with the total of partial index (l >> 2) & 15.
template <int NV, int LB>
__device__ __forceinline__ void treduce_step(float (&part)[DG], int lane) {
  constexpr int HALF = NV / 2;
  const bool upper = (lane & LB) != 0;
#pragma unroll
  for (int i = 0; i < HALF; ++i) {
    const float send = upper ? part[i] : part[i + HALF];
    const float keep = upper ? part[i + HALF] : part[i];
    part[i] = keep + __shfl_xor(send, LB, 64);
  }
}
__device__ __forceinline__ float transpose_reduce16(float (&part)[DG], int lane) {
  treduce_step<16, 32>(part, lane);
  treduce_step<8, 16>(part, lane);
  treduce_step<4, 8>(part, lane);
  treduce_step<2, 4>(part, lane);
  float v = part[0];
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 1, 64);
  return v;
}

// One wave per (b, pixel). grid = (ceil(HW / 4), B), block = 256 (4 pixels).
__global__ __launch_bounds__(256) void k_cost_fwd(int J, int C, int H, int W, int D, int depth_per_pixel,
                                                  const float* __restrict__ ref, const float* __restrict__ tgt_hwc,
                                                  const float* __restrict__ intr, const float* __restrict__ pose,
                                                  const float* __restrict__ depth, float clampz,
                                                  float* __restrict__ cost) {
  const int HW = H * W;
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= HW) return;
  const float px = (float)(p % W), py = (float)(p / W);
  const float scale = 1.0f / (sqrtf((float)C) * (float)J);
  for (int d0 = 0; d0 < D; d0 += DG) {
    float part[DG];
#pragma unroll
    for (int i = 0; i < DG; ++i) part[i] = 0.f;
    for (int j = 0; j < J; ++j) {
      Cam cam;
      load_cam(intr + ((size_t)b * J + j) * 9, pose + ((size_t)b * J + j) * 16, cam);
      const float qx = cam.Kinv[0] * px + cam.Kinv[1] * py + cam.Kinv[2];
      const float qy = cam.Kinv[3] * px + cam.Kinv[4] * py + cam.Kinv[5];
      const float qz = cam.Kinv[6] * px + cam.Kinv[7] * py + cam.Kinv[8];
      const float prx = cam.R[0] * qx + cam.R[1] * qy + cam.R[2] * qz;
      const float pry = cam.R[3] * qx + cam.R[4] * qy + cam.R[5] * qz;
      const float prz = cam.R[6] * qx + cam.R[7] * qy + cam.R[8] * qz;
      const float* tg = tgt_hwc + ((size_t)b * J + j) * (HW + 1) * C;
      for (int c0 = 0; c0 < C; c0 += 64) {
        const int c = c0 + lane;
        const bool cv = c < C;
        const float r = cv ? ref[((size_t)b * C + c) * HW + p] : 0.f;
#pragma unroll
        for (int i = 0; i < DG; ++i) {
          const int d = d0 + i;
          if (d >= D) continue;
          const float dep = depth_per_pixel ? depth[((size_t)b * D + d) * HW + p] : depth[(size_t)b * D + d];
          Taps tp;
          taps_at(cam, prx, pry, prz, dep, clampz, H, W, tp);
          float s = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (tp.idx[k] >= 0 && cv) s += tp.w[k] * tg[(size_t)tp.idx[k] * C + c];
          part[i] += r * s;
        }
      }
    }
    const float tot = transpose_reduce16(part, lane);
    const int d = d0 + (lane >> 2);
    if ((lane & 3) == 0 && d < D) cost[((size_t)b * D + d) * HW + p] = tot * scale;
  }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- epipolar-group formulation on the matrix cores -------------------------------------
// The bilinear warp is linear, so
//   cost(p, d) = sum_j sum_taps w * <ref[:, p], tgt_j[:, q_tap]> / (sqrt(C) J):
// every (pixel, depth) sample needs the correlations of its reference pixel with the <= 4
// target pixels it taps. All depth samples of pixel p lie on p's epipolar line in target
// view j, and reference pixels on ONE epipolar line of the reference image map to ONE
// epipolar line of the target image. So the reference pixels are grouped by the epipolar
// line they lie on (the k_epi_* passes: a counting sort by line, per (batch, view)); 16 pixels of
// a group tap a thin band around a single target line, and their correlations with the
// band's U distinct pixels are one [16 x U x C] GEMM on the matrix cores
// (v_mfma_f32_16x16x4_f32, exact f32), finished by the 4-tap bilinear gather from LDS. With
// row-segment groups (the round-2 band kernel) a diagonal epipolar line made U = the whole
// bounding box of 16 parallel lines (thousands of pixels at the config-D rig); along the line
// it is the line's length x ~3.
constexpr int EG = 16;                       // reference pixels per group (MFMA M)
// samples per thread SPT (kernel template): 8 (128 depth hypotheses per workgroup) or 2 (32,
// for D <= 32: the per-pixel candidate windows of the finer scale); 16 depth lanes x SPT
constexpr int kEUMax = 256;                  // band pixels per GEMM pass (LDS)
constexpr int kECorr = kEUMax + 1;           // odd row stride: the gather's lanes spread over banks
// Line key of reference pixel (px, py) w.r.t. one source view (see the grouping passes below).
struct EpiKey {
  int mode;        // 0: by row (no baseline), 1: angle about a finite epipole, 2: offset across parallel lines
  float ex, ey;    // epipole (mode 1)
  float nx, ny;    // unit normal of the parallel lines (mode 2)
  float o0, inv;   // bucket = floor((value - o0) * inv)
  int nb;
};
static_assert(sizeof(EpiKey) == 32, "EpiKey is 8 words in the workspace");
__device__ __forceinline__ int epi_bucket(const EpiKey& k, float px, float py) {
  float v;
  if (k.mode == 0) return min((int)py, k.nb - 1);
  if (k.mode == 1) {
    v = atan2f(py - k.ey, px - k.ex);  // the line through the epipole, folded to [0, pi)
    if (v < 0.f) v += 3.14159265358979f;
  } else {
    v = k.nx * px + k.ny * py;
  }
  return min(max((int)((v - k.o0) * k.inv), 0), k.nb - 1);
}

// ---- epipolar grouping (round 6: a grid-wide pass pipeline) --------------------------------
// groups[b, j, :] = the reference pixel ids ordered by the epipolar line (w.r.t. view j) they lie
// on. The epipole e = K c, c = -R^T t the source camera centre in reference camera coordinates
// (pose = [R | t] maps reference to source coordinates). Finite epipole: lines are buckets of the
// angle about e, 1 / dmax radians wide (dmax: farthest pixel from e), so neighbouring buckets are
// <= 1 px apart anywhere in the image; epipole far outside the image (sideways baseline): parallel
// lines, 1-px buckets of the offset across them; no baseline: rows. Inside a line the pixels are
// ordered by where their middle depth candidate lands along the target line: each line's key
// range is cut into ceil(n / 16) segments (about one 16-pixel group each), the pixels are
// counting-sorted by (line, segment) and, inside a segment, by pixel id. With per-pixel candidate
// windows (scale > 0) a group's 16 pixels then tap nearby stretches of the line and its band is
// their windows' union, not the whole line. The order is a function of the inputs only (never of
// atomic arrival), so the groups, and with them the backward's MFMA blocking and bits, are the
// same in every run, at every image size. (Results of the forward do not depend on the grouping
// at all: each output is computed from its own correlations.)
// Round 5 did this in ONE workgroup per (scene, view) (48 workgroups at config D: 129 us at
// scale 1, and above 24,544 pixels it fell back to an arrival-ordered line sort). Here every step
// that touches pixels is a grid over the pixels:
//   k_epi_init     per image: line-key parameters + geom; clears the line / bin tables
//   k_epi_count    per pixel: line, sort key; per line: count, key min / max (wave-run atomics)
//   k_epi_segs     per image: first segment bin of each line (scan of ceil(n / 16))
//   k_epi_bin      per pixel: its segment bin; per bin: count
//   k_epi_binscan  per image: bin starts (scan)
//   k_epi_scatter  per pixel: into its bin (arrival order)
//   k_epi_rank     per position: the bin's pixels re-ordered by id (the arrival order is erased)
// geom[b, j] = {M = K R K^-1 (row-major), K t} (double, rounded once): the projection of
// reference pixel p at depth d is M [px, py, 1] d + K t (see epi_ray).
constexpr int kEpiBuckets = 8192;  // epipolar-line buckets per (batch, view)
__host__ __device__ constexpr int epi_bin_stride(int HW) { return (HW + 15) / 16 + kEpiBuckets + 1; }
// grouping scratch inside the forward workspace, after geom
struct EpiScratch {
  EpiKey* keys;                             // [BJ]
  uint32_t *hist, *lmin, *lmax, *bst;       // [BJ][kEpiBuckets]
  uint32_t *bcount, *bstart;                // [BJ][epi_bin_stride]
  uint32_t *pl, *pkv;                       // [BJ][HW]: line (then bin), sort-key bits
  int* stage;                               // [BJ][HW]: pixels by bin, arrival order
};
__host__ __device__ inline size_t epi_scratch_words(int BJ, int HW) {
  return (size_t)BJ * (8 + 4 * (size_t)kEpiBuckets + 2 * (size_t)epi_bin_stride(HW) + 3 * (size_t)HW);
}
__host__ __device__ inline EpiScratch epi_scratch(void* base, int BJ, int HW) {
  uint32_t* p = static_cast<uint32_t*>(base);
  EpiScratch s;
  s.keys = reinterpret_cast<EpiKey*>(p);
  p += (size_t)BJ * 8;
  s.hist = p;
  p += (size_t)BJ * kEpiBuckets;
  s.lmin = p;
  p += (size_t)BJ * kEpiBuckets;
  s.lmax = p;
  p += (size_t)BJ * kEpiBuckets;
  s.bst = p;
  p += (size_t)BJ * kEpiBuckets;
  const size_t bsz = (size_t)BJ * epi_bin_stride(HW);
  s.bcount = p;
  p += bsz;
  s.bstart = p;
  p += bsz;
  s.pl = p;
  p += (size_t)BJ * HW;
  s.pkv = p;
  p += (size_t)BJ * HW;
  s.stage = reinterpret_cast<int*>(p);
  return s;
}
// orderable bits of a float (monotone as unsigned) and back
__device__ __forceinline__ uint32_t epi_obits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float epi_ofloat(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

// The line-key parameters of one (scene, view) from its K and pose (double).
__device__ EpiKey epi_key_of(const float* __restrict__ k, const float* __restrict__ P, int H, int W) {
  EpiKey key;
  const double tx = P[3], ty = P[7], tz = P[11];
  const double cx = -(P[0] * tx + P[4] * ty + P[8] * tz);
  const double cy = -(P[1] * tx + P[5] * ty + P[9] * tz);
  const double cz = -(P[2] * tx + P[6] * ty + P[10] * tz);
  const double exh = k[0] * cx + k[1] * cy + k[2] * cz;
  const double eyh = k[3] * cx + k[4] * cy + k[5] * cz;
  const double ezh = k[6] * cx + k[7] * cy + k[8] * cz;
  const double diag = sqrt((double)W * W + (double)H * H);
  const double mx = 0.5 * (W - 1), my = 0.5 * (H - 1);
  key.ex = key.ey = key.nx = key.ny = key.o0 = 0.f;
  key.inv = 1.f;
  if (fabs(exh) + fabs(eyh) + fabs(ezh) < 1e-12) {
    key.mode = 0;
    key.nb = min(H, kEpiBuckets);
  } else if (fabs(ezh) > 1e-12 && hypot(exh / ezh - mx, eyh / ezh - my) < 64.0 * diag) {
    key.mode = 1;
    key.ex = (float)(exh / ezh);
    key.ey = (float)(eyh / ezh);
    double dmax = 1.0;
    for (int c = 0; c < 4; ++c)
      dmax = fmax(dmax, hypot((c & 1) * (W - 1) - (double)key.ex, (c >> 1) * (H - 1) - (double)key.ey));
    const double nb = ceil(3.14159265358979 * dmax) + 1;
    key.nb = (int)fmin(nb, (double)kEpiBuckets);
    key.inv = (float)(key.nb / 3.14159265358979);
  } else {
    key.mode = 2;
    const double n = hypot(exh, eyh);
    key.nx = (float)(-eyh / n);
    key.ny = (float)(exh / n);
    float lo = 3.4e38f, hi = -3.4e38f;
    for (int c = 0; c < 4; ++c) {
      const float v = key.nx * (float)((c & 1) * (W - 1)) + key.ny * (float)((c >> 1) * (H - 1));
      lo = fminf(lo, v);
      hi = fmaxf(hi, v);
    }
    key.o0 = lo;
    key.nb = min(kEpiBuckets, (int)ceilf(hi - lo) + 1);
    key.inv = (float)key.nb / fmaxf(hi - lo + 1.f, 1.f);
  }
  return key;
}

// grid (ceil(max(kEpiBuckets, bin stride) / 256), B * J), 256 threads. Block 0 of each image
// writes its key and geom; every block clears its share of the tables.
__global__ __launch_bounds__(256) void k_epi_init(int J, int H, int W, const float* __restrict__ intr,
                                                  const float* __restrict__ pose, float* __restrict__ geom,
                                                  EpiScratch s) {
  const int bj = blockIdx.y, tid = threadIdx.x, HW = H * W, nbs = epi_bin_stride(HW);
  const float* k = intr + (size_t)bj * 9;
  const float* P = pose + (size_t)bj * 16;
  if (blockIdx.x == 0 && tid < 12) {
    // Kinv by the adjugate, M = K R Kinv, bt = K t
    const double a = k[0], bb = k[1], c = k[2], d = k[3], e = k[4], f = k[5], g = k[6], h = k[7], i = k[8];
    const double A = e * i - f * h, Bc = -(d * i - f * g), Cc = d * h - e * g;
    const double id = 1.0 / (a * A + bb * Bc + c * Cc);
    const double Ki[9] = {A * id, -(bb * i - c * h) * id, (bb * f - c * e) * id,
                          Bc * id, (a * i - c * g) * id, -(a * f - c * d) * id,
                          Cc * id, -(a * h - bb * g) * id, (a * e - bb * d) * id};
    const int r = tid / 3, q = tid % 3;
    double v = 0.0;
    if (tid < 9) {
      for (int m = 0; m < 3; ++m) {
        double rk = 0.0;  // (R Kinv)[m][q]
        for (int n = 0; n < 3; ++n) rk += (double)P[m * 4 + n] * Ki[n * 3 + q];
        v += (double)k[r * 3 + m] * rk;
      }
    } else {
      const int rr = tid - 9;
      v = k[rr * 3 + 0] * (double)P[3] + k[rr * 3 + 1] * (double)P[7] + k[rr * 3 + 2] * (double)P[11];
    }
    geom[(size_t)bj * 12 + tid] = (float)v;
  }
  if (blockIdx.x == 0 && tid == 32) s.keys[bj] = epi_key_of(k, P, H, W);
  const int i = blockIdx.x * 256 + tid;
  if (i < kEpiBuckets) {
    s.hist[(size_t)bj * kEpiBuckets + i] = 0u;
    s.lmin[(size_t)bj * kEpiBuckets + i] = 0xFFFFFFFFu;
    s.lmax[(size_t)bj * kEpiBuckets + i] = 0u;
  }
  if (i < nbs) s.bcount[(size_t)bj * nbs + i] = 0u;
}

// The pixel passes run 1024-thread workgroups over kEpiPix = 4096 pixels (4 per thread, each
// step coalesced) and combine their per-line / per-bin updates in LDS first: on the diagonal
// epipolar lines of the config-D rig neighbouring pixels of a row lie on different lines, so
// per-pixel (or per-wave-run) global atomics were the passes' cost (round-6 first version,
// 256-pixel workgroups: 21 / 24 / 34 us for count / bin / scatter at 24 x 2 x 112 x 192).
constexpr int kEpiPix = 4096;

// grid (ceil(HW / kEpiPix), B * J), 1024 threads, dynamic LDS 3 kEpiBuckets words: each pixel's
// line and sort key (where its middle candidate lands, projected on the direction of its own
// near-to-far step, canonically oriented: x > 0, or y > 0 on vertical lines, so the pixels of one
// target line, whose directions agree to a fraction of a degree, order along it); per line the
// count and the key range.
// HWC: the first half of the forward's channel-last copies ride along as extra workgroups (a
// 1-D grid: pb B J counting workgroups, then 4 copy tiles of 256 threads per workgroup, tiles
// [0, t1); the rest go with the rank pass): the copy is HBM-bound, this pass latency-bound.
template <bool HWC>
__global__ __launch_bounds__(1024) void k_epi_count(int H, int W, int D, int depth_per_pixel,
                                                    const float* __restrict__ depth, const float* __restrict__ geom,
                                                    int J, EpiScratch s, int pb, int BJ, HwcJob jb, int t1) {
  extern __shared__ uint32_t epi_lds[];
  uint32_t* l_cnt = epi_lds;
  uint32_t* l_min = epi_lds + kEpiBuckets;
  uint32_t* l_max = epi_lds + 2 * kEpiBuckets;
  int bx_ = blockIdx.x, bj_ = blockIdx.y;
  if (HWC) {
    const int ncount = pb * BJ;
    if ((int)blockIdx.x >= ncount) {
      const int t = ((int)blockIdx.x - ncount) * 4 + (int)(threadIdx.x >> 8);
      const int nx = (jb.HW + 63) / 64, ny = (jb.C + 63) / 64;
      const int bz = t / (nx * ny), r = t - bz * nx * ny, by = r / nx, bx = r - by * nx;
      hwc4_tile(jb, bx, by, bz, reinterpret_cast<float(*)[65]>(epi_lds) + (threadIdx.x >> 8) * 64, threadIdx.x & 255,
                t < t1);
      return;
    }
    bj_ = (int)blockIdx.x / pb;
    bx_ = (int)blockIdx.x - bj_ * pb;
  }
  const int bj = bj_, HW = H * W, b = bj / J, tid = threadIdx.x;
  const EpiKey key = s.keys[bj];
  const int nb = key.nb;
  for (int l = tid; l < nb; l += 1024) {
    l_cnt[l] = 0u;
    l_min[l] = 0xFFFFFFFFu;
    l_max[l] = 0u;
  }
  __syncthreads();
  const float* gm = geom + (size_t)bj * 12;
  const float* dp = depth + (size_t)b * D * (depth_per_pixel ? HW : 1);
  const int dm = D / 2, d1 = D > 1 ? D - 1 : 0;
  constexpr int PPT = kEpiPix / 1024;
  float dmids[PPT], dfars[PPT];  // every pixel's two depth loads in flight together
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int p = min(bx_ * kEpiPix + k * 1024 + tid, HW - 1);
    dmids[k] = depth_per_pixel ? dp[(size_t)dm * HW + p] : dp[dm];
    dfars[k] = depth_per_pixel ? dp[(size_t)d1 * HW + p] : dp[d1];
  }
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int p = bx_ * kEpiPix + k * 1024 + tid;
    if (p >= HW) break;
    const float dmid = dmids[k], dfar = dfars[k];
    const float px = (float)(p % W), py = (float)(p / W);
    auto target = [&](float d, float& u, float& v) {
      const float x = fmaf(fmaf(gm[0], px, fmaf(gm[1], py, gm[2])), d, gm[9]);
      const float y = fmaf(fmaf(gm[3], px, fmaf(gm[4], py, gm[5])), d, gm[10]);
      const float z = fmaxf(fmaf(fmaf(gm[6], px, fmaf(gm[7], py, gm[8])), d, gm[11]), 1e-3f);
      u = x / z;
      v = y / z;
    };
    float u0, v0, u1, v1;
    target(dmid, u0, v0);
    target(dfar, u1, v1);
    float dx = u1 - u0, dy = v1 - v0;
    const float l = sqrtf(dx * dx + dy * dy);
    if (l > 1e-6f && l < 3.0e38f) {
      dx /= l;
      dy /= l;
    } else {
      dx = 1.f;
      dy = 0.f;
    }
    if (dx < -1e-3f || (!(dx > 1e-3f) && dy < 0.f)) {
      dx = -dx;
      dy = -dy;
    }
    float kv = fmaf(u0, dx, v0 * dy);
    kv = (kv == kv && fabsf(kv) < 1e30f) ? kv : 1e30f;  // NaN / inf: last
    const uint32_t line = (uint32_t)epi_bucket(key, px, py);
    const uint32_t ob = epi_obits(kv);
    s.pl[(size_t)bj * HW + p] = line;
    s.pkv[(size_t)bj * HW + p] = ob;
    atomicAdd(&l_cnt[line], 1u);
    atomicMin(&l_min[line], ob);
    atomicMax(&l_max[line], ob);
  }
  __syncthreads();
  for (int l = tid; l < nb; l += 1024) {
    const uint32_t c = l_cnt[l];
    if (c) {
      const size_t o = (size_t)bj * kEpiBuckets + l;
      atomicAdd(&s.hist[o], c);
      atomicMin(&s.lmin[o], l_min[l]);
      atomicMax(&s.lmax[o], l_max[l]);
    }
  }
}

// Exclusive scan of n words by one 1024-thread workgroup (chunks of 8192, carried): out[i] =
// sum of load(k) for k < i; out2 (optional) gets a copy. Returns the total.
template <typename Load>
__device__ uint32_t epi_block_scan(int n, Load load, uint32_t* __restrict__ out, uint32_t* __restrict__ out2,
                                   uint32_t* wsum) {
  constexpr int PT = 8;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint32_t carry = 0;
  for (int base = 0; base < n; base += 1024 * PT) {
    uint32_t v[PT], tot = 0;
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int k = base + tid * PT + i;
      v[i] = k < n ? load(k) : 0u;
      tot += v[i];
    }
    const uint32_t incl = dsplat::wave_incl_scan(tot, lane);
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t off = carry + incl - tot, total = 0;
    for (int k = 0; k < 16; ++k) {
      if (k < wv) off += wsum[k];
      total += wsum[k];
    }
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int k = base + tid * PT + i;
      if (k < n) {
        out[k] = off;
        if (out2) out2[k] = off;
      }
      off += v[i];
    }
    carry += total;
    __syncthreads();  // wsum reused by the next chunk
  }
  return carry;
}

// grid B * J, 1024 threads: bst[line] = the line's first segment bin.
__global__ __launch_bounds__(1024) void k_epi_segs(EpiScratch s) {
  __shared__ uint32_t wsum[16];
  const size_t o = (size_t)blockIdx.x * kEpiBuckets;
  const uint32_t* hist = s.hist + o;
  epi_block_scan(kEpiBuckets, [&](int k) { return (hist[k] + 15u) / 16u; }, s.bst + o, nullptr, wsum);
}

// grid (ceil(HW / kEpiPix), B * J), 1024 threads, dynamic LDS epi_bin_stride(HW) words: each
// pixel's segment bin (its line's key range cut into ceil(n / 16) equal parts); per bin the count.
__global__ __launch_bounds__(1024) void k_epi_bin(int HW, EpiScratch s) {
  extern __shared__ uint32_t epi_lds[];
  const int bj = blockIdx.y, tid = threadIdx.x, nbs = epi_bin_stride(HW);
  for (int i = tid; i < nbs; i += 1024) epi_lds[i] = 0u;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kEpiPix / 1024; ++k) {
    const int p = blockIdx.x * kEpiPix + k * 1024 + tid;
    if (p >= HW) break;
    const int l = (int)s.pl[(size_t)bj * HW + p];
    const size_t o = (size_t)bj * kEpiBuckets + l;
    const uint32_t nseg = (s.hist[o] + 15u) / 16u;
    const float lo = epi_ofloat(s.lmin[o]), hi = epi_ofloat(s.lmax[o]);
    const float kv = epi_ofloat(s.pkv[(size_t)bj * HW + p]);
    const float f = hi > lo ? (kv - lo) / (hi - lo) : 0.f;
    const uint32_t bin = s.bst[o] + (uint32_t)min((int)nseg - 1, max(0, (int)(f * (float)nseg)));
    s.pl[(size_t)bj * HW + p] = bin;
    atomicAdd(&epi_lds[bin], 1u);
  }
  __syncthreads();
  for (int i = tid; i < nbs; i += 1024) {
    const uint32_t c = epi_lds[i];
    if (c) atomicAdd(&s.bcount[(size_t)bj * nbs + i], c);
  }
}

// grid B * J, 1024 threads: bin starts (bstart; bcount becomes the scatter's cursor).
__global__ __launch_bounds__(1024) void k_epi_binscan(int HW, EpiScratch s) {
  __shared__ uint32_t wsum[16];
  const int nbs = epi_bin_stride(HW);
  const size_t o = (size_t)blockIdx.x * nbs;
  uint32_t* bc = s.bcount + o;
  // the image's bins end where its last line's segments end; bstart of that end is read too
  const int nb = s.keys[blockIdx.x].nb;
  const size_t ol = (size_t)blockIdx.x * kEpiBuckets + (nb - 1);
  const int nbins = nb > 0 ? (int)(s.bst[ol] + (s.hist[ol] + 15u) / 16u) : 0;
  epi_block_scan(min(nbins + 1, nbs), [&](int k) { return bc[k]; }, s.bstart + o, bc, wsum);
}

// grid (ceil(HW / kEpiPix), B * J), 1024 threads, dynamic LDS epi_bin_stride(HW) words: every
// pixel into its bin, in arrival order: local ranks from LDS counters, then one global
// reservation per (workgroup, bin).
__global__ __launch_bounds__(1024) void k_epi_scatter(int HW, EpiScratch s) {
  extern __shared__ uint32_t epi_lds[];
  const int bj = blockIdx.y, tid = threadIdx.x, nbs = epi_bin_stride(HW);
  for (int i = tid; i < nbs; i += 1024) epi_lds[i] = 0u;
  __syncthreads();
  uint32_t bin[kEpiPix / 1024], rank[kEpiPix / 1024];
#pragma unroll
  for (int k = 0; k < kEpiPix / 1024; ++k) {
    const int p = blockIdx.x * kEpiPix + k * 1024 + tid;
    bin[k] = p < HW ? s.pl[(size_t)bj * HW + p] : 0xFFFFFFFFu;
  }
#pragma unroll
  for (int k = 0; k < kEpiPix / 1024; ++k)
    if (bin[k] != 0xFFFFFFFFu) rank[k] = atomicAdd(&epi_lds[bin[k]], 1u);
  __syncthreads();
  for (int i = tid; i < nbs; i += 1024) {  // count -> this workgroup's base in the bin
    const uint32_t c = epi_lds[i];
    if (c) epi_lds[i] = atomicAdd(&s.bcount[(size_t)bj * nbs + i], c);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kEpiPix / 1024; ++k)
    if (bin[k] != 0xFFFFFFFFu)
      s.stage[(size_t)bj * HW + epi_lds[bin[k]] + rank[k]] = blockIdx.x * kEpiPix + k * 1024 + tid;
}

// grid (ceil(HW / 256), B * J): output position -> the pixel of that rank (by id) in its bin.
__device__ __forceinline__ void epi_rank_one(int HW, const EpiScratch& s, int* __restrict__ groups, int bj, int pos) {
  if (pos >= HW) return;
  const int* st = s.stage + (size_t)bj * HW;
  const int p = st[pos];
  const uint32_t bin = s.pl[(size_t)bj * HW + p];
  const uint32_t* bs = s.bstart + (size_t)bj * epi_bin_stride(HW);
  const int b0 = (int)bs[bin], b1 = (int)bs[bin + 1];
  int r = 0;
  for (int q = b0; q < b1; ++q) r += st[q] < p ? 1 : 0;
  groups[(size_t)bj * HW + b0 + r] = p;
}
__global__ __launch_bounds__(256) void k_epi_rank(int HW, EpiScratch s, int* __restrict__ groups) {
  epi_rank_one(HW, s, groups, blockIdx.y, blockIdx.x * 256 + threadIdx.x);
}

// k_epi_rank with the forward's channel-last copies (hwc4_tile) as extra workgroups after its
// own (round 6): the copy is HBM-bound and the rank pass latency-bound, so the two overlap
// instead of running back to back. Workgroups [0, pg BJ) rank, the rest copy tiles [t0, ...)
// (k_epi_count<true> took the tiles before t0).
__global__ __launch_bounds__(256) void k_epi_rank_hwc(int HW, EpiScratch s, int* __restrict__ groups, int pg, int BJ,
                                                      HwcJob jb, int t0) {
  __shared__ float tile[64][65];
  const int nrank = pg * BJ;
  if ((int)blockIdx.x < nrank) {
    const int bj = blockIdx.x / pg, pos = (blockIdx.x - bj * pg) * 256 + threadIdx.x;
    epi_rank_one(HW, s, groups, bj, pos);
    return;
  }
  const int t = blockIdx.x - nrank, nx = (jb.HW + 63) / 64, ny = (jb.C + 63) / 64;
  const int tt = t + t0;
  const int bz = tt / (nx * ny), r = tt - bz * nx * ny, by = r / nx, bx = r - by * nx;
  hwc4_tile(jb, bx, by, bz, tile, threadIdx.x);
}

// The target image of (b, j): its own copy, or view tmap[bj] of the per-view copy (views mode;
// the index is clamped to the B views: a bad caller index must not reach past the buffer).
__device__ __forceinline__ size_t cv_target(const int* __restrict__ tmap, size_t bj, int B) {
  return tmap ? (size_t)min(max(tmap[bj], 0), B - 1) : bj;
}

// Shared set-up of the forward and backward group kernels: the workgroup's (b, group) with
// a given view's groups on a contiguous range of one XCD (their target bands overlap: L2).
__device__ __forceinline__ bool epi_item(int B, int ngroups, int& b, int& g) {
  const int items = B * ngroups, per = (items + 7) >> 3;
  const int item = (int)(blockIdx.x & 7u) * per + (int)(blockIdx.x >> 3);
  if ((int)(blockIdx.x >> 3) >= per || item >= items) return false;
  b = item / ngroups;
  g = item - b * ngroups;
  return true;
}

// The band lives on an extended grid of (W + 2) x (H + 2) positions (image x, y in [-1, W]
// x [-1, H]: every tap of a sample whose top-left tap is in [-1, W - 1] x [-1, H - 1]; other
// samples tap nothing inside the image). A sample marks only its top-left tap (one LDS atomic
// instead of four); the tapped set is that base bitmap OR-ed with itself shifted by one
// column, one row and both (a word-parallel pass), so the sample's four taps have ranks
// r(e), r(e) + 1, r(e + Wx), r(e + Wx) + 1. Band positions outside the image correlate to 0
// (zero B operand) = grid_sample's zeros padding.
struct EpiLds {
  float* aref;      // [EG][C + 4]
  uint32_t* base;   // [NWx] top-left taps
  uint2* wb;        // [NWx] {tapped positions, exclusive popcount prefix} per word
  int* nzw;         // [NWx] the non-zero words of bm, ascending
  int* list;        // [kEUMax] image pixel of each band position of the current pass (-1: outside)
  float* corr;      // [2^PXB][band + 1] correlations (forward) / gradient weights (backward)
  uint32_t* misc;   // [32]: scan partials, totals, the band box
};
__host__ __device__ constexpr int epi_words(int H, int W) { return ((W + 2) * (H + 2) + 31) / 32 + 1; }
// The group's reference tile [EG][C] into LDS from the channel-last copy (rows of 16-byte
// vectors; a past-the-end pixel reads the zero row HW), loads issued together.
template <int NK, int ROWS = EG>
__device__ __forceinline__ void epi_aref(const EpiLds& L, int HW, int b, const int* gids,
                                         const float* __restrict__ ref_hwc) {
  constexpr int C = 4 * NK, N4 = ROWS * C / 4, IT = (N4 + 255) / 256;
  float4 v[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int k = min((int)threadIdx.x + 256 * it, N4 - 1), r = k / (C / 4), c4 = k - r * (C / 4);
    const int pr = gids[r] >= 0 ? gids[r] : HW;
    v[it] = *reinterpret_cast<const float4*>(ref_hwc + ((size_t)b * (HW + 1) + pr) * C + 4 * c4);
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int k = (int)threadIdx.x + 256 * it, r = k / (C / 4), c4 = k - r * (C / 4);
    if (k < N4) *reinterpret_cast<float4*>(L.aref + r * (C + 4) + 4 * c4) = v[it];
  }
}

// Per-pixel ray terms: the projection of depth d is (ax d + bx, ay d + by, az d + bz) with
// a = M [px, py, 1], M = K R K^-1 and b = K t (from k_epi_init's geom; matching.py:47-65
// regrouped, each coefficient rounded once from double: within a few ulp of the reference's
// K (R K^-1 p d + t); the parity bar is 1e-4).
struct EpiRay {
  float ax, ay, az, bx, by, bz;
};
__device__ __forceinline__ EpiRay epi_ray(const float* __restrict__ gm, float px, float py) {
  EpiRay r;
  r.ax = fmaf(gm[0], px, fmaf(gm[1], py, gm[2]));
  r.ay = fmaf(gm[3], px, fmaf(gm[4], py, gm[5]));
  r.az = fmaf(gm[6], px, fmaf(gm[7], py, gm[8]));
  r.bx = gm[9];
  r.by = gm[10];
  r.bz = gm[11];
  return r;
}
// Sample position (grid_sample's unnormalised coordinates = the projected pixel, align_corners
// = True) and its top-left tap (tx0, ty0) in [-1, W - 1] x [-1, H - 1] packed as
// (ty0 + 1) << 16 | (tx0 + 1), or -1 when no tap is inside the image. 1 / z is the hardware
// reciprocal (1 ulp; the parity bar is 1e-4).
__device__ __forceinline__ int epi_sample(const EpiRay& ry, float dep, float clampz, int H, int W, float& ix,
                                          float& iy) {
  const float xx = fmaf(ry.ax, dep, ry.bx), yy = fmaf(ry.ay, dep, ry.by);
  const float zz = fmaxf(fmaf(ry.az, dep, ry.bz), clampz);
  const float rz = __builtin_amdgcn_rcpf(zz);
  ix = xx * rz;
  iy = yy * rz;
  if (!(ix > -1.f && ix < (float)W && iy > -1.f && iy < (float)H)) return -1;  // also NaN
  const int tx0 = (int)floorf(ix), ty0 = (int)floorf(iy);
  return ((ty0 + 1) << 16) | (tx0 + 1);
}

// The band box (round 5): the bitmap, its word pass and the band list cover only the bounding
// box of the group's top-left taps (+1 column and row for the other three taps), not the whole
// (W + 2) x (H + 2) extended image: at config-D scale 1 a group's 16 x 32 per-pixel samples tap a
// few short segments (tens to a few hundred positions) while the image has 22 K, and the
// per-word band set-up was the workgroup's largest fixed cost. Local index of top-left tap
// (tx0, ty0): (ty0 - y0) wb + (tx0 - x0); taps e, e + 1, e + wb, e + wb + 1.
struct EpiBox {
  int x0, y0, wb, nw;  // box origin (extended-grid coordinates, i.e. + 1), row width, bitmap words
};
// Block-wide box of the packed taps es[] (all threads; one barrier). Empty box: nw = 0.
template <int SPT>
__device__ __forceinline__ EpiBox epi_box(const EpiLds& L, const int (&es)[SPT]) {
  int mnx = 1 << 30, mny = 1 << 30, mxx = -1, mxy = -1;
#pragma unroll
  for (int s = 0; s < SPT; ++s)
    if (es[s] >= 0) {
      const int x = es[s] & 0xFFFF, y = es[s] >> 16;
      mnx = min(mnx, x);
      mny = min(mny, y);
      mxx = max(mxx, x);
      mxy = max(mxy, y);
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mnx = min(mnx, __shfl_xor(mnx, off, 64));
    mny = min(mny, __shfl_xor(mny, off, 64));
    mxx = max(mxx, __shfl_xor(mxx, off, 64));
    mxy = max(mxy, __shfl_xor(mxy, off, 64));
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    L.misc[16 + 4 * wv] = (uint32_t)mnx;
    L.misc[17 + 4 * wv] = (uint32_t)mny;
    L.misc[18 + 4 * wv] = (uint32_t)mxx;
    L.misc[19 + 4 * wv] = (uint32_t)mxy;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    mnx = min(mnx, (int)L.misc[16 + 4 * k]);
    mny = min(mny, (int)L.misc[17 + 4 * k]);
    mxx = max(mxx, (int)L.misc[18 + 4 * k]);
    mxy = max(mxy, (int)L.misc[19 + 4 * k]);
  }
  EpiBox bx;
  bx.x0 = mnx;
  bx.y0 = mny;
  bx.wb = mxx - mnx + 2;
  bx.nw = mxx < 0 ? 0 : ((mxx - mnx + 2) * (mxy - mny + 2) + 31) / 32 + 1;
  return bx;
}
__device__ __forceinline__ int epi_local(const EpiBox& bx, int es) {
  return es < 0 ? -1 : ((es >> 16) - bx.y0) * bx.wb + ((es & 0xFFFF) - bx.x0);
}

// Front half shared by the forward and the backward:
//   epi_depths   the samples' depth candidates (global loads, issued early: their latency runs
//                under the reference tile load in the forward);
//   epi_taps     the samples' packed top-left taps (registers);
//   epi_box      (one barrier) their bounding box;
//   epi_mark     the taps into the box's base bitmap (LDS atomics; the bitmap's words must be
//                zero: cleared before the box's barrier);
//   epi_band     after a barrier: the tapped set (base | shifted copies) of each thread's own
//                contiguous run of words, its popcount prefix (wave scans) and the non-zero
//                words; returns U (band positions). Two barriers.
// es[s]: local index of sample s's top-left tap (-1: zero sample).
// PXB: log2 of the pixels per depth slot (4: 16-pixel groups, thread t has pixel t & 15 and
// depths d0 + (t >> 4) + 16 s; 6: the backward's 64-pixel groups, depths d0 + (t >> 6) + 4 s)
template <int SPT, int PXB = 4>
__device__ __forceinline__ void epi_depths(int HW, int D, int depth_per_pixel, int b, int d0, int pix,
                                           const float* __restrict__ depth, float (&dep)[SPT]) {
  constexpr int DST = 256 >> PXB;
  const int dl = threadIdx.x >> PXB;
  const float* dp = depth + (size_t)b * D * (depth_per_pixel ? HW : 1);
  const int dstride = depth_per_pixel ? HW : 1, pc = depth_per_pixel ? max(pix, 0) : 0;
#pragma unroll
  for (int s = 0; s < SPT; ++s) dep[s] = dp[(uint32_t)(min(d0 + dl + DST * s, D - 1) * dstride + pc)];
}
template <int SPT, int PXB = 4>
__device__ __forceinline__ void epi_taps(int H, int W, int D, int d0, int pix, const EpiRay& ry,
                                         const float (&dep)[SPT], float clampz, float (&sx)[SPT], float (&sy)[SPT],
                                         int (&es)[SPT]) {
  constexpr int DST = 256 >> PXB;
  const int dl = threadIdx.x >> PXB;
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const int d = d0 + dl + DST * s;
    es[s] = epi_sample(ry, dep[s], clampz, H, W, sx[s], sy[s]);
    if (pix < 0 || d >= D) es[s] = -1;
  }
}
template <int SPT>
__device__ __forceinline__ void epi_mark(const EpiLds& L, const EpiBox& bx, int (&es)[SPT]) {
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    es[s] = epi_local(bx, es[s]);
    if (es[s] >= 0) atomicOr(&L.base[es[s] >> 5], 1u << (es[s] & 31));
  }
}
__device__ __forceinline__ int epi_band(const EpiLds& L, const EpiBox& bx) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wb = bx.wb, NWx = bx.nw;
  // tapped = base | base << 1 | base << wb | base << (wb + 1) (bit shifts across the words)
  auto shl = [&](int w, int sft) -> uint32_t {
    const int wo = sft >> 5, bo = sft & 31;
    const uint32_t lo = w - wo >= 0 ? L.base[w - wo] : 0u;
    if (bo == 0) return lo;
    const uint32_t hi = w - wo - 1 >= 0 ? L.base[w - wo - 1] : 0u;
    return (lo << bo) | (hi >> (32 - bo));
  };
  // thread t owns the contiguous words [t per, (t + 1) per): it forms them and counts them, so
  // no barrier separates the two
  const int per = (NWx + 255) / 256;
  const int w0 = tid * per, w1 = min(NWx, w0 + per);
  uint32_t tot = 0, nz = 0;
  for (int w = w0; w < w1; ++w) {
    const uint32_t bits = shl(w, 0) | shl(w, 1) | shl(w, wb) | shl(w, wb + 1);
    L.wb[w].x = bits;
    const uint32_t c = __popc(bits);
    tot += c;
    nz += c != 0u;
  }
  const uint32_t incl = dsplat::wave_incl_add_dpp(tot), inz = dsplat::wave_incl_add_dpp(nz);
  if (lane == 63) {
    L.misc[wv] = incl;
    L.misc[8 + wv] = inz;
  }
  __syncthreads();
  uint32_t off = incl - tot, offz = inz - nz;
  for (int k = 0; k < wv; ++k) {
    off += L.misc[k];
    offz += L.misc[8 + k];
  }
  for (int w = w0; w < w1; ++w) {
    const uint32_t bits = L.wb[w].x;
    L.wb[w].y = off;
    off += __popc(bits);
    if (bits) L.nzw[offz++] = w;
  }
  if (tid == 255) {
    L.misc[4] = off;
    L.misc[5] = offz;
  }
  __syncthreads();
  return (int)L.misc[4];
}
// clear the words of a box (or, before the first one, of the whole extended image)
__device__ __forceinline__ void epi_clear_words(const EpiLds& L, int nw) {
  for (int w = threadIdx.x; w < nw; w += 256) L.base[w] = 0u;
}
// the steps for one depth chunk with their own barriers (the backward's per-chunk loop); the
// base words of the previous chunk's box (nw_prev, the whole image before the first) are
// cleared before the box barrier
template <int SPT, int PXB>
__device__ __forceinline__ int epi_front(const EpiLds& L, int H, int W, int HW, int D, int depth_per_pixel, int b,
                                         int d0, int pix, const EpiRay& ry, const float* __restrict__ depth,
                                         float clampz, float (&sx)[SPT], float (&sy)[SPT], int (&es)[SPT],
                                         EpiBox& bx, int nw_prev) {
  float dep[SPT];
  epi_depths<SPT, PXB>(HW, D, depth_per_pixel, b, d0, pix, depth, dep);
  epi_taps<SPT, PXB>(H, W, D, d0, pix, ry, dep, clampz, sx, sy, es);
  epi_clear_words(L, nw_prev);
  bx = epi_box<SPT>(L, es);
  epi_mark<SPT>(L, bx, es);
  __syncthreads();
  return bx.nw ? epi_band(L, bx) : 0;
}

// list[] = the target row of band ranks [r0, r0 + n): the image pixel, or HW (the all-zero
// padding row of the channel-last copy) for positions outside the image and for the slots
// [n, round_up(n, kEPad)) past the band. 32 lanes per non-zero word, one bit each.
constexpr int kEPad = 32;
__device__ __forceinline__ int epi_padded(int n) { return (n + kEPad - 1) / kEPad * kEPad; }
__device__ __forceinline__ void epi_list(const EpiLds& L, int H, int W, const EpiBox& bx, int r0, int n) {
  const int wb = bx.wb, nnz = (int)L.misc[5], bit = threadIdx.x & 31, HW = H * W;
  if ((int)threadIdx.x < epi_padded(n) - n) L.list[n + threadIdx.x] = HW;
  const float rwb = 1.0f / (float)wb;
  for (int k = threadIdx.x >> 5; k < nnz; k += 8) {
    const int w = L.nzw[k];
    const uint2 wv2 = L.wb[w];
    const uint32_t bits = wv2.x;
    if (!((bits >> bit) & 1u)) continue;
    const int r = (int)(wv2.y + __popc(bits & ((1u << bit) - 1u)));
    if (r < r0 || r >= r0 + n) continue;
    const int e = w * 32 + bit;
    int ye = (int)((float)e * rwb), xe = e - ye * wb;  // the float quotient is within 1 of e / wb
    if (xe < 0) {
      --ye;
      xe += wb;
    } else if (xe >= wb) {
      ++ye;
      xe -= wb;
    }
    const int x = bx.x0 + xe - 1, y = bx.y0 + ye - 1;  // box origin is in extended (+1) coordinates
    L.list[r - r0] = (x >= 0 && x < W && y >= 0 && y < H) ? y * W + x : HW;
  }
}
__device__ __forceinline__ int epi_rank(const EpiLds& L, int e) {
  const uint2 w = L.wb[e >> 5];
  return (int)(w.y + __popc(w.x & ((1u << (e & 31)) - 1u)));
}

// Workgroups of 2^PXB reference pixels (round 5): 16 (one group of the grouping's order) or
// 32 / 64 (2 / 4 consecutive groups: neighbours along one epipolar line, whose target bands
// overlap), their samples' bands merged into one. The band set-up (bitmap, box, word pass,
// list), the target rows' loads and the barriers are then paid once per 2^PXB pixels; the
// GEMM covers the union band.
constexpr int kEGWMax = 64;             // widest group
// Band positions per GEMM pass (the [2^PXB][band + 1] LDS tile). Forward (16-pixel groups):
// 128 for the per-pixel-candidate shapes (SPT = 2: short bands; the smaller tile lets 6
// instead of 4 workgroups share a CU: config D scale 1 forward 0.852 -> 0.761 ms, same box,
// profiles/r05t_ab_cv_pass128.log), 256 otherwise (per-image candidates: long bands, a second
// pass cost more there: scale 0 0.436 -> 0.474 ms at 128). Backward (round 6): the backward is
// latency-bound (MFMA busy 0.22, more wait than issue cycles), so the tile is sized for
// occupancy: 64 positions at 64-pixel groups (3 workgroups per CU instead of 2), 128 at 32 (4
// instead of 2): config D fwd + bwd scale 1 2.50 -> 2.27 ms, scale 0 2.01 -> 1.97 ms (same box,
// profiles/r06s_ab_cv_bwd_occupancy.log); 32 / 64 (4 / 5 per CU) lost (r06t: 2.37 / 2.14).
__host__ __device__ constexpr int epi_pass(int pxb, int spt) {
  return pxb == 6 ? 64 : pxb == 5 ? 128 : spt == 2 ? 128 : 256;
}
// workgroups per CU the backward's LDS allows (launch bounds: the VGPR budget to match)
// (late round 6: the C = 128 32-pixel instance at 3, where it needs no scratch spills and both
// GEMMs reuse their A fragments: scale 0 fwd + bwd -2.4 %, profiles/r06av_ab_cvbwd_scale0.txt)
__host__ __device__ constexpr int bwd_occ(int pxb, int c) { return pxb == 4 ? 3 : pxb == 6 ? 3 : c == 128 ? 3 : 4; }
template <int PXB, int SPT>
constexpr int bwd_band() { return epi_pass(PXB, SPT); }
static_assert(epi_pass(4, 8) <= kEUMax && epi_pass(6, 8) <= kEUMax, "the band list holds a pass");
template <int PXB, int SPT>
__device__ __forceinline__ EpiLds epi_lds_wide(float* p, int C, int NWx) {
  constexpr int EGW = 1 << PXB, kECorrB = bwd_band<PXB, SPT>() + 1;
  EpiLds L;
  L.aref = p;
  p += EGW * (C + 4);
  L.corr = p;
  p += EGW * kECorrB;
  L.list = reinterpret_cast<int*>(p);
  p += kEUMax;
  L.base = reinterpret_cast<uint32_t*>(p);
  p += NWx;
  p += (NWx & 1);
  L.wb = reinterpret_cast<uint2*>(p);
  p += 2 * NWx;
  L.nzw = reinterpret_cast<int*>(p);
  p += NWx;
  L.misc = reinterpret_cast<uint32_t*>(p);
  return L;
}
size_t epi_lds_bytes_wide(int pxb, int spt, int C, int H, int W) {
  const size_t egw = (size_t)1 << pxb, corr = (size_t)epi_pass(pxb, spt) + 1;
  return sizeof(float) * (egw * (C + 4) + egw * corr + kEUMax + 4 * epi_words(H, W) + 1 + 32);
}
// Forward, view j: grid.x = 8 * ceil(B * ngroups / 8) (XCD-contiguous, ngroups of 2^PXB
// pixels), grid.y = D chunks of (256 >> PXB) * SPT. Thread t has pixel t & (2^PXB - 1) and
// depths d0 + (t >> PXB) + (256 >> PXB) s. Writes (accumulate = 0) or adds (accumulate = 1:
// views after the first, launched in view order, so the sum over views is deterministic)
// scale * sum_taps w * corr. ref_hwc [B][HW + 1][C], tgt_hwc [B][J][HW + 1][C]: channel-last
// copies, row HW zero. tmap (views mode, round 6): tgt_hwc is the per-view copy [BV][HW + 1][C]
// (the same buffer as ref_hwc) and (b, j)'s target image is view tmap[b J + j].
template <int NK, int SPT, int PXB>
__global__ __launch_bounds__(256, PXB == 4 ? 4 : 2) void k_cost_epi(int B, int j, int J, int H, int W, int D,
                                                                  int depth_per_pixel, int accumulate,
                                                                  const float* __restrict__ ref_hwc,
                                                                  const float* __restrict__ tgt_hwc,
                                                                  const int* __restrict__ tmap,
                                                                  const int* __restrict__ groups,
                                                                  const float* __restrict__ geom,
                                                                  const float* __restrict__ depth, float clampz,
                                                                  float scale, float* __restrict__ cost) {
  constexpr int C = 4 * NK, EGW = 1 << PXB, MB = EGW / 16, DSL = 256 >> PXB;
  constexpr int kEU = bwd_band<PXB, SPT>(), kEC = kEU + 1;
  extern __shared__ __attribute__((aligned(16))) float cv_lds[];
  const int HW = H * W, ngw = (HW + EGW - 1) / EGW;
  int b, g;
  if (!epi_item(B, ngw, b, g)) return;
  const EpiLds L = epi_lds_wide<PXB, SPT>(cv_lds, C, epi_words(H, W));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i = tid & (EGW - 1), dl = tid >> PXB, d0 = blockIdx.y * DSL * SPT;
  const size_t bj = (size_t)b * J + j;
  __shared__ int s_gid[kEGWMax];
  if (tid < EGW) s_gid[tid] = g * EGW + tid < HW ? groups[bj * HW + g * EGW + tid] : -1;
  epi_clear_words(L, epi_words(H, W));
  __syncthreads();
  // depth loads, then the reference tile's loads, all in flight together; the taps go into the
  // base bitmap of their box while the tile's LDS stores drain, and one barrier covers both
  const int pix = s_gid[i];  // -1: past the last pixel
  float dep[SPT];
  epi_depths<SPT, PXB>(HW, D, depth_per_pixel, b, d0, pix, depth, dep);
  epi_aref<NK, EGW>(L, HW, b, s_gid, ref_hwc);
  const EpiRay ry = epi_ray(geom + bj * 12, pix >= 0 ? (float)(pix % W) : 0.f, pix >= 0 ? (float)(pix / W) : 0.f);
  float sx[SPT], sy[SPT];
  int es[SPT];
  epi_taps<SPT, PXB>(H, W, D, d0, pix, ry, dep, clampz, sx, sy, es);
  const EpiBox bx = epi_box<SPT>(L, es);
  epi_mark<SPT>(L, bx, es);
  __syncthreads();
  const int U = bx.nw ? epi_band(L, bx) : 0;
  const int Wx = bx.wb;
  // per sample: sum over its taps of grid_sample's weight x correlation, taps in a fixed order
  // (a band of more than kEU positions takes several passes, each adding its taps)
  float* cb = cost + (size_t)b * D * HW;  // this scene's cost volume (< 2^32 elements)
  float acc[SPT], prev[SPT];
#pragma unroll
  for (int s = 0; s < SPT; ++s) acc[s] = prev[s] = 0.f;
  auto load_prev = [&]() {
    int pc = max(pix, 0);
    asm volatile("" : "+v"(pc));  // addresses formed here, not hoisted (register pressure)
#pragma unroll
    for (int s = 0; s < SPT; ++s) prev[s] = cb[(uint32_t)(min(d0 + dl + DSL * s, D - 1) * HW + pc)];
  };
  const float* tg = tgt_hwc + cv_target(tmap, bj, B) * (size_t)(HW + 1) * C;
  for (int r0 = 0; r0 < U; r0 += kEU) {
    const int n = min(kEU, U - r0);
    epi_list(L, H, W, bx, r0, n);
    __syncthreads();
    // corr[EGW x n] = aref[EGW x C] . tgt[n x C]^T; per 16-channel step lane l feeds channels
    // cb + 4 (l >> 4) + s to MFMA s (A and B permuted alike). The C / 16 row loads of a
    // block are issued together and feed all MB row blocks.
    for (int blk = wv; blk * 16 < n; blk += 4) {
      const int u = blk * 16 + (lane & 15);
      const float* brow = tg + (size_t)L.list[u] * C + 4 * (lane >> 4);
      float4 bv[NK / 4];
#pragma unroll
      for (int t = 0; t < NK / 4; ++t) bv[t] = *reinterpret_cast<const float4*>(brow + 16 * t);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const float* arow = L.aref + (mb * 16 + (lane & 15)) * (C + 4) + 4 * (lane >> 4);
        f32x4 c4[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int t = 0; t < NK / 4; ++t) {
          const float4 av = *reinterpret_cast<const float4*>(arow + 16 * t);
          f32x4& a4 = c4[t & 1];  // two independent accumulation chains
          a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv[t].x, a4, 0, 0, 0);
          a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv[t].y, a4, 0, 0, 0);
          a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv[t].z, a4, 0, 0, 0);
          a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv[t].w, a4, 0, 0, 0);
        }
        // D[row][col]: col = lane & 15 (band position u), row = 4 (lane >> 4) + r (pixel)
#pragma unroll
        for (int r = 0; r < 4; ++r) L.corr[(mb * 16 + 4 * (lane >> 4) + r) * kEC + u] = c4[0][r] + c4[1][r];
      }
    }
    __syncthreads();
    if (r0 == 0 && accumulate) load_prev();  // the earlier views' sum, in flight across the gather
    const float* crow = L.corr + i * kEC;
    if (n == U) {
      // the one pass holds every tap: straight-line gather; a zero sample reads ranks 0 / 1
      // (written: the first 16 columns always are) with zero weights
#pragma unroll
      for (int s = 0; s < SPT; ++s) {
        const bool ok = es[s] >= 0;
        float x = ok ? sx[s] : 0.f, y = ok ? sy[s] : 0.f;
        int e = ok ? es[s] : 0;
        asm volatile("" : "+v"(x), "+v"(y), "+v"(e));  // weights formed here, not kept live across the GEMM
        int ra = epi_rank(L, e), rb = epi_rank(L, e + Wx);  // taps (0, 1), (2, 3)
        asm volatile("" : "+v"(ra), "+v"(rb));             // both reads issued, no branch
        ra = ok ? ra : 0;
        rb = ok ? rb : 0;
        const float fx0 = floorf(x), fy0 = floorf(y);
        const float wx0 = (fx0 + 1.f) - x, wx1 = x - fx0;
        const float wy0 = ok ? (fy0 + 1.f) - y : 0.f, wy1 = ok ? y - fy0 : 0.f;
        acc[s] = wx0 * wy0 * crow[ra] + wx1 * wy0 * crow[ra + 1] + wx0 * wy1 * crow[rb] + wx1 * wy1 * crow[rb + 1];
      }
    } else {
#pragma unroll
      for (int s = 0; s < SPT; ++s) {
        if (es[s] < 0) continue;
        float x = sx[s], y = sy[s];
        int e = es[s];
        asm volatile("" : "+v"(x), "+v"(y), "+v"(e));
        const int ra = epi_rank(L, e) - r0, rb = epi_rank(L, e + Wx) - r0;
        const float fx0 = floorf(x), fy0 = floorf(y);
        const float wx0 = (fx0 + 1.f) - x, wx1 = x - fx0, wy0 = (fy0 + 1.f) - y, wy1 = y - fy0;
        if (ra >= 0 && ra < n) acc[s] += wx0 * wy0 * crow[ra];
        if (ra + 1 >= 0 && ra + 1 < n) acc[s] += wx1 * wy0 * crow[ra + 1];
        if (rb >= 0 && rb < n) acc[s] += wx0 * wy1 * crow[rb];
        if (rb + 1 >= 0 && rb + 1 < n) acc[s] += wx1 * wy1 * crow[rb + 1];
      }
    }
    __syncthreads();  // list / corr reused by the next pass
  }
  if (pix < 0) return;
  if (U == 0 && accumulate) load_prev();  // no pass ran: no tap of this group is inside view j
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const int d = d0 + dl + DSL * s;
    if (d < D) cb[(uint32_t)(d * HW + pix)] = accumulate ? prev[s] + acc[s] * scale : acc[s] * scale;
  }
}

// Deterministic sums of the backward (round 5). Float atomics make a sum depend on the order in
// which the adds arrive, so the gradients differed run to run in the last bits. Both sums that
// several writers share are now integer (fixed point), whose result does not depend on order:
//   * G[p][u] (LDS): each add is dcost * scale * w rounded to units of 2^(kg - 23), kg the
//     exponent of the largest |dcost * scale| of the workgroup's depth chunk; an element takes at
//     most (256 >> PXB) SPT <= 128 adds of <= 2^23 units (one per sample of its pixel in the
//     chunk), so int32 never overflows;
//   * dtgt (HBM): each workgroup's MFMA partial G^T aref (a fixed-order float) rounded to units
//     of 2^(kt - 40), 2^kt bounding one partial (2^PXB pixels x (256 >> PXB) SPT samples each =
//     256 SPT x max|dcost scale| x max|ref|, from
//     the per-block maxima of k_cv_absmax, the same in every workgroup), added as int64: 2^23
//     partials of the bound fit. k_fx_to_chw converts the sum back to float while transposing.
// dref needs none of this: each element has one writer (its pixel's group, views in launch order).
// 256 workgroups of 1024 threads (16 waves per CU: the pass reads dcost and ref at HBM rate;
// 256 threads per workgroup ran at ~3.5 TB/s, 57 us at config D scale 1)
constexpr int kCvMaxBlocks = 256;
__global__ __launch_bounds__(1024) void k_cv_absmax(size_t n1, const float* __restrict__ a1, size_t n2,
                                                   const float* __restrict__ a2, float* __restrict__ out) {
  float m1 = 0.f, m2 = 0.f;
  const size_t stride = (size_t)1024 * gridDim.x, i0 = (size_t)blockIdx.x * 1024 + threadIdx.x;
  // 16-byte loads, 4 in flight per thread, then the scalar tail (an unaligned array: all scalar)
  auto vmax = [&](size_t n, const float* __restrict__ a, float& m) {
    const float4* a4 = reinterpret_cast<const float4*>(a);
    const size_t n4 = ((uintptr_t)a & 15u) == 0 ? n / 4 : 0;
    size_t i = i0;
    for (; i + 3 * stride < n4; i += 4 * stride) {
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = a4[i + k * stride];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[k].x), fabsf(v[k].y)), fmaxf(fabsf(v[k].z), fabsf(v[k].w))));
    }
    for (; i < n4; i += stride) {
      const float4 v = a4[i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    for (size_t t = n4 * 4 + i0; t < n; t += stride) m = fmaxf(m, fabsf(a[t]));
  };
  vmax(n1, a1, m1);
  vmax(n2, a2, m2);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    m1 = fmaxf(m1, __shfl_xor(m1, off, 64));
    m2 = fmaxf(m2, __shfl_xor(m2, off, 64));
  }
  __shared__ float s1[16], s2[16];
  if ((threadIdx.x & 63) == 0) {
    s1[threadIdx.x >> 6] = m1;
    s2[threadIdx.x >> 6] = m2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, c = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a = fmaxf(a, s1[k]);
      c = fmaxf(c, s2[k]);
    }
    out[blockIdx.x] = a;
    out[kCvMaxBlocks + blockIdx.x] = c;
  }
}
// The dtgt unit from the per-block maxima (every caller reads the same values). One partial is
// bounded by 2^lgS max|dcost| scale max|ref| (2^lgS = 256 SPT samples of a workgroup's chunk)
// and an element takes at most 2^lgP partials (one per workgroup and depth chunk of its image:
// host-computed), so unit = 2^(e1 + e2 + es + lgS + lgP - 62) keeps every sum below 2^62: the
// finest unit the int64 range allows for this shape (round 5 used 2^(kt - 40) whatever the shape:
// 12+ bits coarser at config D). The exponents are added as integers, so no intermediate product
// overflows; a non-finite maximum, or a unit beyond float range (where the float gradients
// themselves overflow), gives 0: the conversion below then writes NaN.
__device__ __forceinline__ float cv_dtgt_unit(const float* __restrict__ bm, float scale, int lgps) {
  const int lane = threadIdx.x & 63;
  float m1 = 0.f, m2 = 0.f;
#pragma unroll
  for (int k = 0; k < kCvMaxBlocks / 64; ++k) {
    m1 = fmaxf(m1, bm[k * 64 + lane]);
    m2 = fmaxf(m2, bm[kCvMaxBlocks + k * 64 + lane]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    m1 = fmaxf(m1, __shfl_xor(m1, off, 64));
    m2 = fmaxf(m2, __shfl_xor(m2, off, 64));
  }
  if (!(m1 <= 3.4e38f) || !(m2 <= 3.4e38f)) return 0.f;
  if (m1 == 0.f || m2 == 0.f) return 1.f;  // every partial is 0
  int e1 = 0, e2 = 0, es = 0;
  frexpf(m1, &e1);  // m1 < 2^e1
  frexpf(m2, &e2);
  frexpf(scale, &es);
  const int ue = e1 + e2 + es + lgps - 62;
  return ue > 127 ? 0.f : ldexpf(1.f, max(ue, -126));
}

// Backward, view j, on groups of 2^PXB reference pixels (round 5): 16 (a group of
// the grouping's order), or 32 / 64 = 2 / 4 consecutive groups (neighbours along one epipolar
// line, whose target bands overlap), depth chunks of (256 >> PXB) x SPT looped inside. Thread t
// has pixel t & (2^PXB - 1) and depths d0 + (t >> PXB) + (256 >> PXB) s. Per chunk the gradient
// weights G[p][u] = sum over p's samples' taps of dcost * scale * w (LDS, fixed point) over the
// union band of the workgroup's pixels, then
//   dref[p] += G[p, :] . tgt[band]   (MFMA, K = band; registers across passes and chunks)
//   dtgt[band] += G^T . aref         (MFMA, K = 2^PXB pixels; int64 fixed-point atomics).
// The dtgt atomics were the backward's largest cost (same-box A/B with them removed: config D
// scale 0 fwd + bwd 2.23 -> 1.34 ms, profiles/r05j_ab_cvbwd_atomics.log); a wider group issues
// them once per union position instead of once per group and position, at the price of GEMM
// work over the union band and fewer workgroups (bwd_pxb picks the width per shape).
// dref_hwc [B][HW][C] is written (view 0) or added to (views after it, in launch order): each
// pixel is in exactly one group per view. cvmax: k_cv_absmax's per-block maxima (dcost, ref).
template <int NK, int PXB, int SPT>
__global__ __launch_bounds__(256, bwd_occ(PXB, 4 * NK)) void k_cost_epi_bwd(int B, int j, int J, int H, int W, int D, int depth_per_pixel,
                                                      int accumulate, const float* __restrict__ ref_hwc,
                                                      const float* __restrict__ tgt_hwc, const int* __restrict__ tmap,
                                                      const int* __restrict__ groups, const float* __restrict__ geom,
                                                      const float* __restrict__ depth,
                                                      float clampz, float scale, const float* __restrict__ dcost,
                                                      const float* __restrict__ cvmax, int lgps,
                                                      float* __restrict__ dref_hwc, long long* __restrict__ dtgt_fx) {
  constexpr int C = 4 * NK, NCB = (C / 16 + 3) / 4;  // channel blocks per wave (dref)
  constexpr int EGW = 1 << PXB, MB = EGW / 16, DSL = 256 >> PXB;  // pixels, row blocks, depth slots
  constexpr int kEUMaxB = bwd_band<PXB, SPT>(), kECorrB = kEUMaxB + 1;
  extern __shared__ __attribute__((aligned(16))) float cv_lds[];
  const int HW = H * W, ngw = (HW + EGW - 1) / EGW;
  int b, g;
  if (!epi_item(B, ngw, b, g)) return;
  const EpiLds L = epi_lds_wide<PXB, SPT>(cv_lds, C, epi_words(H, W));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const size_t bj = (size_t)b * J + j;
  const float unit_t = cv_dtgt_unit(cvmax, scale, lgps);
  const float unit_t_inv = unit_t > 0.f ? 1.f / unit_t : 0.f;  // exact: a power of 2
  __shared__ int s_gid[kEGWMax];
  // per pixel of the group: the largest |dcost scale| of its samples in the current chunk (float
  // bits; LDS atomicMax), whose exponent sets that pixel's fixed-point unit for G (round 6: the
  // unit was per workgroup, so a pixel next to one with a 1e4x larger gradient kept ~4 bits)
  __shared__ uint32_t s_pmax[kEGWMax];
  if (tid < EGW) {
    s_gid[tid] = g * EGW + tid < HW ? groups[bj * HW + g * EGW + tid] : -1;
    s_pmax[tid] = 0u;
  }
  __syncthreads();
  // unit 2^(E - 149) and its inverse for a pixel whose bound has float exponent field E (every
  // |G| add then is < 2^23 units, at most DSL SPT <= 128 of them per element: int32 holds the
  // sum); E = 255 (inf / NaN gradient): unit 0, the pixel adds nothing
  auto unit_of = [&](int p) -> float {
    const uint32_t E = s_pmax[p] >> 23;
    return E == 255u ? 0.f : __uint_as_float((max(E, 23u) - 22u) << 23);
  };
  auto uinv_of = [&](int p) -> float {
    const uint32_t E = s_pmax[p] >> 23;
    return E == 255u ? 0.f : __uint_as_float((276u - max(E, 23u)) << 23);
  };
  epi_aref<NK, EGW>(L, HW, b, s_gid, ref_hwc);
  const int i = tid & (EGW - 1), dl = tid >> PXB;
  const int pix = s_gid[i];
  const EpiRay ry = epi_ray(geom + bj * 12, pix >= 0 ? (float)(pix % W) : 0.f, pix >= 0 ? (float)(pix / W) : 0.f);
  // views mode: (b, j)'s target view; its gradient accumulates in that view's rows (int64 sums:
  // the order of the (b, j) pairs sharing a view does not matter)
  const size_t tb = cv_target(tmap, bj, B);
  const float* tg = tgt_hwc + tb * (size_t)(HW + 1) * C;
  long long* dtg = dtgt_fx + tb * (size_t)(HW + 1) * C;
  int* gi = reinterpret_cast<int*>(L.corr);  // G in fixed point, [EGW][kECorrB]
  f32x4 dacc[NCB][MB];
#pragma unroll
  for (int q = 0; q < NCB; ++q)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) dacc[q][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
  int nw_prev = epi_words(H, W);
  for (int d0 = 0; d0 < D; d0 += DSL * SPT) {  // depth chunks in turn
    float gs[SPT];
    {
      const float* gp = dcost + (size_t)b * D * HW;
#pragma unroll
      for (int s = 0; s < SPT; ++s) gs[s] = gp[(uint32_t)(min(d0 + dl + DSL * s, D - 1) * HW + max(pix, 0))];
    }
    float sx[SPT], sy[SPT];
    int es[SPT];
    EpiBox bx;
    const int U = epi_front<SPT, PXB>(L, H, W, HW, D, depth_per_pixel, b, d0, pix, ry, depth, clampz, sx, sy, es, bx,
                                      nw_prev);
    nw_prev = bx.nw;
    const int Wx = bx.wb;
    // the pixel's fixed-point unit for this chunk (unit_of): from its samples' largest |dcost scale|
    float gm = 0.f;
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      gs[s] = es[s] >= 0 ? gs[s] * scale : 0.f;
      gm = fmaxf(gm, fabsf(gs[s]));
    }
    if (gm != 0.f) atomicMax(&s_pmax[i], __float_as_uint(gm));  // (non-negative: orderable as uint)
    for (int r0 = 0; r0 < U; r0 += kEUMaxB) {
      const int n = min(kEUMaxB, U - r0), np = epi_padded(n);
      for (int k = tid; k < EGW * np; k += 256) gi[(k & (EGW - 1)) * kECorrB + (k >> PXB)] = 0;
      epi_list(L, H, W, bx, r0, n);
      __syncthreads();
      const float unit_g_inv = uinv_of(i);
      int* grow = gi + i * kECorrB;
#pragma unroll
      for (int s = 0; s < SPT; ++s) {
        if (gs[s] == 0.f) continue;
        float x = sx[s], y = sy[s];
        int e = es[s];
        asm volatile("" : "+v"(x), "+v"(y), "+v"(e));
        const float fx0 = floorf(x), fy0 = floorf(y);
        const float wx0 = (fx0 + 1.f) - x, wx1 = x - fx0, wy0 = (fy0 + 1.f) - y, wy1 = y - fy0;
        const int ra = epi_rank(L, e) - r0, rb = epi_rank(L, e + Wx) - r0;
        const float gu = gs[s] * unit_g_inv;
        if (ra >= 0 && ra < n) atomicAdd(&grow[ra], (int)rintf(gu * (wx0 * wy0)));
        if (ra + 1 >= 0 && ra + 1 < n) atomicAdd(&grow[ra + 1], (int)rintf(gu * (wx1 * wy0)));
        if (rb >= 0 && rb < n) atomicAdd(&grow[rb], (int)rintf(gu * (wx0 * wy1)));
        if (rb + 1 >= 0 && rb + 1 < n) atomicAdd(&grow[rb + 1], (int)rintf(gu * (wx1 * wy1)));
      }
      __syncthreads();
      // dref[EGW x C] += G[EGW x np] . tgt[np x C]: wave wv owns channel blocks wv, wv + 4, ...
      // for all MB row blocks (one target load feeds MB MFMAs); 32 band positions per batch
      float urow[MB];  // the units of this lane's A rows (pixel mb 16 + (lane & 15))
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) urow[mb] = unit_of(mb * 16 + (lane & 15));
      if constexpr (C == 128 && PXB == 5) {
        // the wave's two channel blocks (wv, wv + 4) in one sweep: each A fragment loaded once
        // for both (the same MFMA order per accumulator: bit-identical)
        const float* tc0 = tg + wv * 16 + (lane & 15);
        const float* tc1 = tc0 + 64;
        for (int u0 = 0; u0 < np; u0 += kEPad) {
          float b0[kEPad / 4], b1[kEPad / 4];
#pragma unroll
          for (int t = 0; t < kEPad / 4; ++t) {
            const size_t o = (size_t)L.list[u0 + 4 * t + (lane >> 4)] * C;
            b0[t] = tc0[o];
            b1[t] = tc1[o];
          }
#pragma unroll
          for (int t = 0; t < kEPad / 4; ++t) {
            const int u = u0 + 4 * t + (lane >> 4);
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) {
              const float av = (float)gi[(mb * 16 + (lane & 15)) * kECorrB + u] * urow[mb];
              dacc[0][mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0[t], dacc[0][mb], 0, 0, 0);
              dacc[1][mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1[t], dacc[1][mb], 0, 0, 0);
            }
          }
        }
      } else
#pragma unroll
      for (int q = 0; q < NCB; ++q) {
        const int cbk = wv + 4 * q;
        if (cbk >= C / 16) break;  // wave-uniform
        const float* tcol = tg + cbk * 16 + (lane & 15);
        for (int u0 = 0; u0 < np; u0 += kEPad) {
          float bv[kEPad / 4];
#pragma unroll
          for (int t = 0; t < kEPad / 4; ++t) bv[t] = tcol[(size_t)L.list[u0 + 4 * t + (lane >> 4)] * C];
#pragma unroll
          for (int t = 0; t < kEPad / 4; ++t) {
            const int u = u0 + 4 * t + (lane >> 4);
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
              dacc[q][mb] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)gi[(mb * 16 + (lane & 15)) * kECorrB + u] * urow[mb],
                                                                 bv[t], dacc[q][mb], 0, 0, 0);
          }
        }
      }
      // dtgt[n x C] += G^T[n x EGW] . aref[EGW x C], added as int64 fixed point
      const int nub = np / 16;
      auto add_dtgt = [&](const f32x4& acc, int q, int r, int cbk) {
        if (q < HW && acc[r] != 0.f) {
          const long long v = (long long)rintf(fminf(fmaxf(acc[r] * unit_t_inv, -4.0e18f), 4.0e18f));
          if (v != 0ll)
            atomicAdd(reinterpret_cast<unsigned long long*>(&dtg[(size_t)q * C + cbk * 16 + (lane & 15)]),
                      (unsigned long long)v);
        }
      };
      if constexpr (PXB == 6 || (PXB == 5 && C == 128)) {
        // band blocks over the waves: a block's A fragments (G^T rows in float, times the
        // pixels' units) loaded once and reused over every channel block (the same MFMA order:
        // bit-identical; scale 1 fwd + bwd -1 %, profiles/r06at_ab_cvbwd_dtgt.txt; half the
        // channel blocks per item was slower; the other 32-pixel instances, at 4 waves per
        // SIMD, would spill)
        for (int ub = wv; ub < nub; ub += 4) {
          float af[EGW / 4];
#pragma unroll
          for (int kk = 0; kk < EGW / 4; ++kk) {
            const int p = 4 * kk + (lane >> 4);
            af[kk] = (float)gi[p * kECorrB + ub * 16 + (lane & 15)] * unit_of(p);
          }
          int qr[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) qr[r] = L.list[ub * 16 + 4 * (lane >> 4) + r];
#pragma unroll 1
          for (int cbk = 0; cbk < C / 16; ++cbk) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < EGW / 4; ++kk)
              acc = __builtin_amdgcn_mfma_f32_16x16x4f32(
                  af[kk], L.aref[(4 * kk + (lane >> 4)) * (C + 4) + cbk * 16 + (lane & 15)], acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) add_dtgt(acc, qr[r], r, cbk);
          }
        }
      } else {  // (band block, channel block) pairs over the waves
        for (int pr = wv; pr < nub * (C / 16); pr += 4) {
          const int ub = pr / (C / 16), cbk = pr - ub * (C / 16);
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k0 = 0; k0 < EGW; k0 += 4) {
            const int u = ub * 16 + (lane & 15), p = k0 + (lane >> 4);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32((float)gi[p * kECorrB + u] * unit_of(p),
                                                       L.aref[p * (C + 4) + cbk * 16 + (lane & 15)], acc, 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) add_dtgt(acc, L.list[ub * 16 + 4 * (lane >> 4) + r], r, cbk);
        }
      }
      __syncthreads();  // G / list reused by the next pass
    }
    // every read of this chunk's units is behind the last barrier above (no pass: none); the next
    // chunk's atomicMax is behind epi_front's barriers
    if (tid < EGW) s_pmax[tid] = 0u;
  }
  // the group's reference-gradient rows, channel-last: dacc[q][mb][r] is row
  // 16 mb + 4 (lane >> 4) + r, channel 16 (wv + 4 q) + (lane & 15)
#pragma unroll
  for (int q = 0; q < NCB; ++q) {
    const int cbk = wv + 4 * q;
    if (cbk >= C / 16) break;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = s_gid[mb * 16 + 4 * (lane >> 4) + r];
        if (p < 0) continue;
        float* o = dref_hwc + ((size_t)b * HW + p) * C + cbk * 16 + (lane & 15);
        *o = accumulate ? *o + dacc[q][mb][r] : dacc[q][mb][r];
      }
  }
}

// [n][rows][C] int64 fixed point (the first HW rows) -> [n][C][HW] float, times the unit of
// k_cost_epi_bwd (cv_dtgt_unit, recomputed from the same maxima); add (views mode: the reference
// gradient [n][HW][C], float) is added to each element (one fixed-order add: deterministic)
__global__ __launch_bounds__(256) void k_fx_to_chw(int C, int HW, int rows, const long long* __restrict__ src,
                                                   const float* __restrict__ cvmax, float scale, int lgps,
                                                   const float* __restrict__ add, float* __restrict__ dst) {
  __shared__ float tile[64][65];
  const float unit = cv_dtgt_unit(cvmax, scale, lgps);
  const bool ok = unit > 0.f;
  const int bj = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const long long* s = src + (size_t)bj * rows * C;
  float* d = dst + (size_t)bj * C * HW;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int p = p0 + r, c = c0 + tx;
    const long long q = (p < HW && c < C) ? s[(size_t)p * C + c] : 0ll;
    const int hi = (int)(q >> 32);
    const unsigned lo = (unsigned)(q & 0xffffffffll);
    // (hi unit first: 2^32 unit may exceed float range where the value itself does not)
    float v = ok ? fmaf((float)hi * unit, 4294967296.0f, (float)lo * unit) : __builtin_nanf("");
    if (add && p < HW && c < C) v += add[((size_t)bj * HW + p) * C + c];
    tile[r][tx] = v;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, p = p0 + tx;
    if (c < C && p < HW) d[(size_t)c * HW + p] = tile[tx][r];
  }
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// k_fx_to_chw with 16-byte accesses (C % 4 == 0, HW % 4 == 0, 16-byte aligned arrays): each
// thread reads 4 consecutive channels of one pixel (2 x 16 B of int64, + 16 B of add) and
// writes 4 consecutive pixels of one channel (the 4-byte form moved ~4.7 TB/s).
__global__ __launch_bounds__(256) void k_fx_to_chw4(int C, int HW, int rows, const long long* __restrict__ src,
                                                    const float* __restrict__ cvmax, float scale, int lgps,
                                                    const float* __restrict__ add, float* __restrict__ dst) {
  __shared__ float tile[64][65];
  const float unit = cv_dtgt_unit(cvmax, scale, lgps);
  const bool ok = unit > 0.f;
  const int bj = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const long long* s = src + (size_t)bj * rows * C;
  float* d = dst + (size_t)bj * C * HW;
  const int q = threadIdx.x & 15, rr = threadIdx.x >> 4;
  auto cvt = [&](long long v) {
    return ok ? fmaf((float)(int)(v >> 32) * unit, 4294967296.0f, (float)(unsigned)(v & 0xffffffffll) * unit)
              : __builtin_nanf("");
  };
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = p0 + rr + 16 * k, c = c0 + 4 * q;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p < HW && c < C) {
      const longlong2* sp = reinterpret_cast<const longlong2*>(s + (size_t)p * C + c);
      const longlong2 a01 = sp[0], a23 = sp[1];
      v = make_float4(cvt(a01.x), cvt(a01.y), cvt(a23.x), cvt(a23.y));
      if (add) {
        const float4 w = *reinterpret_cast<const float4*>(add + ((size_t)bj * HW + p) * C + c);
        v.x += w.x;
        v.y += w.y;
        v.z += w.z;
        v.w += w.w;
      }
    }
    float* t = &tile[rr + 16 * k][4 * q];  // tile[p - p0][c - c0]
    t[0] = v.x;
    t[1] = v.y;
    t[2] = v.z;
    t[3] = v.w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + rr + 16 * k, p = p0 + 4 * q;
    if (c < C && p < HW)
      *reinterpret_cast<float4*>(d + (size_t)c * HW + p) =
          make_float4(tile[4 * q][rr + 16 * k], tile[4 * q + 1][rr + 16 * k], tile[4 * q + 2][rr + 16 * k],
                      tile[4 * q + 3][rr + 16 * k]);
  }
}

// [n][rows][C] int64 -> [n][C][HW] float (+ add): the 16-byte form where the shape allows
static int fx_to_chw(int n, int C, int HW, const long long* src, const float* cvmax, float scale, int lgps,
                     const float* add, float* dst, hipStream_t st) {
  const dim3 grid((HW + 63) / 64, (C + 63) / 64, n);
  if (C % 4 == 0 && HW % 4 == 0 && aligned16(src) && aligned16(dst) && (!add || aligned16(add)))
    k_fx_to_chw4<<<grid, 256, 0, st>>>(C, HW, HW + 1, src, cvmax, scale, lgps, add, dst);
  else
    k_fx_to_chw<<<grid, 256, 0, st>>>(C, HW, HW + 1, src, cvmax, scale, lgps, add, dst);
  return dsplat::check_launch("k_fx_to_chw");
}

// ---- forward on the matrix cores, band form (small grids: configs A / B) ---------------
// Round-2 kernel, kept for shapes where one epipolar group per workgroup underfills the chip
// (band_fwd below): one launch, no channel-last copies and no grouping pass.
// One workgroup per (16 reference pixels of a row, 64 depth hypotheses): thread t owns pixel
// t & 15 and depths (t >> 4) + 16 s, s < 4, and keeps those samples' positions in registers.
// Per source view the workgroup takes the bounding box of every target pixel its samples tap
// (a block min / max: no LDS atomics, no bitmap), computes the correlations of its 16
// reference pixels with ALL box pixels as one exact-f32 GEMM on v_mfma_f32_16x16x4_f32
// (A = the reference tile, loaded once into registers straight from [B,C,H,W]; B = target
// columns loaded straight from [B,J,C,H,W], no channel-last copy), and finishes with the
// 4-tap bilinear gather from LDS. A small-baseline epipolar band fills its box (a few tens
// to a few hundred pixels at these scales); a box above kBandMax pixels is computed by direct
// dot products from global memory instead (wide, scattered taps; rare).
constexpr int BTP = 16;                       // reference pixels per workgroup
constexpr int BDCH = 64;                      // depth hypotheses per workgroup
constexpr int BSPT = BTP * BDCH / 256;        // samples per thread
constexpr int kBandMax = 512;                 // box pixels whose correlations fit in LDS (33 KB:
                                              // 4 workgroups per CU, all of config B's in one round)
constexpr int kCorrStride = kBandMax + 1;     // odd row stride: the gather's lanes spread over banks

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
  return v;
}

template <int NK>  // NK = C / 4 matrix-core steps
__global__ __launch_bounds__(256) void k_cost_band(int J, int H, int W, int D, int depth_per_pixel,
                                                   const float* __restrict__ ref, const float* __restrict__ tgt,
                                                   const float* __restrict__ intr, const float* __restrict__ pose,
                                                   const float* __restrict__ depth, float clampz,
                                                   float* __restrict__ cost) {
  constexpr int C = 4 * NK;
  extern __shared__ __attribute__((aligned(16))) float cv_lds[];
  float* s_corr = cv_lds;                                           // [BTP][kCorrStride]
  int* s_box = reinterpret_cast<int*>(cv_lds + BTP * kCorrStride);  // [4 waves][4]
  const int HW = H * W;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int tpr = (W + BTP - 1) / BTP;
  const int y = blockIdx.x / tpr, x0 = (blockIdx.x % tpr) * BTP;
  const int b = blockIdx.y, d0 = blockIdx.z * BDCH;
  const int i = tid & (BTP - 1), dl = tid >> 4;
  const int px = x0 + i;
  const float scale = 1.0f / (sqrtf((float)C) * (float)J);
  // A operand (v_mfma_f32_16x16x4f32: lane l holds A[l & 15][l >> 4]): channel 4 s + (l >> 4) of
  // reference pixel x0 + (l & 15), for every step s — the whole 16 x C tile in NK registers
  float a[NK];
  {
    const int ax = x0 + (lane & 15);
    const float* rp = ref + ((size_t)b * C + (lane >> 4)) * HW + (size_t)y * W + ax;
#pragma unroll
    for (int s = 0; s < NK; ++s) a[s] = ax < W ? rp[(size_t)4 * s * HW] : 0.f;
  }
  float acc[BSPT];
#pragma unroll
  for (int s = 0; s < BSPT; ++s) acc[s] = 0.f;
  for (int j = 0; j < J; ++j) {
    Cam cam;
    load_cam(intr + ((size_t)b * J + j) * 9, pose + ((size_t)b * J + j) * 16, cam);
    // sample positions (reference operation order, as k_cost_mfma) and the taps' bounding box
    float sx[BSPT], sy[BSPT];
    int bx0 = 0x7fffffff, bx1 = -1, by0 = 0x7fffffff, by1 = -1;
    {
      const float fpx = (float)px, fpy = (float)y;
      const float qx = cam.Kinv[0] * fpx + cam.Kinv[1] * fpy + cam.Kinv[2];
      const float qy = cam.Kinv[3] * fpx + cam.Kinv[4] * fpy + cam.Kinv[5];
      const float qz = cam.Kinv[6] * fpx + cam.Kinv[7] * fpy + cam.Kinv[8];
      const float prx = cam.R[0] * qx + cam.R[1] * qy + cam.R[2] * qz;
      const float pry = cam.R[3] * qx + cam.R[4] * qy + cam.R[5] * qz;
      const float prz = cam.R[6] * qx + cam.R[7] * qy + cam.R[8] * qz;
#pragma unroll
      for (int s = 0; s < BSPT; ++s) {
        const int d = d0 + dl + 16 * s;
        sx[s] = __int_as_float(0x7fc00000);
        sy[s] = 0.f;
        if (d < D && px < W) {
          const float dep = depth_per_pixel ? depth[((size_t)b * D + d) * HW + (size_t)y * W + px]
                                            : depth[(size_t)b * D + d];
          const float X = prx * dep + cam.t[0];
          const float Y = pry * dep + cam.t[1];
          const float Z = prz * dep + cam.t[2];
          const float xx = cam.K[0] * X + cam.K[1] * Y + cam.K[2] * Z;
          const float yy = cam.K[3] * X + cam.K[4] * Y + cam.K[5] * Z;
          const float zz = fmaxf(cam.K[6] * X + cam.K[7] * Y + cam.K[8] * Z, clampz);
          const float u = xx / zz, v = yy / zz;
          const float gxn = 2 * u / (W - 1) - 1;
          const float gyn = 2 * v / (H - 1) - 1;
          const float ix = ((gxn + 1) / 2) * (W - 1);
          const float iy = ((gyn + 1) / 2) * (H - 1);
          if (ix > -2.f && ix < (float)W + 1.f && iy > -2.f && iy < (float)H + 1.f) {
            sx[s] = ix;
            sy[s] = iy;
            const int tx = (int)floorf(ix), ty = (int)floorf(iy);
            const int cx0 = max(tx, 0), cx1 = min(tx + 1, W - 1), cy0 = max(ty, 0), cy1 = min(ty + 1, H - 1);
            if (cx0 <= cx1 && cy0 <= cy1) {
              bx0 = min(bx0, cx0);
              bx1 = max(bx1, cx1);
              by0 = min(by0, cy0);
              by1 = max(by1, cy1);
            }
          }
        }
      }
    }
    bx0 = wave_min_i(bx0);
    by0 = wave_min_i(by0);
    bx1 = wave_max_i(bx1);
    by1 = wave_max_i(by1);
    if (lane == 0) {
      s_box[wv * 4] = bx0;
      s_box[wv * 4 + 1] = bx1;
      s_box[wv * 4 + 2] = by0;
      s_box[wv * 4 + 3] = by1;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bx0 = min(bx0, s_box[k * 4]);
      bx1 = max(bx1, s_box[k * 4 + 1]);
      by0 = min(by0, s_box[k * 4 + 2]);
      by1 = max(by1, s_box[k * 4 + 3]);
    }
    const float* tg = tgt + ((size_t)b * J + j) * (size_t)C * HW;
    if (bx1 >= bx0) {  // uniform: some sample taps the image
      const int bw = bx1 - bx0 + 1, U = bw * (by1 - by0 + 1);
      if (U <= kBandMax) {
        // corr[16 x U] on the matrix cores: wave wv takes column blocks wv, wv + 4, ...
        const int nblk = (U + 15) / 16;
        for (int blk = wv; blk < nblk; blk += 4) {
          const int u = blk * 16 + (lane & 15);
          int q = -1;
          if (u < U) {
            const int r = u / bw;
            q = (by0 + r) * W + bx0 + (u - r * bw);
          }
          float bv[NK];
          const float* bp = tg + (size_t)(lane >> 4) * HW + (q < 0 ? 0 : q);
#pragma unroll
          for (int s = 0; s < NK; ++s) bv[s] = q >= 0 ? bp[(size_t)4 * s * HW] : 0.f;
          // four independent accumulation chains (a dependent v_mfma_f32_16x16x4f32 waits ~40
          // cycles for its accumulator), summed at the end
          f32x4 c4[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) c4[k] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < NK; ++s) c4[s & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bv[s], c4[s & 3], 0, 0, 0);
          c4[0] = (c4[0] + c4[1]) + (c4[2] + c4[3]);
          // D[row][col]: col = lane & 15 (box pixel u), row = 4 (lane >> 4) + r (reference pixel)
#pragma unroll
          for (int r = 0; r < 4; ++r) s_corr[(4 * (lane >> 4) + r) * kCorrStride + u] = c4[0][r];
        }
        __syncthreads();
        const float* crow = s_corr + i * kCorrStride;
#pragma unroll
        for (int s = 0; s < BSPT; ++s) {
          if (!(sx[s] == sx[s])) continue;
          const float fx0 = floorf(sx[s]), fy0 = floorf(sy[s]);
          const int tx0 = (int)fx0, ty0 = (int)fy0;
          const float wx0 = (float)(tx0 + 1) - sx[s], wx1 = sx[s] - fx0, wy0 = (float)(ty0 + 1) - sy[s],
                      wy1 = sy[s] - fy0;
          const float wt[4] = {wx0 * wy0, wx1 * wy0, wx0 * wy1, wx1 * wy1};
          float sum = 0.f;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1);
            if (tx >= 0 && tx < W && ty >= 0 && ty < H) sum += wt[t] * crow[(ty - by0) * bw + (tx - bx0)];
          }
          acc[s] += sum;
        }
      } else {
        // the box is too large for LDS: each tap's dot product over C straight from memory
#pragma unroll
        for (int s = 0; s < BSPT; ++s) {
          if (!(sx[s] == sx[s])) continue;
          const float fx0 = floorf(sx[s]), fy0 = floorf(sy[s]);
          const int tx0 = (int)fx0, ty0 = (int)fy0;
          const float wx0 = (float)(tx0 + 1) - sx[s], wx1 = sx[s] - fx0, wy0 = (float)(ty0 + 1) - sy[s],
                      wy1 = sy[s] - fy0;
          const float wt[4] = {wx0 * wy0, wx1 * wy0, wx0 * wy1, wx1 * wy1};
          float sum = 0.f;
          for (int t = 0; t < 4; ++t) {
            const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1);
            if (!(tx >= 0 && tx < W && ty >= 0 && ty < H)) continue;
            const float* rp = ref + (size_t)b * C * HW + (size_t)y * W + px;
            const float* qp = tg + (size_t)ty * W + tx;
            float dot = 0.f;
            for (int c = 0; c < C; ++c) dot += rp[(size_t)c * HW] * qp[(size_t)c * HW];
            sum += wt[t] * dot;
          }
          acc[s] += sum;
        }
      }
    }
    __syncthreads();  // s_corr / s_box reused by the next view
  }
#pragma unroll
  for (int s = 0; s < BSPT; ++s) {
    const int d = d0 + dl + 16 * s;
    if (d < D && px < W) cost[((size_t)b * D + d) * HW + (size_t)y * W + px] = acc[s] * scale;
  }
}

size_t cost_band_lds_bytes() { return (size_t)(BTP * kCorrStride + 16) * sizeof(float); }

// Backward: one wave per (b, pixel); lanes over channels.
//   dref[c,p]   += sum_{j,d} g(d) * warp_j[c,d,p]
//   dtgt[q,c]   += g(d) * w_k * ref[c,p] for each tap (atomics into channel-last scratch)
__global__ __launch_bounds__(256) void k_cost_bwd(int J, int C, int H, int W, int D, int depth_per_pixel,
                                                  const float* __restrict__ ref, const float* __restrict__ tgt_hwc,
                                                  const float* __restrict__ intr, const float* __restrict__ pose,
                                                  const float* __restrict__ depth, float clampz,
                                                  const float* __restrict__ dcost, float* __restrict__ dref,
                                                  float* __restrict__ dtgt_hwc) {
  const int HW = H * W;
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= HW) return;
  const float px = (float)(p % W), py = (float)(p / W);
  const float scale = 1.0f / (sqrtf((float)C) * (float)J);
  for (int c0 = 0; c0 < C; c0 += 64) {
    const int c = c0 + lane;
    const bool cv = c < C;
    const float r = cv ? ref[((size_t)b * C + c) * HW + p] : 0.f;
    float dr = 0.f;
    for (int j = 0; j < J; ++j) {
      Cam cam;
      load_cam(intr + ((size_t)b * J + j) * 9, pose + ((size_t)b * J + j) * 16, cam);
      const float qx = cam.Kinv[0] * px + cam.Kinv[1] * py + cam.Kinv[2];
      const float qy = cam.Kinv[3] * px + cam.Kinv[4] * py + cam.Kinv[5];
      const float qz = cam.Kinv[6] * px + cam.Kinv[7] * py + cam.Kinv[8];
      const float prx = cam.R[0] * qx + cam.R[1] * qy + cam.R[2] * qz;
      const float pry = cam.R[3] * qx + cam.R[4] * qy + cam.R[5] * qz;
      const float prz = cam.R[6] * qx + cam.R[7] * qy + cam.R[8] * qz;
      const float* tg = tgt_hwc + ((size_t)b * J + j) * (HW + 1) * C;
      float* dtg = dtgt_hwc + ((size_t)b * J + j) * (HW + 1) * C;
      for (int d = 0; d < D; ++d) {
        const float g = dcost[((size_t)b * D + d) * HW + p] * scale;
        if (g == 0.f) continue;
        const float dep = depth_per_pixel ? depth[((size_t)b * D + d) * HW + p] : depth[(size_t)b * D + d];
        Taps tp;
        taps_at(cam, prx, pry, prz, dep, clampz, H, W, tp);
        const float gr = g * r;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (tp.idx[k] >= 0 && cv) {
            dr += g * tp.w[k] * tg[(size_t)tp.idx[k] * C + c];
            atomicAdd(&dtg[(size_t)tp.idx[k] * C + c], gr * tp.w[k]);
          }
        }
      }
    }
    if (cv) dref[((size_t)b * C + c) * HW + p] = dr;
  }
}

// Materialising warp: out[b, c, d, y, x]. Thread per (b, d, pixel), loop over channels
// (feature in [B,C,H,W]; out written coalesced across pixels).
__global__ __launch_bounds__(256) void k_warp(int C, int H, int W, int D, const float* __restrict__ feat,
                                              const float* __restrict__ intr, const float* __restrict__ pose,
                                              const float* __restrict__ depth, float clampz,
                                              float* __restrict__ out) {
  const int HW = H * W;
  const int b = blockIdx.z, d = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= HW) return;
  Cam cam;
  load_cam(intr + (size_t)b * 9, pose + (size_t)b * 16, cam);
  const float px = (float)(p % W), py = (float)(p / W);
  const float qx = cam.Kinv[0] * px + cam.Kinv[1] * py + cam.Kinv[2];
  const float qy = cam.Kinv[3] * px + cam.Kinv[4] * py + cam.Kinv[5];
  const float qz = cam.Kinv[6] * px + cam.Kinv[7] * py + cam.Kinv[8];
  const float prx = cam.R[0] * qx + cam.R[1] * qy + cam.R[2] * qz;
  const float pry = cam.R[3] * qx + cam.R[4] * qy + cam.R[5] * qz;
  const float prz = cam.R[6] * qx + cam.R[7] * qy + cam.R[8] * qz;
  Taps tp;
  taps_at(cam, prx, pry, prz, depth[((size_t)b * D + d) * HW + p], clampz, H, W, tp);
  const float* f = feat + (size_t)b * C * HW;
  for (int c = 0; c < C; ++c) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (tp.idx[k] >= 0) s += tp.w[k] * f[(size_t)c * HW + tp.idx[k]];
    out[(((size_t)b * C + c) * D + d) * HW + p] = s;
  }
}

// Backward of k_warp w.r.t. the feature map: scatter-add through the same bilinear taps.
__global__ __launch_bounds__(256) void k_warp_bwd(int C, int H, int W, int D, const float* __restrict__ dout,
                                                  const float* __restrict__ intr, const float* __restrict__ pose,
                                                  const float* __restrict__ depth, float clampz,
                                                  float* __restrict__ dfeat) {
  const int HW = H * W;
  const int b = blockIdx.z, d = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= HW) return;
  Cam cam;
  load_cam(intr + (size_t)b * 9, pose + (size_t)b * 16, cam);
  const float px = (float)(p % W), py = (float)(p / W);
  const float qx = cam.Kinv[0] * px + cam.Kinv[1] * py + cam.Kinv[2];
  const float qy = cam.Kinv[3] * px + cam.Kinv[4] * py + cam.Kinv[5];
  const float qz = cam.Kinv[6] * px + cam.Kinv[7] * py + cam.Kinv[8];
  const float prx = cam.R[0] * qx + cam.R[1] * qy + cam.R[2] * qz;
  const float pry = cam.R[3] * qx + cam.R[4] * qy + cam.R[5] * qz;
  const float prz = cam.R[6] * qx + cam.R[7] * qy + cam.R[8] * qz;
  Taps tp;
  taps_at(cam, prx, pry, prz, depth[((size_t)b * D + d) * HW + p], clampz, H, W, tp);
  float* f = dfeat + (size_t)b * C * HW;
  for (int c = 0; c < C; ++c) {
    const float g = dout[(((size_t)b * C + c) * D + d) * HW + p];
    if (g == 0.f) continue;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (tp.idx[k] >= 0) atomicAdd(&f[(size_t)c * HW + tp.idx[k]], g * tp.w[k]);
  }
}

}  // namespace

extern "C" {

int dcv_warp_bwd(int B, int C, int H, int W, int D, const float* dout, const float* intr, const float* pose,
                 const float* depth, float clamp_min_depth, float* dfeature, void* stream) {
  DSPLAT_REQUIRE(B > 0 && C > 0 && H > 1 && W > 1 && D > 0, "dcv_warp_bwd: bad sizes");
  DSPLAT_REQUIRE(dout && intr && pose && depth && dfeature, "dcv_warp_bwd: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int HW = H * W;
  if (int e = dsplat::zero_async(dfeature, (size_t)B * C * HW * 4, st, "zero dfeature")) return e;
  k_warp_bwd<<<dim3((HW + 255) / 256, D, B), 256, 0, st>>>(C, H, W, D, dout, intr, pose, depth, clamp_min_depth,
                                                           dfeature);
  return dsplat::check_launch("k_warp_bwd");
}

// forward workspace: tgt_hwc [B][J][HW + 1][C] | ref_hwc [B][HW + 1][C] | groups [B][J][HW] | geom [B][J][12]
// | the grouping passes' scratch (EpiScratch)
size_t dcv_cost_volume_workspace_size(int B, int J, int C, int H, int W) {
  if (B <= 0 || J <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
  const size_t rows = (size_t)H * W + 1;
  return ((size_t)B * J * rows * C + (size_t)B * rows * C + (size_t)B * J * 12) * sizeof(float) +
         (size_t)B * J * H * W * sizeof(int32_t) + epi_scratch_words(B * J, H * W) * sizeof(uint32_t);
}
// backward workspace: dtgt [B][J][HW + 1][C] (int64 fixed point on the matrix-core path, float
// on the direct one) | dref_hwc [B][HW][C] float | per-block maxima of |dcost| and |ref|
size_t dcv_cost_volume_bwd_workspace_size(int B, int J, int C, int H, int W) {
  if (B <= 0 || J <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
  return (size_t)B * J * ((size_t)H * W + 1) * C * sizeof(long long) + (size_t)B * H * W * C * sizeof(float) +
         2 * kCvMaxBlocks * sizeof(float);
}

// group width (log2 pixels) and samples per thread (depth chunk = (256 >> pxb) spt) of the
// epipolar kernels
struct BwdShape {
  int pxb, spt;
};
// The forward keeps 16-pixel groups: wider ones lost at every shape (same-box A/B,
// profiles/r05r_ab_cvfwd_width.log, fwd ms at widths 16 / 32 / 64: config D scale 1
// 0.855 / 1.11 / 1.12, scale 0 0.437 / 0.64 / 0.955): neighbouring groups' windows sit at
// different places along their line, so the union band is close to the sum of the bands and
// the GEMM and gather grow with it, while the set-up it saves is a small part of a workgroup.
static BwdShape fwd_shape(int D) { return {4, D <= 32 ? 2 : 8}; }
// Same-box A/B (profiles/r05n_ab_cvbwd_width.log, fwd + bwd ms, widths 16 / 32 / 64):
// config D scale 1 (per-pixel candidates, D = 32) 3.38 / 3.15 / 3.00; scale 0 (per-image,
// D = 128: every group's band is a long stretch of its line, the union grows almost as fast as
// the pixels) 2.25 / 2.18 / 2.79; config B (512 groups: a wide group underfills the chip) best
// at 16.
static BwdShape bwd_shape(int B, int H, int W, int D, int depth_per_pixel) {
  const int64_t groups16 = (int64_t)B * ((H * W + 15) / 16);
  if (groups16 < 4096) return {4, D <= 32 ? 2 : 8};
  return {depth_per_pixel ? 6 : 5, 8};
}
static bool epi_path(int C, int H, int W, bool bwd) {
  (void)bwd;  // (both directions fit the widest group's layout)
  // the channel counts the epipolar kernels are instantiated for (C = 48, 80, ... take the
  // direct kernels: the dispatch below has no instance for them)
  return (C == 16 || C == 32 || C == 64 || C == 128) && epi_lds_bytes_wide(6, 8, C, H, W) <= 160 * 1024 &&
         epi_lds_bytes_wide(5, 8, C, H, W) <= 160 * 1024 &&
         (size_t)epi_bin_stride(H * W) * sizeof(uint32_t) <= 160 * 1024;  // grouping's LDS bin counters
}

// Small grids take the band kernel for the forward: one launch with no channel-last copies
// and no grouping pass. The epipolar path's set-up is fixed cost (3 launches) and one
// epipolar group per workgroup leaves a small grid's workgroups short of work (round 3: config A
// 16.4 -> 27.5 us, config B scale 0 25.6 -> 38.5 us when every shape took it). Large grids
// (config D's rig, diagonal epipolar lines whose row-segment boxes overflow kBandMax) keep
// the epipolar groups. DSPLAT_CV_PATH=band / epi overrides the choice (A/B timing tools); the
// caller asks once per forward and hands the answer to both calls (the backward
// used to re-read the variable and could disagree with its forward).
constexpr long kBandMaxPixels = 32768;  // B * H * W
static bool band_ok(int C) { return C == 16 || C == 32 || C == 64 || C == 128; }


// The epipolar grouping passes (k_epi_init .. k_epi_rank) of B x J (reference, source view)
// pairs into groups [B J][HW] and geom [B J][12], scratch after geom.
static int epi_group(int B, int J, int H, int W, int D, int depth_per_pixel, const float* intr, const float* pose,
                     const float* depth, int* groups, float* geom, hipStream_t st, const HwcJob* hwc = nullptr,
                     int hwc_planes = 0) {
  const int HW = H * W, BJ = B * J, nbs = epi_bin_stride(HW), pg = (HW + 255) / 256;
  const EpiScratch sc = epi_scratch(geom + (size_t)BJ * 12, BJ, HW);
  k_epi_init<<<dim3((std::max(kEpiBuckets, nbs) + 255) / 256, BJ), 256, 0, st>>>(J, H, W, intr, pose, geom, sc);
  if (int e = dsplat::check_launch("k_epi_init")) return e;
  const int pb = (HW + kEpiPix - 1) / kEpiPix;
  const size_t lds_count = 3 * kEpiBuckets * sizeof(uint32_t), lds_bins = (size_t)nbs * sizeof(uint32_t);
  DSPLAT_REQUIRE(lds_bins <= 160 * 1024, "cost volume: %d pixels exceed the grouping's LDS bin counters", HW);
  if (int e = dsplat::ensure_dyn_lds((const void*)(hwc ? k_epi_count<true> : k_epi_count<false>), lds_count,
                                     "hipFuncSetAttribute(k_epi_count)"))
    return e;
  if (int e = dsplat::ensure_dyn_lds((const void*)k_epi_bin, lds_bins, "hipFuncSetAttribute(k_epi_bin)")) return e;
  if (int e = dsplat::ensure_dyn_lds((const void*)k_epi_scatter, lds_bins, "hipFuncSetAttribute(k_epi_scatter)"))
    return e;
  // the channel-last copy tiles: the first half with the counting pass, the rest with the rank pass
  const int ntiles = hwc ? hwc4_blocks(*hwc, hwc_planes) : 0, t1 = ntiles / 2;
  if (hwc)
    k_epi_count<true><<<(unsigned)(pb * BJ + (t1 + 3) / 4), 1024, lds_count, st>>>(H, W, D, depth_per_pixel, depth,
                                                                                    geom, J, sc, pb, BJ, *hwc, t1);
  else
    k_epi_count<false><<<dim3(pb, BJ), 1024, lds_count, st>>>(H, W, D, depth_per_pixel, depth, geom, J, sc, pb, BJ,
                                                              HwcJob{}, 0);
  if (int e = dsplat::check_launch("k_epi_count")) return e;
  k_epi_segs<<<BJ, 1024, 0, st>>>(sc);
  if (int e = dsplat::check_launch("k_epi_segs")) return e;
  k_epi_bin<<<dim3(pb, BJ), 1024, lds_bins, st>>>(HW, sc);
  if (int e = dsplat::check_launch("k_epi_bin")) return e;
  k_epi_binscan<<<BJ, 1024, 0, st>>>(HW, sc);
  if (int e = dsplat::check_launch("k_epi_binscan")) return e;
  k_epi_scatter<<<dim3(pb, BJ), 1024, lds_bins, st>>>(HW, sc);
  if (int e = dsplat::check_launch("k_epi_scatter")) return e;
  if (hwc) {  // the channel-last copies as extra workgroups of the last grouping launch
    const unsigned nblk = (unsigned)pg * BJ + (unsigned)(ntiles - t1);
    k_epi_rank_hwc<<<nblk, 256, 0, st>>>(HW, sc, groups, pg, BJ, *hwc, t1);
    return dsplat::check_launch("k_epi_rank_hwc");
  }
  k_epi_rank<<<dim3(pg, BJ), 256, 0, st>>>(HW, sc, groups);
  return dsplat::check_launch("k_epi_rank");
}

// Channel-last copies (+ the epipolar groups when the epipolar kernels run): the forward's
// set-up on the epipolar / generic paths, and the backward's when the forward took the band
// kernel (which needs none of it).
static int epi_setup(int B, int J, int C, int H, int W, int D, int depth_per_pixel, const float* ref, const float* tgt,
                     const float* intr, const float* pose, const float* depth, void* workspace, hipStream_t st) {
  const int HW = H * W;
  float* tgt_hwc = static_cast<float*>(workspace);
  float* ref_hwc = tgt_hwc + (size_t)B * J * (HW + 1) * C;
  int* groups = reinterpret_cast<int*>(ref_hwc + (size_t)B * (HW + 1) * C);
  float* geom = reinterpret_cast<float*>(groups + (size_t)B * J * HW);
  // a band pixel's C channels are one contiguous row for the GEMM's operands; row HW of each
  // image is zero (the padding / out-of-image row)
  const bool v4 = C % 4 == 0 && HW % 4 == 0 && aligned16(tgt) && aligned16(ref) && aligned16(workspace);
  const bool epi = epi_path(C, H, W, false);
  if (v4) {  // tgt (and, for the epipolar kernels, ref) in one launch
    const HwcJob jb{C, HW, HW + 1, B * J, tgt, tgt_hwc, ref, ref_hwc};
    if (epi)  // the copies ride along the grouping's last launch (k_epi_rank_hwc)
      return epi_group(B, J, H, W, D, depth_per_pixel, intr, pose, depth, groups, geom, st, &jb, B * J + B);
    k_to_hwc4<<<dim3((HW + 63) / 64, (C + 63) / 64, B * J), 256, 0, st>>>(jb);
    if (int e = dsplat::check_launch("k_to_hwc4")) return e;
  } else {
    k_to_hwc<<<dim3((HW + 63) / 64, (C + 63) / 64, B * J), 256, 0, st>>>(C, HW, HW + 1, tgt, tgt_hwc);
    if (int e = dsplat::check_launch("k_to_hwc")) return e;
    if (epi) {
      k_to_hwc<<<dim3((HW + 63) / 64, (C + 63) / 64, B), 256, 0, st>>>(C, HW, HW + 1, ref, ref_hwc);
      if (int e = dsplat::check_launch("k_to_hwc(ref)")) return e;
    }
  }
  if (!epi) return 0;
  return epi_group(B, J, H, W, D, depth_per_pixel, intr, pose, depth, groups, geom, st);
}

// The epipolar forward launches (one per source view, in view order). tmap: views mode.
static int epi_fwd_launch(int B, int J, int C, int H, int W, int D, int depth_per_pixel, const float* ref_hwc,
                          const float* tgt_hwc, const int* tmap, const int* groups, const float* geom,
                          const float* depth, float clamp_min_depth, float* cost, hipStream_t st) {
  const int HW = H * W;
  const float scale = 1.0f / (sqrtf((float)C) * (float)J);
  const BwdShape fs = fwd_shape(D);
  const size_t lds = epi_lds_bytes_wide(fs.pxb, fs.spt, C, H, W);
  const int ngw = (HW + (1 << fs.pxb) - 1) >> fs.pxb, chunk = (256 >> fs.pxb) * fs.spt;
  const dim3 grid(8u * (unsigned)((B * ngw + 7) / 8), (unsigned)((D + chunk - 1) / chunk));
  // one instance per (C, samples per thread)
  auto kern = [&](auto nk) -> const void* {
    constexpr int NK = decltype(nk)::value;
    return fs.spt == 2 ? (const void*)k_cost_epi<NK, 2, 4> : (const void*)k_cost_epi<NK, 8, 4>;
  };
  const void* f = C == 16 ? kern(std::integral_constant<int, 4>{})
                : C == 32 ? kern(std::integral_constant<int, 8>{})
                : C == 64 ? kern(std::integral_constant<int, 16>{})
                          : kern(std::integral_constant<int, 32>{});
  if (int e = dsplat::ensure_dyn_lds(f, lds, "hipFuncSetAttribute(k_cost_epi)")) return e;
  for (int j = 0; j < J; ++j) {  // views in order: the sum over views is deterministic
    int a_B = B, a_j = j, a_J = J, a_H = H, a_W = W, a_D = D, a_dpp = depth_per_pixel, a_acc = j > 0;
    float a_clamp = clamp_min_depth, a_scale = scale;
    void* args[] = {&a_B, &a_j, &a_J, &a_H, &a_W, &a_D, &a_dpp, &a_acc, (void*)&ref_hwc, (void*)&tgt_hwc,
                    (void*)&tmap, (void*)&groups, (void*)&geom, (void*)&depth, &a_clamp, &a_scale, (void*)&cost};
    if (int e = dsplat::check_hip(hipLaunchKernel(f, grid, dim3(256), args, lds, st), "k_cost_epi")) return e;
  }
  return 0;
}

// The epipolar backward launches: |dcost|, |ref| maxima, then one launch per source view.
// fanin: an upper bound on the (b, j) pairs whose gradient lands on one target image (1: own
// copies; views mode: how often a view is a neighbour). Returns the dtgt unit's lgps via *lgps.
static int epi_bwd_launch(int B, int J, int C, int H, int W, int D, int depth_per_pixel, int fanin,
                          const float* ref_for_max, const float* ref_hwc, const float* tgt_hwc, const int* tmap,
                          const int* groups, const float* geom, const float* depth, float clamp_min_depth,
                          const float* dcost, float* cvmax, float* dref_hwc, long long* dtgt_fx, int* lgps_out,
                          hipStream_t st) {
  const int HW = H * W;
  const float scale = 1.0f / (sqrtf((float)C) * (float)J);
  k_cv_absmax<<<kCvMaxBlocks, 1024, 0, st>>>((size_t)B * D * HW, dcost, (size_t)B * C * HW, ref_for_max, cvmax);
  if (int e = dsplat::check_launch("k_cv_absmax")) return e;
  const BwdShape bs = bwd_shape(B, H, W, D, depth_per_pixel);
  const size_t lds = epi_lds_bytes_wide(bs.pxb, bs.spt, C, H, W);
  const int ngw = (HW + (1 << bs.pxb) - 1) >> bs.pxb;
  const dim3 grid(8u * (unsigned)((B * ngw + 7) / 8));
  // dtgt unit (cv_dtgt_unit): 2^lgS bounds a partial over |dcost| scale |ref|, 2^lgP the partials
  // per element (one per workgroup of the image and depth chunk, times the fan-in)
  const int chunk = (256 >> bs.pxb) * bs.spt;
  const long long nparts = (long long)ngw * ((D + chunk - 1) / chunk) * std::max(fanin, 1);
  int lgp = 0;
  while ((1ll << lgp) < nparts) ++lgp;
  const int lgps = 8 + (bs.spt == 8 ? 3 : 1) + lgp;
  *lgps_out = lgps;
  // one instance per (C, width, samples per thread)
  auto kern = [&](auto nk) -> const void* {
    constexpr int NK = decltype(nk)::value;
    if (bs.pxb == 6) return (const void*)k_cost_epi_bwd<NK, 6, 8>;
    if (bs.pxb == 5) return (const void*)k_cost_epi_bwd<NK, 5, 8>;
    return bs.spt == 2 ? (const void*)k_cost_epi_bwd<NK, 4, 2> : (const void*)k_cost_epi_bwd<NK, 4, 8>;
  };
  const void* f = C == 16 ? kern(std::integral_constant<int, 4>{})
                : C == 32 ? kern(std::integral_constant<int, 8>{})
                : C == 64 ? kern(std::integral_constant<int, 16>{})
                          : kern(std::integral_constant<int, 32>{});
  if (int e = dsplat::ensure_dyn_lds(f, lds, "hipFuncSetAttribute(k_cost_epi_bwd)")) return e;
  for (int j = 0; j < J; ++j) {
    int a_j = j, a_acc = j > 0;
    int a_B = B, a_J = J, a_H = H, a_W = W, a_D = D, a_dpp = depth_per_pixel;
    float a_clamp = clamp_min_depth, a_scale = scale;
    int a_lgps = lgps;
    void* args[] = {&a_B, &a_j, &a_J, &a_H, &a_W, &a_D, &a_dpp, &a_acc, (void*)&ref_hwc, (void*)&tgt_hwc,
                    (void*)&tmap, (void*)&groups, (void*)&geom, (void*)&depth, &a_clamp, &a_scale, (void*)&dcost,
                    (void*)&cvmax, &a_lgps, (void*)&dref_hwc, (void*)&dtgt_fx};
    if (int e = dsplat::check_hip(hipLaunchKernel(f, grid, dim3(256), args, lds, st), "k_cost_epi_bwd")) return e;
  }
  return 0;
}

int dcv_cost_volume_path(int B, int J, int C, int H, int W) {
  if (B <= 0 || J <= 0 || C <= 0 || H <= 1 || W <= 1) return -1;
  if (const char* f = getenv("DSPLAT_CV_PATH")) {
    if (!strcmp(f, "band") && band_ok(C)) return DCV_PATH_BAND;
    if (!strcmp(f, "epi") && epi_path(C, H, W, false)) return DCV_PATH_EPI;
  }
  if (band_ok(C) && (long)B * H * W <= kBandMaxPixels) return DCV_PATH_BAND;
  return epi_path(C, H, W, false) ? DCV_PATH_EPI : DCV_PATH_DIRECT;
}

int dcv_cost_volume_bwd_shape(int B, int C, int H, int W, int D, int depth_per_pixel, int* pxb, int* spt) {
  DSPLAT_REQUIRE(B > 0 && C > 0 && H > 1 && W > 1 && D > 0 && pxb && spt, "dcv_cost_volume_bwd_shape: bad arguments");
  DSPLAT_REQUIRE(epi_path(C, H, W, true), "dcv_cost_volume_bwd_shape: C=%d H=%d W=%d has no matrix-core backward", C,
                 H, W);
  const BwdShape bs = bwd_shape(B, H, W, D, depth_per_pixel);
  *pxb = bs.pxb;
  *spt = bs.spt;
  return 0;
}

static bool path_ok(int path, int C, int H, int W) {
  return path == DCV_PATH_DIRECT || (path == DCV_PATH_BAND && band_ok(C)) ||
         (path == DCV_PATH_EPI && epi_path(C, H, W, false));
}

int dcv_cost_volume_fwd(int B, int J, int C, int H, int W, int D, int depth_per_pixel, int path, const float* ref,
                        const float* tgt, const float* intr, const float* pose, const float* depth,
                        float clamp_min_depth, void* workspace, float* cost, void* stream) {
  DSPLAT_REQUIRE(B > 0 && J > 0 && C > 0 && H > 1 && W > 1 && D > 0, "dcv_cost_volume_fwd: bad sizes B=%d J=%d C=%d H=%d W=%d D=%d", B, J, C, H, W, D);
  DSPLAT_REQUIRE(ref && tgt && intr && pose && depth && workspace && cost, "dcv_cost_volume_fwd: null pointer");
  DSPLAT_REQUIRE(path_ok(path, C, H, W), "dcv_cost_volume_fwd: path %d not available for C=%d H=%d W=%d", path, C, H, W);
  hipStream_t st = (hipStream_t)stream;
  const int HW = H * W;
  if (path == DCV_PATH_BAND) {
    const size_t lds = cost_band_lds_bytes();
#define DCV_BAND(NK)                                                                                              \
  do {                                                                                                            \
    if (int e = dsplat::ensure_dyn_lds((const void*)k_cost_band<NK>, lds, "hipFuncSetAttribute(k_cost_band)"))    \
      return e;                                                                                                   \
    k_cost_band<NK><<<grid, 256, lds, st>>>(J, H, W, D, depth_per_pixel, ref, tgt, intr, pose, depth,            \
                                            clamp_min_depth, cost);                                               \
  } while (0)
    const dim3 grid((unsigned)(((W + BTP - 1) / BTP) * H), (unsigned)B, (unsigned)((D + BDCH - 1) / BDCH));
    switch (C) {
      case 16: DCV_BAND(4); break;
      case 32: DCV_BAND(8); break;
      case 64: DCV_BAND(16); break;
      default: DCV_BAND(32); break;
    }
#undef DCV_BAND
    return dsplat::check_launch("k_cost_band");
  }
  if (int e = epi_setup(B, J, C, H, W, D, depth_per_pixel, ref, tgt, intr, pose, depth, workspace, st)) return e;
  float* tgt_hwc = static_cast<float*>(workspace);
  float* ref_hwc = tgt_hwc + (size_t)B * J * (HW + 1) * C;
  int* groups = reinterpret_cast<int*>(ref_hwc + (size_t)B * (HW + 1) * C);
  float* geom = reinterpret_cast<float*>(groups + (size_t)B * J * HW);
  if (path == DCV_PATH_EPI)
    return epi_fwd_launch(B, J, C, H, W, D, depth_per_pixel, ref_hwc, tgt_hwc, nullptr, groups, geom, depth,
                          clamp_min_depth, cost, st);
  k_cost_fwd<<<dim3((HW + 3) / 4, B), 256, 0, st>>>(J, C, H, W, D, depth_per_pixel, ref, tgt_hwc, intr, pose,
                                                   depth, clamp_min_depth, cost);
  return dsplat::check_launch("k_cost_fwd");
}

int dcv_cost_volume_bwd(int B, int J, int C, int H, int W, int D, int depth_per_pixel, int fwd_path, const float* ref,
                        const float* tgt, void* workspace, const float* intr, const float* pose, const float* depth,
                        float clamp_min_depth, const float* dcost, float* dref, float* dtgt, void* bwd_workspace,
                        void* stream) {
  DSPLAT_REQUIRE(B > 0 && J > 0 && C > 0 && H > 1 && W > 1 && D > 0, "dcv_cost_volume_bwd: bad sizes");
  DSPLAT_REQUIRE(ref && tgt && workspace && intr && pose && depth && dcost && dref && dtgt && bwd_workspace,
                 "dcv_cost_volume_bwd: null pointer");
  DSPLAT_REQUIRE(path_ok(fwd_path, C, H, W), "dcv_cost_volume_bwd: forward path %d not available for C=%d H=%d W=%d",
                 fwd_path, C, H, W);
  hipStream_t st = (hipStream_t)stream;
  const int HW = H * W;
  // the band forward skipped the channel-last copies and the grouping: done here
  if (fwd_path == DCV_PATH_BAND)
    if (int e = epi_setup(B, J, C, H, W, D, depth_per_pixel, ref, tgt, intr, pose, depth, workspace, st)) return e;
  const float* tgt_hwc = static_cast<const float*>(workspace);
  const float* ref_hwc = tgt_hwc + (size_t)B * J * (HW + 1) * C;
  const int* groups = reinterpret_cast<const int*>(ref_hwc + (size_t)B * (HW + 1) * C);
  const float* geom = reinterpret_cast<const float*>(groups + (size_t)B * J * HW);
  const size_t ntg = (size_t)B * J * (HW + 1) * C;
  long long* dtgt_fx = static_cast<long long*>(bwd_workspace);
  float* dref_hwc = reinterpret_cast<float*>(dtgt_fx + ntg);
  float* cvmax = dref_hwc + (size_t)B * HW * C;
  const bool epi = epi_path(C, H, W, true) && epi_path(C, H, W, false);
  if (int e = dsplat::zero_async(dtgt_fx, ntg * (epi ? sizeof(long long) : sizeof(float)), st, "zero dtgt")) return e;
  if (epi) {
    int lgps = 0;
    if (int e = epi_bwd_launch(B, J, C, H, W, D, depth_per_pixel, 1, ref, ref_hwc, tgt_hwc, nullptr, groups, geom,
                               depth, clamp_min_depth, dcost, cvmax, dref_hwc, dtgt_fx, &lgps, st))
      return e;
    (C % 4 == 0 && HW % 4 == 0 && aligned16(dref) && aligned16(bwd_workspace) ? k_to_chw4 : k_to_chw)<<<
        dim3((HW + 63) / 64, (C + 63) / 64, B), 256, 0, st>>>(C, HW, HW, dref_hwc, dref);
    if (int e = dsplat::check_launch("k_to_chw(dref)")) return e;
    const float scale = 1.0f / (sqrtf((float)C) * (float)J);
    return fx_to_chw(B * J, C, HW, dtgt_fx, cvmax, scale, lgps, nullptr, dtgt, st);
  }
  float* dtgt_hwc = reinterpret_cast<float*>(dtgt_fx);
  k_cost_bwd<<<dim3((HW + 3) / 4, B), 256, 0, st>>>(J, C, H, W, D, depth_per_pixel, ref, tgt_hwc, intr, pose,
                                                   depth, clamp_min_depth, dcost, dref, dtgt_hwc);
  if (int e = dsplat::check_launch("k_cost_bwd")) return e;
  (C % 4 == 0 && HW % 4 == 0 && aligned16(dtgt) && aligned16(bwd_workspace) ? k_to_chw4 : k_to_chw)<<<
      dim3((HW + 63) / 64, (C + 63) / 64, B * J), 256, 0, st>>>(C, HW, HW + 1, dtgt_hwc, dtgt);
  return dsplat::check_launch("k_to_chw");
}

// ---- views mode (round 6) -----------------------------------------------------------------
// The reference stacks each view's neighbours' features into tgt [BV, J, C, H, W]
// (batch_features_camera_parameters, mv_transformer.py:653-747: a gather that copies every
// feature map J more times) and differentiates back through that gather. Here the features are
// read once: ONE channel-last copy [BV][HW + 1][C] serves as the reference tile of view b and as
// the target band rows of every (b, j) whose neighbour it is (nn[b J + j]); in the backward the
// target gradients accumulate straight into the neighbour view's int64 rows (order-independent)
// and one conversion adds the reference gradient: dfeatures in one pass.
// workspace: fhwc [BV][HW + 1][C] | groups [BV][J][HW] | geom [BV][J][12] | grouping scratch
size_t dcv_cost_volume_views_workspace_size(int BV, int J, int C, int H, int W) {
  if (BV <= 0 || J <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
  const size_t rows = (size_t)H * W + 1;
  return ((size_t)BV * rows * C + (size_t)BV * J * 12) * sizeof(float) + (size_t)BV * J * H * W * sizeof(int32_t) +
         epi_scratch_words(BV * J, H * W) * sizeof(uint32_t);
}
// backward workspace: dfeat_fx [BV][HW + 1][C] int64 | dref_hwc [BV][HW][C] | maxima
size_t dcv_cost_volume_views_bwd_workspace_size(int BV, int J, int C, int H, int W) {
  if (BV <= 0 || J <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
  return (size_t)BV * ((size_t)H * W + 1) * C * sizeof(long long) + (size_t)BV * H * W * C * sizeof(float) +
         2 * kCvMaxBlocks * sizeof(float);
}

int dcv_cost_volume_views_fwd(int BV, int J, int C, int H, int W, int D, int depth_per_pixel, const float* features,
                              const int32_t* nn, const float* intr, const float* pose, const float* depth,
                              float clamp_min_depth, void* workspace, float* cost, void* stream) {
  DSPLAT_REQUIRE(BV > 0 && J > 0 && C > 0 && H > 1 && W > 1 && D > 0,
                 "dcv_cost_volume_views_fwd: bad sizes BV=%d J=%d C=%d H=%d W=%d D=%d", BV, J, C, H, W, D);
  DSPLAT_REQUIRE(features && nn && intr && pose && depth && workspace && cost, "dcv_cost_volume_views_fwd: null pointer");
  DSPLAT_REQUIRE(epi_path(C, H, W, false), "dcv_cost_volume_views_fwd: C=%d H=%d W=%d needs the matrix-core path", C, H,
                 W);
  hipStream_t st = (hipStream_t)stream;
  const int HW = H * W;
  float* fhwc = static_cast<float*>(workspace);
  int* groups = reinterpret_cast<int*>(fhwc + (size_t)BV * (HW + 1) * C);
  float* geom = reinterpret_cast<float*>(groups + (size_t)BV * J * HW);
  if (C % 4 == 0 && HW % 4 == 0 && aligned16(features) && aligned16(workspace)) {
    const HwcJob jb{C, HW, HW + 1, BV, features, fhwc, nullptr, nullptr};
    if (int e = epi_group(BV, J, H, W, D, depth_per_pixel, intr, pose, depth, groups, geom, st, &jb, BV)) return e;
  } else {
    k_to_hwc<<<dim3((HW + 63) / 64, (C + 63) / 64, BV), 256, 0, st>>>(C, HW, HW + 1, features, fhwc);
    if (int e = dsplat::check_launch("k_to_hwc(features)")) return e;
    if (int e = epi_group(BV, J, H, W, D, depth_per_pixel, intr, pose, depth, groups, geom, st)) return e;
  }
  return epi_fwd_launch(BV, J, C, H, W, D, depth_per_pixel, fhwc, fhwc, nn, groups, geom, depth, clamp_min_depth, cost,
                        st);
}

int dcv_cost_volume_views_bwd(int BV, int J, int C, int H, int W, int D, int depth_per_pixel, int max_fanin,
                              const float* features, const int32_t* nn, void* workspace, const float* intr,
                              const float* pose, const float* depth, float clamp_min_depth, const float* dcost,
                              float* dfeatures, void* bwd_workspace, void* stream) {
  DSPLAT_REQUIRE(BV > 0 && J > 0 && C > 0 && H > 1 && W > 1 && D > 0, "dcv_cost_volume_views_bwd: bad sizes");
  DSPLAT_REQUIRE(features && nn && workspace && intr && pose && depth && dcost && dfeatures && bwd_workspace,
                 "dcv_cost_volume_views_bwd: null pointer");
  DSPLAT_REQUIRE(epi_path(C, H, W, true), "dcv_cost_volume_views_bwd: C=%d H=%d W=%d needs the matrix-core path", C, H,
                 W);
  hipStream_t st = (hipStream_t)stream;
  const int HW = H * W;
  const float* fhwc = static_cast<const float*>(workspace);
  const int* groups = reinterpret_cast<const int*>(fhwc + (size_t)BV * (HW + 1) * C);
  const float* geom = reinterpret_cast<const float*>(groups + (size_t)BV * J * HW);
  const size_t nfx = (size_t)BV * (HW + 1) * C;
  long long* dfx = static_cast<long long*>(bwd_workspace);
  float* dref_hwc = reinterpret_cast<float*>(dfx + nfx);
  float* cvmax = dref_hwc + (size_t)BV * HW * C;
  if (int e = dsplat::zero_async(dfx, nfx * sizeof(long long), st, "zero dfeatures")) return e;
  // a view is the neighbour of at most BV J (b, j) pairs; the caller may know a smaller bound
  const int fanin = max_fanin > 0 ? std::min(max_fanin, BV * J) : BV * J;
  int lgps = 0;
  if (int e = epi_bwd_launch(BV, J, C, H, W, D, depth_per_pixel, fanin, features, fhwc, fhwc, nn, groups, geom, depth,
                             clamp_min_depth, dcost, cvmax, dref_hwc, dfx, &lgps, st))
    return e;
  const float scale = 1.0f / (sqrtf((float)C) * (float)J);
  return fx_to_chw(BV, C, HW, dfx, cvmax, scale, lgps, dref_hwc, dfeatures, st);
}

int dcv_warp_fwd(int B, int C, int H, int W, int D, const float* feature, const float* intr, const float* pose,
                 const float* depth, float clamp_min_depth, float* out, void* stream) {
  DSPLAT_REQUIRE(B > 0 && C > 0 && H > 1 && W > 1 && D > 0, "dcv_warp_fwd: bad sizes");
  DSPLAT_REQUIRE(feature && intr && pose && depth && out, "dcv_warp_fwd: null pointer");
  const int HW = H * W;
  k_warp<<<dim3((HW + 255) / 256, D, B), 256, 0, (hipStream_t)stream>>>(C, H, W, D, feature, intr, pose, depth,
                                                                        clamp_min_depth, out);
  return dsplat::check_launch("k_warp");
}

}  // extern "C"
