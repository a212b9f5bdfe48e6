// dcv_cost_volume.hip — fused plane-sweep warp + correlation for gfx950 (wave64).
//
// Replaces, in one pass and without materialising the [B, C, D, H, W] warped tensor,
//   warp_with_pose_depth_candidates   src/model/encoder/unimatch/matching.py:24-90
//   cost = mean_j(sum_c ref * warped_j) / sqrt(C)   src/model/encoder/unimatch/mv_unimatch.py:494-505
//
// Layout: target features are first copied channel-last ([B,J,H,W,C]) so every bilinear
// tap is one contiguous C-float row; a wave owns one reference pixel with its 64 lanes
// over channels (coalesced 256-B tap reads), accumulates the per-depth partial dot
// products of 64 depth hypotheses in registers and finishes them with a transpose
// reduction (63 shuffles for 64 outputs) instead of 64 full wave reductions.
// Geometry per (pixel, depth, view) is wave-uniform and follows the reference's
// operation order: p_rot = R K^-1 [x, y, 1]; X = p_rot * depth + t; x = K X;
// uv = x.xy / max(x.z, clamp); grid = 2 uv / (size - 1) - 1; grid_sample unnormalise
// ((g + 1) / 2) * (size - 1), bilinear, zeros padding (align_corners=True).

#include "dsplat_common.h"

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
__global__ __launch_bounds__(256) void k_to_hwc(int C, int HW, const float* __restrict__ src,
                                                float* __restrict__ dst) {
  __shared__ float tile[64][65];
  const int bj = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const float* s = src + (size_t)bj * C * HW;
  float* d = dst + (size_t)bj * C * HW;
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

__global__ __launch_bounds__(256) void k_to_chw(int C, int HW, const float* __restrict__ src,
                                                float* __restrict__ dst) {
  __shared__ float tile[64][65];
  const int bj = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const float* s = src + (size_t)bj * C * HW;
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
      const float* tg = tgt_hwc + ((size_t)b * J + j) * HW * C;
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

// ---- MFMA formulation ------------------------------------------------------------------
// The bilinear warp is linear, so cost(p, d) = sum_j sum_taps w * (ref[p] . tgt_j[q_tap]) / (sqrt C J):
// every (pixel, depth) only needs the correlation of its pixel with the <= 4 target pixels it
// taps. A workgroup takes TP = 16 consecutive reference pixels of a row; for each source view
// it finds the distinct target pixels all its (pixel, depth) samples tap (an LDS bitmap over
// the target image + a prefix of popcounts = a rank for every tapped pixel), computes the
// correlations [16 pixels x U tapped pixels] as an exact-f32 GEMM on the matrix cores
// (v_mfma_f32_16x16x4_f32, K = C channels, channel-last target rows as B), and finishes with
// the 4-tap bilinear gather from LDS. Small-baseline epipolar segments of neighbouring pixels
// overlap, so U is a few tens to a few hundred, far below 16 x D x 4 taps. Tiles whose U
// exceeds kUMax fall back to a direct dot product per tap.
constexpr int TP = 16;      // reference pixels per workgroup
constexpr int DCH = 128;    // depth hypotheses per pass
constexpr int kUMax = 512;  // tapped target pixels held in LDS per (tile, view)

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct CvLds {
  float* aref;   // [TP][C]
  float2* samp;  // [DCH][TP] sample position (ix, iy); ix = NaN: outside
  uint32_t* bm;  // [NW] tapped-pixel bitmap
  uint32_t* bmp; // [NW] exclusive popcount prefix
  int* list;     // [kUMax] tapped pixel ids in rank order
  float* corr;   // [TP][kUMax]
  float* acc;    // [DCH][TP] cost accumulated over views
  uint32_t* misc;
};

__device__ __forceinline__ int tap_rank(const CvLds& L, int q) {
  const uint32_t w = L.bm[q >> 5];
  return (int)(L.bmp[q >> 5] + __popc(w & ((1u << (q & 31)) - 1u)));
}

__global__ __launch_bounds__(256) void k_cost_mfma(int J, int C, int H, int W, int D, int depth_per_pixel,
                                                   const float* __restrict__ ref,
                                                   const float* __restrict__ tgt_hwc,
                                                   const float* __restrict__ intr, const float* __restrict__ pose,
                                                   const float* __restrict__ depth, float clampz,
                                                   float* __restrict__ cost) {
  extern __shared__ __attribute__((aligned(16))) float cv_lds[];
  const int HW = H * W, NW = (HW + 31) / 32;
  CvLds L;
  {
    float* p = cv_lds;
    L.aref = p;
    p += TP * C;
    L.samp = reinterpret_cast<float2*>(p);
    p += 2 * DCH * TP;
    L.acc = p;
    p += DCH * TP;
    L.corr = p;
    p += TP * kUMax;
    L.list = reinterpret_cast<int*>(p);
    p += kUMax;
    L.bm = reinterpret_cast<uint32_t*>(p);
    p += NW;
    L.bmp = reinterpret_cast<uint32_t*>(p);
    p += NW;
    L.misc = reinterpret_cast<uint32_t*>(p);
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int tpr = (W + TP - 1) / TP;
  const int y = blockIdx.x / tpr, x0 = (blockIdx.x % tpr) * TP;
  const int b = blockIdx.y;
  const float scale = 1.0f / (sqrtf((float)C) * (float)J);
  // reference tile as the A operand: aref[i][c]
  for (int k = tid; k < TP * C; k += 256) {
    const int i = k & (TP - 1), c = k >> 4;
    L.aref[i * C + c] = (x0 + i < W) ? ref[((size_t)b * C + c) * HW + (size_t)y * W + x0 + i] : 0.f;
  }
  for (int d0 = 0; d0 < D; d0 += DCH) {
    for (int k = tid; k < DCH * TP; k += 256) L.acc[k] = 0.f;
    for (int j = 0; j < J; ++j) {
      Cam cam;
      load_cam(intr + ((size_t)b * J + j) * 9, pose + ((size_t)b * J + j) * 16, cam);
      for (int w = tid; w < NW; w += 256) L.bm[w] = 0u;
      __syncthreads();
      // sample positions of every (pixel, depth) of the tile, taps marked in the bitmap
      for (int k = tid; k < DCH * TP; k += 256) {
        const int i = k & (TP - 1), dd = k >> 4, d = d0 + dd;
        float2 sp = make_float2(__int_as_float(0x7fc00000), 0.f);
        if (d < D && x0 + i < W) {
          const float px = (float)(x0 + i), py = (float)y;
          const float qx = cam.Kinv[0] * px + cam.Kinv[1] * py + cam.Kinv[2];
          const float qy = cam.Kinv[3] * px + cam.Kinv[4] * py + cam.Kinv[5];
          const float qz = cam.Kinv[6] * px + cam.Kinv[7] * py + cam.Kinv[8];
          const float prx = cam.R[0] * qx + cam.R[1] * qy + cam.R[2] * qz;
          const float pry = cam.R[3] * qx + cam.R[4] * qy + cam.R[5] * qz;
          const float prz = cam.R[6] * qx + cam.R[7] * qy + cam.R[8] * qz;
          const float dep = depth_per_pixel ? depth[((size_t)b * D + d) * HW + (size_t)y * W + x0 + i]
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
            sp = make_float2(ix, iy);
            const int tx0 = (int)floorf(ix), ty0 = (int)floorf(iy);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1);
              if (tx >= 0 && tx < W && ty >= 0 && ty < H) {
                const int q = ty * W + tx;
                atomicOr(&L.bm[q >> 5], 1u << (q & 31));
              }
            }
          }
        }
        L.samp[k] = sp;
      }
      __syncthreads();
      // exclusive prefix of the bitmap popcounts (thread t owns a contiguous run of words)
      {
        const int per = (NW + 255) / 256;
        const int w0 = tid * per, w1 = min(NW, w0 + per);
        uint32_t tot = 0;
        for (int w = w0; w < w1; ++w) tot += __popc(L.bm[w]);
        const uint32_t incl = dsplat::wave_incl_scan(tot, lane);
        if (lane == 63) L.misc[wv] = incl;
        __syncthreads();
        uint32_t off = incl - tot;
        for (int k = 0; k < wv; ++k) off += L.misc[k];
        for (int w = w0; w < w1; ++w) {
          L.bmp[w] = off;
          off += __popc(L.bm[w]);
        }
        if (tid == 255) L.misc[4] = off;
      }
      __syncthreads();
      const int U = (int)L.misc[4];
      if (U <= kUMax) {
        for (int w = tid; w < NW; w += 256) {
          uint32_t bits = L.bm[w];
          int r = (int)L.bmp[w];
          while (bits) {
            const int bpos = __builtin_ctz(bits);
            bits &= bits - 1u;
            L.list[r++] = w * 32 + bpos;
          }
        }
        __syncthreads();
        // corr[16 x U] = aref[16 x C] . tgt[U x C]^T on the matrix cores; per 16-channel step
        // lane l feeds channels cb + 4 (l >> 4) + s in MFMA s (A and B permuted alike)
        const float* tg = tgt_hwc + ((size_t)b * J + j) * (size_t)HW * C;
        const int nblk = (U + 15) / 16;
        for (int blk = wv; blk < nblk; blk += 4) {
          const int u = blk * 16 + (lane & 15);
          const int q = u < U ? L.list[u] : -1;
          f32x4 acc4 = {0.f, 0.f, 0.f, 0.f};
          const float* brow = tg + (size_t)(q < 0 ? 0 : q) * C + 4 * (lane >> 4);
          const float* arow = L.aref + (lane & 15) * C + 4 * (lane >> 4);
          for (int cb = 0; cb < C; cb += 16) {
            float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q >= 0) bv = *reinterpret_cast<const float4*>(brow + cb);
            const float4 av = *reinterpret_cast<const float4*>(arow + cb);
            acc4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc4, 0, 0, 0);
            acc4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc4, 0, 0, 0);
            acc4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc4, 0, 0, 0);
            acc4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc4, 0, 0, 0);
          }
          // D[row][col]: col = lane & 15 (tapped pixel), row = 4 (lane >> 4) + r (ref pixel)
#pragma unroll
          for (int r = 0; r < 4; ++r) L.corr[(4 * (lane >> 4) + r) * kUMax + u] = acc4[r];
        }
        __syncthreads();
        for (int k = tid; k < DCH * TP; k += 256) {
          const float2 sp = L.samp[k];
          if (!(sp.x == sp.x)) continue;
          const int i = k & (TP - 1);
          const float fx0 = floorf(sp.x), fy0 = floorf(sp.y);
          const int tx0 = (int)fx0, ty0 = (int)fy0;
          const float wx0 = (float)(tx0 + 1) - sp.x, wx1 = sp.x - fx0, wy0 = (float)(ty0 + 1) - sp.y,
                      wy1 = sp.y - fy0;
          const float wt[4] = {wx0 * wy0, wx1 * wy0, wx0 * wy1, wx1 * wy1};
          float s = 0.f;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1);
            if (tx >= 0 && tx < W && ty >= 0 && ty < H) s += wt[t] * L.corr[i * kUMax + tap_rank(L, ty * W + tx)];
          }
          L.acc[k] += s;
        }
      } else {
        // too many distinct taps for LDS: direct dot products (rare: very wide epipolar bands)
        const float* tg = tgt_hwc + ((size_t)b * J + j) * (size_t)HW * C;
        for (int k = tid; k < DCH * TP; k += 256) {
          const float2 sp = L.samp[k];
          if (!(sp.x == sp.x)) continue;
          const int i = k & (TP - 1);
          const float fx0 = floorf(sp.x), fy0 = floorf(sp.y);
          const int tx0 = (int)fx0, ty0 = (int)fy0;
          const float wx0 = (float)(tx0 + 1) - sp.x, wx1 = sp.x - fx0, wy0 = (float)(ty0 + 1) - sp.y,
                      wy1 = sp.y - fy0;
          const float wt[4] = {wx0 * wy0, wx1 * wy0, wx0 * wy1, wx1 * wy1};
          float s = 0.f;
          for (int t = 0; t < 4; ++t) {
            const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1);
            if (!(tx >= 0 && tx < W && ty >= 0 && ty < H)) continue;
            const float* row = tg + (size_t)(ty * W + tx) * C;
            float dot = 0.f;
            for (int c = 0; c < C; ++c) dot += L.aref[i * C + c] * row[c];
            s += wt[t] * dot;
          }
          L.acc[k] += s;
        }
      }
      __syncthreads();
    }
    for (int k = tid; k < DCH * TP; k += 256) {
      const int i = k & (TP - 1), d = d0 + (k >> 4);
      if (d < D && x0 + i < W) cost[((size_t)b * D + d) * HW + (size_t)y * W + x0 + i] = L.acc[k] * scale;
    }
    __syncthreads();
  }
}

// Backward with the same tiling. Per (tile, view): G[i][u] = sum over the tile's (pixel i,
// depth d) samples tapping target pixel list[u] of dcost(i, d) * w_tap / (sqrt C J) (LDS
// float atomics), then on the matrix cores
//   dref[i][c] += sum_u G[i][u] tgt[list[u]][c]      ([16 x U] x [U x C], K = U)
//   dtgt[list[u]][c] += sum_i G[i][u] ref[i][c]       ([U x 16] x [16 x C], K = 16; global atomics)
__global__ __launch_bounds__(256) void k_cost_mfma_bwd(int J, int C, int H, int W, int D, int depth_per_pixel,
                                                       const float* __restrict__ ref,
                                                       const float* __restrict__ tgt_hwc,
                                                       const float* __restrict__ intr,
                                                       const float* __restrict__ pose,
                                                       const float* __restrict__ depth, float clampz,
                                                       const float* __restrict__ dcost, float* __restrict__ dref,
                                                       float* __restrict__ dtgt_hwc) {
  extern __shared__ __attribute__((aligned(16))) float cv_lds[];
  const int HW = H * W, NW = (HW + 31) / 32;
  CvLds L;
  float* dacc;  // [TP][C] dref accumulated over views and depth chunks
  {
    float* p = cv_lds;
    L.aref = p;
    p += TP * C;
    L.samp = reinterpret_cast<float2*>(p);
    p += 2 * DCH * TP;
    L.acc = p;  // G: [TP][kUMax]
    p += TP * kUMax;
    dacc = p;
    p += TP * C;
    L.list = reinterpret_cast<int*>(p);
    p += kUMax;
    L.bm = reinterpret_cast<uint32_t*>(p);
    p += NW;
    L.bmp = reinterpret_cast<uint32_t*>(p);
    p += NW;
    L.misc = reinterpret_cast<uint32_t*>(p);
  }
  float* Gm = L.acc;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int tpr = (W + TP - 1) / TP;
  const int y = blockIdx.x / tpr, x0 = (blockIdx.x % tpr) * TP;
  const int b = blockIdx.y;
  const float scale = 1.0f / (sqrtf((float)C) * (float)J);
  for (int k = tid; k < TP * C; k += 256) {
    const int i = k & (TP - 1), c = k >> 4;
    L.aref[i * C + c] = (x0 + i < W) ? ref[((size_t)b * C + c) * HW + (size_t)y * W + x0 + i] : 0.f;
    dacc[i * C + c] = 0.f;
  }
  for (int d0 = 0; d0 < D; d0 += DCH) {
    for (int j = 0; j < J; ++j) {
      Cam cam;
      load_cam(intr + ((size_t)b * J + j) * 9, pose + ((size_t)b * J + j) * 16, cam);
      for (int w = tid; w < NW; w += 256) L.bm[w] = 0u;
      __syncthreads();
      for (int k = tid; k < DCH * TP; k += 256) {
        const int i = k & (TP - 1), dd = k >> 4, d = d0 + dd;
        float2 sp = make_float2(__int_as_float(0x7fc00000), 0.f);
        if (d < D && x0 + i < W) {
          const float px = (float)(x0 + i), py = (float)y;
          const float qx = cam.Kinv[0] * px + cam.Kinv[1] * py + cam.Kinv[2];
          const float qy = cam.Kinv[3] * px + cam.Kinv[4] * py + cam.Kinv[5];
          const float qz = cam.Kinv[6] * px + cam.Kinv[7] * py + cam.Kinv[8];
          const float prx = cam.R[0] * qx + cam.R[1] * qy + cam.R[2] * qz;
          const float pry = cam.R[3] * qx + cam.R[4] * qy + cam.R[5] * qz;
          const float prz = cam.R[6] * qx + cam.R[7] * qy + cam.R[8] * qz;
          const float dep = depth_per_pixel ? depth[((size_t)b * D + d) * HW + (size_t)y * W + x0 + i]
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
            sp = make_float2(ix, iy);
            const int tx0 = (int)floorf(ix), ty0 = (int)floorf(iy);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1);
              if (tx >= 0 && tx < W && ty >= 0 && ty < H) {
                const int q = ty * W + tx;
                atomicOr(&L.bm[q >> 5], 1u << (q & 31));
              }
            }
          }
        }
        L.samp[k] = sp;
      }
      __syncthreads();
      {
        const int per = (NW + 255) / 256;
        const int w0 = tid * per, w1 = min(NW, w0 + per);
        uint32_t tot = 0;
        for (int w = w0; w < w1; ++w) tot += __popc(L.bm[w]);
        const uint32_t incl = dsplat::wave_incl_scan(tot, lane);
        if (lane == 63) L.misc[wv] = incl;
        __syncthreads();
        uint32_t off = incl - tot;
        for (int k = 0; k < wv; ++k) off += L.misc[k];
        for (int w = w0; w < w1; ++w) {
          L.bmp[w] = off;
          off += __popc(L.bm[w]);
        }
        if (tid == 255) L.misc[4] = off;
      }
      __syncthreads();
      const int U = (int)L.misc[4];
      float* dtg = dtgt_hwc + ((size_t)b * J + j) * (size_t)HW * C;
      const float* tg = tgt_hwc + ((size_t)b * J + j) * (size_t)HW * C;
      if (U <= kUMax) {
        const int Up = (U + 15) & ~15;
        for (int w = tid; w < NW; w += 256) {
          uint32_t bits = L.bm[w];
          int r = (int)L.bmp[w];
          while (bits) {
            const int bpos = __builtin_ctz(bits);
            bits &= bits - 1u;
            L.list[r++] = w * 32 + bpos;
          }
        }
        for (int k = tid; k < TP * Up; k += 256) Gm[(k / Up) * kUMax + (k % Up)] = 0.f;
        __syncthreads();
        for (int k = tid; k < DCH * TP; k += 256) {
          const float2 sp = L.samp[k];
          if (!(sp.x == sp.x)) continue;
          const int i = k & (TP - 1), d = d0 + (k >> 4);
          const float g = dcost[((size_t)b * D + d) * HW + (size_t)y * W + x0 + i] * scale;
          const float fx0 = floorf(sp.x), fy0 = floorf(sp.y);
          const int tx0 = (int)fx0, ty0 = (int)fy0;
          const float wx0 = (float)(tx0 + 1) - sp.x, wx1 = sp.x - fx0, wy0 = (float)(ty0 + 1) - sp.y,
                      wy1 = sp.y - fy0;
          const float wt[4] = {wx0 * wy0, wx1 * wy0, wx0 * wy1, wx1 * wy1};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1);
            if (tx >= 0 && tx < W && ty >= 0 && ty < H) atomicAdd(&Gm[i * kUMax + tap_rank(L, ty * W + tx)], g * wt[t]);
          }
        }
        __syncthreads();
        // dref[16 x C] += G[16 x U] . T[U x C]: blocks of 16 channels, K = taps (4 per MFMA)
        for (int cb = wv * 16; cb < C; cb += 64) {
          f32x4 acc4 = {0.f, 0.f, 0.f, 0.f};
          for (int u0 = 0; u0 < Up; u0 += 4) {
            const int u = u0 + (lane >> 4);
            const float a = Gm[(lane & 15) * kUMax + u];
            const float bv = u < U ? tg[(size_t)L.list[u] * C + cb + (lane & 15)] : 0.f;
            acc4 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc4, 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) dacc[(4 * (lane >> 4) + r) * C + cb + (lane & 15)] += acc4[r];
        }
        // dtgt[U x C] += G^T[U x 16] . aref[16 x C]: blocks of 16 taps x 16 channels, K = pixels
        const int nub = Up / 16, ncb = C / 16;
        for (int blk = wv; blk < nub * ncb; blk += 4) {
          const int ub = (blk / ncb) * 16, cb = (blk % ncb) * 16;
          f32x4 acc4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) {
            const int i = 4 * s2 + (lane >> 4);
            const float a = Gm[i * kUMax + ub + (lane & 15)];
            const float bv = L.aref[i * C + cb + (lane & 15)];
            acc4 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc4, 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int u = ub + 4 * (lane >> 4) + r;
            if (u < U && acc4[r] != 0.f) atomicAdd(&dtg[(size_t)L.list[u] * C + cb + (lane & 15)], acc4[r]);
          }
        }
      } else {
        // direct scatter (very wide tap sets): per sample and tap, all channels
        for (int k = tid; k < DCH * TP; k += 256) {
          const float2 sp = L.samp[k];
          if (!(sp.x == sp.x)) continue;
          const int i = k & (TP - 1), d = d0 + (k >> 4);
          const float g = dcost[((size_t)b * D + d) * HW + (size_t)y * W + x0 + i] * scale;
          const float fx0 = floorf(sp.x), fy0 = floorf(sp.y);
          const int tx0 = (int)fx0, ty0 = (int)fy0;
          const float wx0 = (float)(tx0 + 1) - sp.x, wx1 = sp.x - fx0, wy0 = (float)(ty0 + 1) - sp.y,
                      wy1 = sp.y - fy0;
          const float wt[4] = {wx0 * wy0, wx1 * wy0, wx0 * wy1, wx1 * wy1};
          for (int t = 0; t < 4; ++t) {
            const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1);
            if (!(tx >= 0 && tx < W && ty >= 0 && ty < H)) continue;
            const float gw = g * wt[t];
            const size_t row = (size_t)(ty * W + tx) * C;
            for (int c = 0; c < C; ++c) {
              atomicAdd(&dacc[i * C + c], gw * tg[row + c]);
              atomicAdd(&dtg[row + c], gw * L.aref[i * C + c]);
            }
          }
        }
      }
      __syncthreads();
    }
  }
  for (int k = tid; k < TP * C; k += 256) {
    const int i = k & (TP - 1), c = k >> 4;
    if (x0 + i < W) dref[((size_t)b * C + c) * HW + (size_t)y * W + x0 + i] = dacc[i * C + c];
  }
}

// ---- forward on the matrix cores, band form (dcv_cost_volume_fwd) ----------------------
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

size_t cost_mfma_bwd_lds_bytes(int C, int HW) {
  const int NW = (HW + 31) / 32;
  return sizeof(float) * ((size_t)2 * TP * C + 2 * DCH * TP + TP * kUMax + kUMax + 2 * NW + 8);
}

size_t cost_mfma_lds_bytes(int C, int HW) {
  const int NW = (HW + 31) / 32;
  return sizeof(float) * ((size_t)TP * C + 2 * DCH * TP + DCH * TP + TP * kUMax + kUMax + 2 * NW + 8);
}

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
      const float* tg = tgt_hwc + ((size_t)b * J + j) * HW * C;
      float* dtg = dtgt_hwc + ((size_t)b * J + j) * HW * C;
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

int dcv_cost_volume_fwd(int B, int J, int C, int H, int W, int D, int depth_per_pixel, const float* ref,
                        const float* tgt, const float* intr, const float* pose, const float* depth,
                        float clamp_min_depth, float* tgt_hwc, float* cost, void* stream) {
  DSPLAT_REQUIRE(B > 0 && J > 0 && C > 0 && H > 1 && W > 1 && D > 0, "dcv_cost_volume_fwd: bad sizes B=%d J=%d C=%d H=%d W=%d D=%d", B, J, C, H, W, D);
  DSPLAT_REQUIRE(ref && tgt && intr && pose && depth && cost, "dcv_cost_volume_fwd: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int HW = H * W;
  // channel-last copy of the target features: only for the backward (when asked for) and the
  // generic-C paths below; the band kernel reads [B,J,C,H,W] directly
  const bool band = C == 16 || C == 32 || C == 64 || C == 128;
  if (tgt_hwc || !band) {
    DSPLAT_REQUIRE(tgt_hwc != nullptr, "dcv_cost_volume_fwd: C=%d needs the tgt_hwc workspace", C);
    k_to_hwc<<<dim3((HW + 63) / 64, (C + 63) / 64, B * J), 256, 0, st>>>(C, HW, tgt, tgt_hwc);
    if (int e = dsplat::check_launch("k_to_hwc")) return e;
  }
  if (band) {
    static bool attr = false;
    const size_t lds = cost_band_lds_bytes();
    if (!attr) {
#define DCV_ATTR(NK)                                                                                          \
  if (int e = dsplat::check_hip(hipFuncSetAttribute((const void*)k_cost_band<NK>,                             \
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), \
                                "hipFuncSetAttribute(k_cost_band)"))                                         \
    return e;
      DCV_ATTR(4) DCV_ATTR(8) DCV_ATTR(16) DCV_ATTR(32)
#undef DCV_ATTR
      attr = true;
    }
    const dim3 grid((unsigned)(((W + BTP - 1) / BTP) * H), (unsigned)B, (unsigned)((D + BDCH - 1) / BDCH));
#define DCV_BAND(NK)                                                                                             \
  k_cost_band<NK><<<grid, 256, lds, st>>>(J, H, W, D, depth_per_pixel, ref, tgt, intr, pose, depth, clamp_min_depth, \
                                          cost)
    switch (C) {
      case 16: DCV_BAND(4); break;
      case 32: DCV_BAND(8); break;
      case 64: DCV_BAND(16); break;
      default: DCV_BAND(32); break;
    }
#undef DCV_BAND
    return dsplat::check_launch("k_cost_band");
  }
  const size_t lds = cost_mfma_lds_bytes(C, HW);
  if (C % 16 == 0 && lds <= 160 * 1024) {  // matrix-core path over the exact tapped set
    static size_t attr = 0;
    if (lds > 64 * 1024 && lds > attr) {
      if (int e = dsplat::check_hip(hipFuncSetAttribute((const void*)k_cost_mfma,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                                    "hipFuncSetAttribute(k_cost_mfma)"))
        return e;
      attr = lds;
    }
    k_cost_mfma<<<dim3((unsigned)(((W + TP - 1) / TP) * H), B), 256, lds, st>>>(
        J, C, H, W, D, depth_per_pixel, ref, tgt_hwc, intr, pose, depth, clamp_min_depth, cost);
    return dsplat::check_launch("k_cost_mfma");
  }
  k_cost_fwd<<<dim3((HW + 3) / 4, B), 256, 0, st>>>(J, C, H, W, D, depth_per_pixel, ref, tgt_hwc, intr, pose,
                                                   depth, clamp_min_depth, cost);
  return dsplat::check_launch("k_cost_fwd");
}

int dcv_cost_volume_bwd(int B, int J, int C, int H, int W, int D, int depth_per_pixel, const float* ref,
                        const float* tgt_hwc, const float* intr, const float* pose, const float* depth,
                        float clamp_min_depth, const float* dcost, float* dref, float* dtgt, float* dtgt_hwc,
                        void* stream) {
  DSPLAT_REQUIRE(B > 0 && J > 0 && C > 0 && H > 1 && W > 1 && D > 0, "dcv_cost_volume_bwd: bad sizes");
  DSPLAT_REQUIRE(ref && tgt_hwc && intr && pose && depth && dcost && dref && dtgt && dtgt_hwc,
                 "dcv_cost_volume_bwd: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int HW = H * W;
  if (int e = dsplat::zero_async(dtgt_hwc, (size_t)B * J * HW * C * 4, st, "zero dtgt_hwc")) return e;
  const size_t lds = cost_mfma_bwd_lds_bytes(C, HW);
  if (C % 16 == 0 && lds <= 160 * 1024) {  // matrix-core path
    static size_t attr = 0;
    if (lds > 64 * 1024 && lds > attr) {
      if (int e = dsplat::check_hip(hipFuncSetAttribute((const void*)k_cost_mfma_bwd,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                                    "hipFuncSetAttribute(k_cost_mfma_bwd)"))
        return e;
      attr = lds;
    }
    k_cost_mfma_bwd<<<dim3((unsigned)(((W + TP - 1) / TP) * H), B), 256, lds, st>>>(
        J, C, H, W, D, depth_per_pixel, ref, tgt_hwc, intr, pose, depth, clamp_min_depth, dcost, dref, dtgt_hwc);
    if (int e = dsplat::check_launch("k_cost_mfma_bwd")) return e;
  } else {
    k_cost_bwd<<<dim3((HW + 3) / 4, B), 256, 0, st>>>(J, C, H, W, D, depth_per_pixel, ref, tgt_hwc, intr, pose,
                                                     depth, clamp_min_depth, dcost, dref, dtgt_hwc);
    if (int e = dsplat::check_launch("k_cost_bwd")) return e;
  }
  k_to_chw<<<dim3((HW + 63) / 64, (C + 63) / 64, B * J), 256, 0, st>>>(C, HW, dtgt_hwc, dtgt);
  return dsplat::check_launch("k_to_chw");
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
