// Shared helpers for the libdsplat_hip.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/dsplat_hip.h"

namespace dsplat {

void set_error(const char* fmt, ...);

// Check the last launch / API status and convert it to the ABI status code.
inline int check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return 2;
  }
  return 0;
}
inline int check_launch(const char* what) { return check_hip(hipGetLastError(), what); }

#define DSPLAT_REQUIRE(cond, ...)       \
  do {                                  \
    if (!(cond)) {                      \
      ::dsplat::set_error(__VA_ARGS__); \
      return 1;                         \
    }                                   \
  } while (0)

constexpr int kWave = 64;

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Inclusive scan over one wave64.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(v, off, 64);
    if (lane >= off) v += t;
  }
  return v;
}

// Inclusive wave64 scans on the DPP network: row_shr 1/2/4/8 scan each 16-lane row, then
// row_bcast:15 / row_bcast:31 carry row totals into the rows above (GFX9-family DPP).
// Lanes a DPP step cannot source read 0, the identity of both + and unsigned max.
template <typename Op>
__device__ __forceinline__ uint32_t wave_incl_dpp(uint32_t v, Op op) {
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_add_dpp(uint32_t v) {
  return wave_incl_dpp(v, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ uint32_t wave_incl_max_dpp(uint32_t v) {
  return wave_incl_dpp(v, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
}

// Zero a buffer with a plain kernel rather than hipMemsetAsync: the fill must be an
// ordinary kernel node when callers capture the stream into a hipGraph (a captured
// small hipMemsetAsync was observed not to re-run on replays 2+, leaving stale counts).
__global__ void k_zero_u32(uint32_t* __restrict__ p, size_t n);
int zero_async(void* p, size_t bytes, hipStream_t st, const char* what);

// Opt kernel `fn` into `bytes` of dynamic LDS on the current device before its launch
// (hipFuncSetAttribute(MaxDynamicSharedMemorySize) is per device). Remembered per (kernel,
// device) under a mutex: safe from concurrent host threads driving different devices/streams.
int ensure_dyn_lds(const void* fn, size_t bytes, const char* what);

// Row-block staging through LDS: the rows of a [*, row] array owned by one block are one
// contiguous span, so it moves as 16-byte vectors (coalesced) and each thread then reads /
// writes its own row in LDS (odd row lengths are bank-conflict free). Per-thread rows of
// 9 / 27 / 37 floats accessed directly make every load instruction touch ~64 cache lines.
// The LDS side moves 16 B per lane too (ds_write_b128 / ds_read_b128: consecutive lanes,
// consecutive 16-B slots, no bank conflict; four scalar ds ops at a 16-B lane stride were a
// 4-way conflict each). `lds` must be 16-byte aligned. The loads go out in batches of
// kStageBatch per thread before any LDS store: a plain copy loop waits for every load before
// its store (one memory round trip per iteration: ~10 serial round trips for a block's
// 37-float head rows).
constexpr int kStageBatch = 8;
template <int NTH, int BATCH = kStageBatch>
__device__ __forceinline__ void stage_in(const float* __restrict__ src, size_t nfloat, float* lds) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(src);
  if ((addr & 15) == 0) {
    const size_t n4 = nfloat / 4;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* l4 = reinterpret_cast<float4*>(lds);
    for (size_t i0 = threadIdx.x; i0 < n4; i0 += (size_t)BATCH * NTH) {
      float4 v[BATCH];  // unconditional loads (clamped index) keep v in registers
#pragma unroll
      for (int k = 0; k < BATCH; ++k) v[k] = s4[min(i0 + (size_t)k * NTH, n4 - 1)];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const size_t i = i0 + (size_t)k * NTH;
        if (i < n4) l4[i] = v[k];
      }
    }
    for (size_t i = 4 * n4 + threadIdx.x; i < nfloat; i += NTH) lds[i] = src[i];
  } else {
    for (size_t i0 = threadIdx.x; i0 < nfloat; i0 += (size_t)BATCH * NTH) {
      float v[BATCH];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) v[k] = src[min(i0 + (size_t)k * NTH, nfloat - 1)];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const size_t i = i0 + (size_t)k * NTH;
        if (i < nfloat) lds[i] = v[k];
      }
    }
  }
}
template <int NTH>
__device__ __forceinline__ void stage_out(float* __restrict__ dst, size_t nfloat, const float* lds) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(dst);
  if ((addr & 15) == 0) {
    const size_t n4 = nfloat / 4;
    float4* d4 = reinterpret_cast<float4*>(dst);
    const float4* l4 = reinterpret_cast<const float4*>(lds);
    for (size_t i = threadIdx.x; i < n4; i += NTH) d4[i] = l4[i];
    for (size_t i = 4 * n4 + threadIdx.x; i < nfloat; i += NTH) dst[i] = lds[i];
  } else {
    for (size_t i = threadIdx.x; i < nfloat; i += NTH) dst[i] = lds[i];
  }
}

// Register prefetch of a workgroup's contiguous row block (nfloat floats, 16-byte aligned src):
// P float4 per thread, issued together, so several row blocks of one workgroup are in flight
// at once (stage_in waits for each block before the next one is requested); pref_put lands
// them in LDS for the row transpose (the tail past the last float4 is read directly).
// P >= ceil(width / 4) covers NTH rows of `width` floats.
template <int NTH, int P>
__device__ __forceinline__ void pref_get(const float* src, size_t nfloat, float4 (&v)[P]) {
  const size_t n4 = nfloat / 4;
  const float4* s4 = reinterpret_cast<const float4*>(src);
#pragma unroll
  for (int k = 0; k < P; ++k)
    v[k] = n4 ? s4[min((size_t)threadIdx.x + (size_t)k * NTH, n4 - 1)] : make_float4(0.f, 0.f, 0.f, 0.f);
}
template <int NTH, int P>
__device__ __forceinline__ void pref_put(const float* src, size_t nfloat, const float4 (&v)[P], float* lds) {
  const size_t n4 = nfloat / 4;
  float4* l4 = reinterpret_cast<float4*>(lds);
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const size_t i = (size_t)threadIdx.x + (size_t)k * NTH;
    if (i < n4) l4[i] = v[k];
  }
  for (size_t i = 4 * n4 + threadIdx.x; i < nfloat; i += NTH) lds[i] = src[i];
}
__device__ __forceinline__ bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

inline int tiles_x(int W) { return (W + DSR_TILE - 1) / DSR_TILE; }
inline int tiles_y(int H) { return (H + DSR_TILE - 1) / DSR_TILE; }

}  // namespace dsplat
