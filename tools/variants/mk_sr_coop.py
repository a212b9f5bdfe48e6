"""Variant sr_coop of dsr_raster.hip (verdict r4 item 1): k_sort_render's 4 waves test each
list entry against all 4 sub-tiles ONCE (one thread per entry, windows of 256 entries, the
waves' live boxes published in LDS) instead of every wave testing every entry; each wave then
stages only the entries whose bit it got. Writes tools/variants/sr_coop/dsr_raster.hip.
usage: python tools/variants/mk_sr_coop.py && python tools/ab_build.py sr_coop=tools/variants/sr_coop/dsr_raster.hip"""
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
src = (ROOT / "my_depthsplat_amd/csrc/dsr_raster.hip").read_text()

coop = r'''
// sr_coop: the tile's list composited in windows of NT entries. Per window, thread t tests
// entry wb + t against the 4 waves' live boxes (published in s_live) and writes the 4-bit
// reach mask over the key's depth word (the sort is done); then each wave stages and
// composites, in list order, only the entries of its bit. Two barriers per window; the
// waves are coupled at window ends (a dead wave keeps testing for the others).
template <bool LAST, int KMAX>
__device__ __forceinline__ void composite_coop(uint64_t* A, uint32_t n, uint32_t gmax, const float* __restrict__ gv,
                                               float fx0, float fy0, const PixUV2& pp, int lane, int w, uint64_t lt,
                                               WaveList* plist, float4* s_live, float& Tr, f2v& C01, float& C2,
                                               uint32_t& last, bool& alive) {
  Tr = alive ? Tr : -Tr;
  const int tid = threadIdx.x;
  for (uint32_t wb = 0; wb < n; wb += NT) {
    {
      const uint64_t live = __ballot(Tr > 0.f);
      float lx0 = 1.f, ly0 = 1.f, lx1 = 0.f, ly1 = 0.f;  // empty box
      if (live) live_rect(live, fx0, fy0, lx0, ly0, lx1, ly1);
      if (lane == 0) s_live[w] = make_float4(lx0, ly0, lx1, ly1);
    }
    __syncthreads();
    const uint32_t i = wb + (uint32_t)tid;
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f), r = q;
    float bcol = 0.f;
    if (i < n) {
      const uint32_t id = min((uint32_t)A[padi<KMAX>(i)], gmax);
      const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)id * GS);
      q = rec[0];
      r = rec[1];
      bcol = rec[2].x;
      uint32_t m = 0u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 b = s_live[k];
        if (b.x <= b.z && rect_hit(q, r, b.x, b.y, b.z, b.w)) m |= 1u << k;
      }
      A[padi<KMAX>(i)] = ((uint64_t)m << 32) | id;
    }
    __syncthreads();
    if (__any(Tr > 0.f)) {
      for (int c = 0; c < NT / 64; ++c) {
        const uint32_t base = wb + (uint32_t)(64 * c);
        if (base >= n) break;
        const uint32_t e = base + (uint32_t)lane;
        const uint64_t kk = e < n ? A[padi<KMAX>(e)] : 0ull;
        const bool mine = ((kk >> (32 + w)) & 1ull) != 0ull;
        const uint64_t bal = __ballot(mine);
        if (!bal) continue;
        float4 cq = q, cr = r;
        float cb = bcol;
        if (c != w && mine) {  // this wave's own chunk is in registers; the others from L1
          const float4* rec = reinterpret_cast<const float4*>(gv + (size_t)(uint32_t)kk * GS);
          cq = rec[0];
          cr = rec[1];
          cb = rec[2].x;
        }
        bool indef = false;
        if (mine) {
          const float4 sq = scaled_conic_q(cq);
          const float C = -0.5f * kLog2e * cr.x;
          indef = !conic_pd(sq.z, sq.w, C);
          pair_put(plist, __popcll(bal & lt), sq.x, sq.y, sq.z, C, sq.w, cr.y, cr.z, cr.w, cb, e + 1u, fx0, fy0);
        }
        const int cnt = __popcll(bal);
        if (lane < 8) pair_pad(plist, cnt + lane);
        __builtin_amdgcn_wave_barrier();
        const PairRec* pl = plist->rec;
        int lastk = -1;
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
        __builtin_amdgcn_wave_barrier();
        if (!__any(Tr > 0.f)) break;
      }
    }
    if (!__syncthreads_or(Tr > 0.f)) break;
  }
  alive = Tr > 0.f;
  Tr = fabsf(Tr);
}

template <int KMAX, bool LAST, int NBL, int WPE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) void k_sort_render('''
anchor = '''
template <int KMAX, bool LAST, int NBL, int WPE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) void k_sort_render('''
assert anchor in src
src = src.replace(anchor, coop, 1)
old = '''  if (in_lds)
    composite_tile<LAST>([&](uint32_t i) { return min((uint32_t)A[padi<KMAX>(i)], gmax); }, 0u, n, gv, (float)sx0,
                         (float)sy0, pp, lane, lt, plist, Tr, C01, C2, last, alive);'''
new = '''  __shared__ float4 s_live[4];
  if (in_lds)
    composite_coop<LAST, KMAX>(A, n, gmax, gv, (float)sx0, (float)sy0, pp, lane, w, lt, plist, s_live, Tr, C01, C2,
                               last, alive);'''
assert old in src
src = src.replace(old, new)
# write_keys: the sorted keys must go back before the masks overwrite their depth words
out = ROOT / "tools/variants/sr_coop/dsr_raster.hip"
out.parent.mkdir(parents=True, exist_ok=True)
out.write_text(src)
print(out)
