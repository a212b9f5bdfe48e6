"""Variant sr_scan of dsr_raster.hip (verdict r4 item 5, north_star's "wavefront prefix-scan for
transmittance"): the compositor's chunk loop transposed — lanes over the chunk's staged entries,
one pixel of the wave's sub-tile at a time; each entry's alpha at that pixel, T before each
entry as the exclusive prefix SUM of log2(1 - alpha) over the lanes (DPP scan) and exp2, the
stop at the first entry whose T (1 - alpha) < 1e-4 (ballot), colour = wave sum of
alpha T rgb over the entries before it. Replaces the serial per-pixel walk of chunks whose conics
are all definite (the common loop); images agree to float rounding (log / exp2 instead of the
product chain), not bit for bit. Writes tools/variants/sr_scan/dsr_raster.hip."""
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
src = (ROOT / "my_depthsplat_amd/csrc/dsr_raster.hip").read_text()

helper = r'''
// sr_scan: exclusive wave prefix sum (DPP row shifts + row broadcasts, as wave_incl_add_dpp)
__device__ __forceinline__ float wave_excl_add_f(float v) {
  float x = v;
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x111, 0xf, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x112, 0xf, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x114, 0xf, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x118, 0xf, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x142, 0xa, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x143, 0xc, 0xf, false));
  return x - v;
}
__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
// one chunk, transposed: lane e holds staged entry e (e < cnt); pixels of the wave in turn
template <bool LAST>
__device__ __forceinline__ void composite_scan(const WaveList* plist, int cnt, float fx0, float fy0, int lane,
                                               float& Tr, f2v& C01, float& C2, int& lastk) {
  const PairRec& P = plist->rec[lane >> 1];
  const int j = lane & 1;
  const float F = P.F[j], D = P.D[j], E = P.E[j], A = P.A[j], Cc = P.C[j], Bb = P.B[j];
  const float r = P.rg[j].x, g = P.rg[j].y, b = P.b[j];
  const bool have = lane < cnt;
  uint64_t live = __ballot(Tr > 0.f);
  while (live) {
    const int px = __builtin_ctzll(live);
    live &= live - 1;
    const float T0 = __shfl(Tr, px, 64);
    // the pixel's offsets from the sub-tile centre (as pix_uv)
    const float u = (float)(px & 7) - 3.5f, v = (float)(px >> 3) - 3.5f;
    const float p2o = fmaf(A, u * u, fmaf(Cc, v * v, fmaf(Bb, u * v, fmaf(D, u, fmaf(E, v, F)))));
    float a = fminf(0.99f, __builtin_amdgcn_exp2f(p2o));
    a = (have && a >= 1.0f / 255.0f) ? a : 0.f;
    const float l = __builtin_amdgcn_logf(1.f - a);  // log2(1 - a)
    const float T = T0 * __builtin_amdgcn_exp2f(wave_excl_add_f(l));
    const bool stop = a > 0.f && T * (1.f - a) < 0.0001f;
    const uint64_t sm = __ballot(stop);
    const int first = sm ? __builtin_ctzll(sm) : 64;
    const float w = lane < first ? a * T : 0.f;
    const float cr = wave_sum_f(w * r), cg = wave_sum_f(w * g), cb = wave_sum_f(w * b);
    // T after the walk: the product up to the stop (or the whole chunk)
    const float Tend = __shfl(T * (1.f - a), first < 64 ? first : 63, 64);
    const float Tstop = __shfl(T, first < 64 ? first : 63, 64);
    if (lane == px) {
      C01.x += cr;
      C01.y += cg;
      C2 += cb;
      Tr = first < 64 ? -Tstop : (cnt > 0 ? Tend : T0);
      if (LAST) {
        const uint64_t bl = __ballot(w > 0.f);
        (void)bl;
      }
    }
  }
  (void)lastk;
}
'''
anchor = '''// One chunk of the walk: keep the entries of [base, base + CH)'''
assert anchor in src
src = src.replace(anchor, helper + '\n' + anchor)
old = '''  if (!__any(indef)) {
    for (int k = 0; k < cnt; k += 4) {
      const PairRec a0 = pl[k >> 1], a1 = pl[(k >> 1) + 1];
      composite_pair<LAST, true>(a0, pp, Tr, C01, C2, lastk, k);
      composite_pair<LAST, true>(a1, pp, Tr, C01, C2, lastk, k + 2);
      if (!__any(Tr > 0.f)) break;
    }
  } else {'''
new = '''  if (!LAST && !__any(indef)) {
    composite_scan<LAST>(plist, cnt, fx0, fy0, lane, Tr, C01, C2, lastk);
  } else if (!__any(indef)) {
    for (int k = 0; k < cnt; k += 4) {
      const PairRec a0 = pl[k >> 1], a1 = pl[(k >> 1) + 1];
      composite_pair<LAST, true>(a0, pp, Tr, C01, C2, lastk, k);
      composite_pair<LAST, true>(a1, pp, Tr, C01, C2, lastk, k + 2);
      if (!__any(Tr > 0.f)) break;
    }
  } else {'''
assert old in src
src = src.replace(old, new)
out = ROOT / "tools/variants/sr_scan/dsr_raster.hip"
out.parent.mkdir(parents=True, exist_ok=True)
out.write_text(src)
print(out)
