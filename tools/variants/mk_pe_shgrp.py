"""Variant pe_shgrp of dsr_raster.hip: the projection's SH rows read in groups of 3
coefficients (9 floats), each group's channel FMAs done before the next group's loads are
issued, so at most 9 SH registers are live instead of 27 (k_project_emit<2> 70 VGPRs, 7 waves
per SIMD; the aim is <= 64 for 8). Same FMA order per channel (k ascending): records
bit-identical. Writes tools/variants/pe_shgrp/dsr_raster.hip."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
src = (ROOT / "my_depthsplat_amd/csrc/dsr_raster.hip").read_text()
GROUP = int(sys.argv[1]) if len(sys.argv) > 1 else 3
old = '''          float sh[GaussIn<DEG>::NC * 3];
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
          }'''
new = '''          constexpr int NC = GaussIn<DEG>::NC, KG = %d;
          float dx = p.x - cam->campos[0], dy = p.y - cam->campos[1], dz = p.z - cam->campos[2];
          const float len = sqrtf(fmaf(dx, dx, fmaf(dy, dy, dz * dz)));
          dx = dx / len;
          dy = dy / len;
          dz = dz / len;
          float acc[3] = {0.f, 0.f, 0.f};
          const float* shp = shs + in.sg * (size_t)M * 3;
#pragma unroll
          for (int k0 = 0; k0 < NC; k0 += KG) {
            float s[KG * 3];
#pragma unroll
            for (int q = 0; q < KG * 3; ++q) {
              const int k = k0 + q / 3, ch = q %% 3;
              s[q] = k < NC ? ((layout & kLayoutShChannelMajor) ? shp[ch * M + k] : shp[k * 3 + ch]) : 0.f;
            }
#pragma unroll
            for (int ch = 0; ch < 3; ++ch)
#pragma unroll
              for (int kk = 0; kk < KG; ++kk) {
                const int k = k0 + kk;
                if (k < NC) acc[ch] = sh_term<DEG>(k, s[kk * 3 + ch], acc[ch], dx, dy, dz);
              }
            asm volatile("" ::: "memory");  // the next group's loads after this group's FMAs
          }
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) {
            float c = acc[ch] + 0.5f;
            clamp_bits |= (c < 0.f ? 1u : 0u) << ch;
            rec[6 + ch] = fmaxf(c, 0.0f);
          }''' % GROUP
assert old in src
src = src.replace(old, new)
term = '''
// term k of sh_eval's per-channel chain: v = SH_C0 s(0), then v = fma(basis_k, s(k), v) in k order
template <int DEG>
__device__ __forceinline__ float sh_term(int k, float s, float v, float x, float y, float z) {
  const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
  switch (k) {
    case 0: return SH_C0 * s;
    case 1: return fmaf(-(SH_C1 * y), s, v);
    case 2: return fmaf(SH_C1 * z, s, v);
    case 3: return fmaf(-(SH_C1 * x), s, v);
    case 4: return fmaf(SH_C2_0 * xy, s, v);
    case 5: return fmaf(SH_C2_1 * yz, s, v);
    case 6: return fmaf(SH_C2_2 * (2.0f * zz - xx - yy), s, v);
    case 7: return fmaf(SH_C2_3 * xz, s, v);
    case 8: return fmaf(SH_C2_4 * (xx - yy), s, v);
    case 9: return fmaf(SH_C3_0 * y * (3.0f * xx - yy), s, v);
    case 10: return fmaf(SH_C3_1 * xy * z, s, v);
    case 11: return fmaf(SH_C3_2 * y * (4.0f * zz - xx - yy), s, v);
    case 12: return fmaf(SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy), s, v);
    case 13: return fmaf(SH_C3_4 * x * (4.0f * zz - xx - yy), s, v);
    case 14: return fmaf(SH_C3_5 * z * (xx - yy), s, v);
    default: return fmaf(SH_C3_6 * x * (xx - 3.0f * yy), s, v);
  }
}
'''
anchor = '''// Input layouts (dsr_preprocess_* `layout` bits).'''
assert anchor in src
src = src.replace(anchor, term + '\n' + anchor)
name = sys.argv[2] if len(sys.argv) > 2 else "pe_shgrp"
out = ROOT / f"tools/variants/{name}/dsr_raster.hip"
out.parent.mkdir(parents=True, exist_ok=True)
out.write_text(src)
print(out)
