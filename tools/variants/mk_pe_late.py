"""Variant pe_late of dsr_raster.hip: k_project_emit evaluates the SH colour LAST, after the
geometry, the exact-binning ellipse terms and the key are formed and the record's first
16 bytes and the radius are stored, so fewer values are live across the 27-float SH row
(k_project_emit<2> 70 VGPRs, 7 waves per SIMD; the aim is <= 64 for 8 without a second memory
round trip). Records bit-identical. Writes tools/variants/pe_late/dsr_raster.hip."""
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
src = (ROOT / "my_depthsplat_amd/csrc/dsr_raster.hip").read_text()
# 1. a colour-only helper (same SH code as project_gauss's COLOR branch)
anchor = '''// dzero (optional): the backward's fixed-point gradient accumulator [V, G, DSR_DGEOM_WORDS];'''
helper = '''// The SH colour of one projected Gaussian (project_gauss's COLOR branch on its own): rgb into
// rec[6..8], clamp bits into rec[11].
template <int DEG>
__device__ __forceinline__ void project_color(const GaussIn<DEG>& in, const dsr_camera* __restrict__ cam, int M,
                                              const float* __restrict__ shs, const float* __restrict__ colors,
                                              int layout, float* rec) {
  uint32_t clamp_bits = 0;
  if constexpr (DEG >= 0) {
    const float gsc = cam->scale;
    const F3 p = {in.m[0] * gsc, in.m[1] * gsc, in.m[2] * gsc};
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
  rec[11] = __uint_as_float(clamp_bits);
}

'''
assert anchor in src
src = src.replace(anchor, helper + anchor)
old = '''  if (g < G) {
    float rec[GS];
    r = project_gauss<DEG>(in, cam, CAM ? s_focal : focal_of(cam, H, W), H, W, gx, gy, M, shs, colors, layout, rec,
                           x0, y0, x1, y1);
    store_geom(geom, radii, (size_t)v * G + g, rec, r, dzero);
    key = ((uint64_t)__float_as_uint(rec[9]) << 32) | (uint32_t)g;
    if constexpr (EXACT) {
      ell = tile_ell(rec, r);
      if (r > 0) tile_rect_alpha(ell, x0, y0, x1, y1);
    }
  }'''
new = '''  if (g < G) {
    float rec[GS];
    r = project_gauss<DEG, false>(in, cam, CAM ? s_focal : focal_of(cam, H, W), H, W, gx, gy, M, shs, colors, layout,
                                  rec, x0, y0, x1, y1);
    key = ((uint64_t)__float_as_uint(rec[9]) << 32) | (uint32_t)g;
    if constexpr (EXACT) {
      ell = tile_ell(rec, r);
      if (r > 0) tile_rect_alpha(ell, x0, y0, x1, y1);
    }
    const size_t vg = (size_t)v * G + g;
    float4* out = reinterpret_cast<float4*>(geom + vg * GS);
    out[0] = make_float4(rec[0], rec[1], rec[2], rec[3]);
    radii[vg] = r;
    if (r > 0) project_color<DEG>(in, cam, M, shs, colors, layout, rec);  // colour last: fewer live values
    out[1] = make_float4(rec[4], rec[5], rec[6], rec[7]);
    out[2] = make_float4(rec[8], rec[9], rec[10], rec[11]);
    if (dzero != nullptr && r > 0) {
      long long* z = dzero + vg * DSR_DGEOM_WORDS;
#pragma unroll
      for (int k = 0; k < DSR_DGEOM_WORDS; ++k) z[k] = 0ll;
    }
  }'''
assert old in src
src = src.replace(old, new)
out = ROOT / "tools/variants/pe_late/dsr_raster.hip"
out.parent.mkdir(parents=True, exist_ok=True)
out.write_text(src)
print(out)
