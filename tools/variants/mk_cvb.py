"""Timing variants of k_cost_epi_bwd (dcv_cost_volume.hip), verdict r4 item 6: where the
deterministic backward's time goes. Writes tools/variants/cvb_<name>/dcv_cost_volume.hip:
  cvb_noatom  the dtgt int64 atomics skipped (wrong dtgt; timing only)
  cvb_f32     dtgt as float atomics into the same buffer (not deterministic; timing only)
  cvb_noglds  G accumulated as float LDS atomics, no fixed-point conversion (timing only)
usage: python tools/variants/mk_cvb.py && python tools/ab_build.py cvb_noatom=tools/variants/cvb_noatom/dcv_cost_volume.hip ..."""
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
src = (ROOT / "my_depthsplat_amd/csrc/dcv_cost_volume.hip").read_text()

ATOM = """              atomicAdd(reinterpret_cast<unsigned long long*>(&dtg[(size_t)q * C + cbk * 16 + (lane & 15)]),
                        (unsigned long long)v);"""
assert src.count(ATOM) == 1


def write(name, text):
    d = ROOT / "tools/variants" / name
    d.mkdir(parents=True, exist_ok=True)
    (d / "dcv_cost_volume.hip").write_text(text)
    print(d / "dcv_cost_volume.hip")


write("cvb_noatom", src.replace(ATOM, "              asm volatile(\"\" :: \"v\"(v));"))
write("cvb_f32", src.replace(ATOM, """              atomicAdd(reinterpret_cast<float*>(&dtg[(size_t)q * C + cbk * 16 + (lane & 15)]), acc[r]);"""))

G_ADD = [("atomicAdd(&grow[ra], (int)rintf(gu * (wx0 * wy0)))", "atomicAdd(&growf[ra], gu * (wx0 * wy0))"),
         ("atomicAdd(&grow[ra + 1], (int)rintf(gu * (wx1 * wy0)))", "atomicAdd(&growf[ra + 1], gu * (wx1 * wy0))"),
         ("atomicAdd(&grow[rb], (int)rintf(gu * (wx0 * wy1)))", "atomicAdd(&growf[rb], gu * (wx0 * wy1))"),
         ("atomicAdd(&grow[rb + 1], (int)rintf(gu * (wx1 * wy1)))", "atomicAdd(&growf[rb + 1], gu * (wx1 * wy1))"),
         ("int* grow = gi + i * kECorr;", "float* growf = reinterpret_cast<float*>(gi) + i * kECorr;"),
         ("av[t] = (float)gi[(lane & 15) * kECorr + u] * unit_g;",
          "av[t] = reinterpret_cast<const float*>(gi)[(lane & 15) * kECorr + u];"),
         ("acc = __builtin_amdgcn_mfma_f32_16x16x4f32((float)gi[p * kECorr + u] * unit_g,",
          "acc = __builtin_amdgcn_mfma_f32_16x16x4f32(reinterpret_cast<const float*>(gi)[p * kECorr + u],")]
t = src
for a, b in G_ADD:
    assert t.count(a) == 1, a
    t = t.replace(a, b)
t = t.replace("const float gu = gs[s] * unit_g_inv;", "const float gu = gs[s];")
write("cvb_noglds", t)
