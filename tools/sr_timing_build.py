"""Build the phase-timing variant of k_sort_render for tools/sr_timing.py (GPU box): a
patched copy of dsr_raster.hip recording per (tile, wave) s_memrealtime at workgroup start,
after the sort and after the wave's compositing, the tile's entry count, HW_ID and XCC_ID
into `scratch` (8 uint64 per (tile, wave)); the product source carries no instrumentation.
usage: python tools/sr_timing_build.py; python tools/sr_timing.py srt [H W V]"""
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from my_depthsplat_amd import _build  # noqa: E402

src = (_build.CSRC / "dsr_raster.hip").read_text()
k0 = src.index("void k_sort_render(")
k1 = src.index("// Sums of 4 entries x 9 gradient values", k0)
body = src[k0:k1]


def sub(old, new):
    global body
    assert body.count(old) == 1, old
    body = body.replace(old, new)


sub("  const bool in_lds = n <= cap;  // uniform\n",
    "  const bool in_lds = n <= cap;  // uniform\n  const uint64_t srt0 = __builtin_amdgcn_s_memrealtime();\n")
sub("  const int sx0 = tx * BX + (w & 1) * SUB, sy0 = ty * BY + (w >> 1) * SUB;\n",
    "  const uint64_t srt1 = __builtin_amdgcn_s_memrealtime();\n"
    "  const int sx0 = tx * BX + (w & 1) * SUB, sy0 = ty * BY + (w >> 1) * SUB;\n")
sub("  if (inside) store_pixel(out, finalT, ncontrib, cams[v].bg, v, H, W, px, py, Tr, C01, C2, last);\n",
    "  if (inside) store_pixel(out, finalT, ncontrib, cams[v].bg, v, H, W, px, py, Tr, C01, C2, last);\n"
    "  const uint64_t srt2 = __builtin_amdgcn_s_memrealtime();\n"
    "  if (lane == 0) {\n"
    "    uint32_t hw, xcc;\n"
    "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\" : \"=s\"(hw));\n"
    "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\" : \"=s\"(xcc));\n"
    "    uint64_t* rec = scratch + ((size_t)seg * 4 + w) * 8;\n"
    "    rec[0] = srt0; rec[1] = srt1; rec[2] = srt2; rec[3] = (uint64_t)n | ((uint64_t)hw << 32);\n"
    "    rec[4] = 0; rec[5] = 0; rec[6] = (uint64_t)xcc << 32; rec[7] = 0;\n"
    "  }\n")
patched = src[:k0] + body + src[k1:]
out = _build.PKG / "lib" / "variants"
d = out / "srt"
d.mkdir(parents=True, exist_ok=True)
with tempfile.TemporaryDirectory() as td:
    p = Path(td) / "dsr_raster.hip"
    p.write_text(patched)
    objs = []
    for s in _build._sources():
        o = d / (s.stem + ".o")
        f = p if s.name == "dsr_raster.hip" else s
        subprocess.run([_build.HIPCC, *_build.CFLAGS, *_build.FILE_FLAGS.get(s.name, []), "-I", str(_build.CSRC), "-c",
                        str(f), "-o", str(o)], check=True)
        objs.append(str(o))
so = out / "libdsplat_srt.so"
subprocess.run([_build.HIPCC, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", str(so), *objs], check=True)
print(so)
