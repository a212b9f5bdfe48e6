"""Build the phase-timing variant of k_cost_epi (forward) for tools/cv_epi_timing.py (GPU
box): a patched copy of dcv_cost_volume.hip that records, per workgroup, s_memrealtime
(100 MHz) at start, after the reference tile load, after the band set-up (epi_front), after
the first pass's GEMM, after its gather, and at the end, plus U and HW_ID, into 8 uint32 words
after the cost volume (the caller enlarges the output). The product source is not changed.
usage: python tools/cv_epi_timing_build.py  ->  lib/variants/libdsplat_cvt.so"""
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from my_depthsplat_amd import _build  # noqa: E402

src = (_build.CSRC / "dcv_cost_volume.hip").read_text()
k0 = src.index("__global__ __launch_bounds__(256, 4) void k_cost_epi(")
k1 = src.index("// Backward, view j", k0)
body = src[k0:k1]


def sub(old, new):
    global body
    assert body.count(old) == 1, old
    body = body.replace(old, new)


T = "__builtin_amdgcn_s_memrealtime()"
sub("  const EpiLds L = epi_lds(cv_lds, C, epi_words(H, W), false);\n",
    f"  const EpiLds L = epi_lds(cv_lds, C, epi_words(H, W), false);\n  uint64_t cvt[6]; cvt[0] = {T};\n")
sub("  const int pix = s_gid[i];  // -1: past the last pixel\n",
    f"  __syncthreads(); cvt[1] = {T};\n  const int pix = s_gid[i];  // -1: past the last pixel\n")
sub("  float* cb = cost + (size_t)b * D * HW;  // this scene's cost volume (< 2^32 elements)\n",
    f"  cvt[2] = {T}; cvt[3] = 0; cvt[4] = 0;\n  float* cb = cost + (size_t)b * D * HW;  // this scene's cost volume (< 2^32 elements)\n")
sub("    __syncthreads();\n    if (r0 == 0 && accumulate) load_prev();",
    f"    __syncthreads();\n    if (r0 == 0) cvt[3] = {T};\n    if (r0 == 0 && accumulate) load_prev();")
sub("    __syncthreads();  // list / corr reused by the next pass\n",
    f"    __syncthreads();  // list / corr reused by the next pass\n    if (r0 == 0) cvt[4] = {T};\n")
sub("  if (pix < 0) return;\n",
    "  __syncthreads();\n"
    f"  cvt[5] = {T};\n"
    "  if (tid == 0) {\n"
    "    uint32_t hw;\n"
    "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\" : \"=s\"(hw));\n"
    "    uint32_t* rec = reinterpret_cast<uint32_t*>(cost + (size_t)B * D * HW) + ((size_t)b * ngroups + g) * 8;\n"
    "    for (int q = 0; q < 6; ++q) rec[q] = (uint32_t)cvt[q];\n"
    "    rec[6] = (uint32_t)U; rec[7] = hw;\n"
    "  }\n"
    "  if (pix < 0) return;\n")
patched = src[:k0] + body + src[k1:]
out = _build.PKG / "lib" / "variants"
d = out / "cvt"
d.mkdir(parents=True, exist_ok=True)
with tempfile.TemporaryDirectory() as td:
    p = Path(td) / "dcv_cost_volume.hip"
    p.write_text(patched)
    objs = []
    for s in _build._sources():
        o = d / (s.stem + ".o")
        f = p if s.name == "dcv_cost_volume.hip" else s
        subprocess.run([_build.HIPCC, *_build.CFLAGS, *_build.FILE_FLAGS.get(s.name, []), "-I", str(_build.CSRC), "-c",
                        str(f), "-o", str(o)], check=True)
        objs.append(str(o))
so = out / "libdsplat_cvt.so"
subprocess.run([_build.HIPCC, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", str(so), *objs], check=True)
print(so)
