"""Build the phase-timing variant of k_project_emit for tools/pe_timing.py (GPU box):
a patched copy of dsr_raster.hip (s_memrealtime at workgroup start, after the projection,
after the count pass, after the range reservation and at the end; pairs per workgroup; HW_ID
and XCC_ID) compiled with the other sources into lib/variants/libdsplat_pet.so. The product
source carries no instrumentation. usage: python tools/pe_timing_build.py"""
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from my_depthsplat_amd import _build  # noqa: E402

src = (_build.CSRC / "dsr_raster.hip").read_text()
k0 = src.index("void k_project_emit(")
k1 = src.index("// Single-workgroup exclusive scan", k0)
body = src[k0:k1]


def sub(old, new, count=1):
    global body
    assert body.count(old) >= count, old
    body = body.replace(old, new, count)


TS = "  uint64_t pet_t[5]; uint32_t pet_pairs = 0;\n"
sub("  const dsr_camera* cam = cams + v;\n", "  const dsr_camera* cam = cams + v;\n" + TS +
    "  pet_t[0] = __builtin_amdgcn_s_memrealtime();\n")
sub("  s_key[tid] = key;\n  if (tid == 0) s_ovf = 0u;\n  __syncthreads();\n",
    "  s_key[tid] = key;\n  if (tid == 0) s_ovf = 0u;\n  __syncthreads();\n  pet_t[1] = __builtin_amdgcn_s_memrealtime();\n")
sub("  if (lane == 0 && wtotal > (uint32_t)kPairCapW) s_ovf = 1u;\n  __syncthreads();\n",
    "  if (lane == 0 && wtotal > (uint32_t)kPairCapW) s_ovf = 1u;\n  __syncthreads();\n"
    "  pet_t[2] = __builtin_amdgcn_s_memrealtime(); pet_pairs = wtotal;\n")
sub("  __syncthreads();\n  uint64_t* vkeys = keys + (size_t)v * T * G;\n",
    "  __syncthreads();\n  pet_t[3] = __builtin_amdgcn_s_memrealtime();\n  uint64_t* vkeys = keys + (size_t)v * T * G;\n")
REC = ("      __syncthreads();\n"
       "      pet_t[4] = __builtin_amdgcn_s_memrealtime();\n"
       "      if (tid == 0) {\n"
       "        uint32_t hw, xcc;\n"
       "        asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\" : \"=s\"(hw));\n"
       "        asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\" : \"=s\"(xcc));\n"
       "        const size_t nwg = gridDim.x;\n"
       "        uint64_t* rec = keys + (size_t)V * T * G - nwg * 8 + (size_t)blockIdx.x * 8;\n"
       "        for (int q = 0; q < 5; ++q) rec[q] = pet_t[q];\n"
       "        rec[5] = pet_pairs; rec[6] = hw; rec[7] = xcc;\n"
       "      }\n")
sub("      vkeys[(size_t)t * G + s_hist[t] + ((p >> 16) & 0xFFu)] = wkey[p >> 24];\n    }\n    return;\n",
    "      vkeys[(size_t)t * G + s_hist[t] + ((p >> 16) & 0xFFu)] = wkey[p >> 24];\n    }\n" + REC + "    return;\n")
patched = src[:k0] + body + src[k1:]
out = _build.PKG / "lib" / "variants"
d = out / "pet"
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
so = out / "libdsplat_pet.so"
subprocess.run([_build.HIPCC, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", str(so), *objs], check=True)
print(so)
