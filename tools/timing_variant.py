"""Build my_depthsplat_amd/lib/variants/libdsplat_timing.so: the library with k_sort_render
instrumented (experiment only; the product sources are not touched). Per (tile, wave) it
writes 8 uint64 into the scratch buffer: s_memrealtime at workgroup start, after the sort and
at the end, the tile's entry count, and s_memtime cycles spent per chunk in the filter (record
wait + rect test + list build) and in the compositing loop, chunks walked, entries composited.
Read back by tools/sr_timing.py.  usage: python tools/timing_variant.py"""
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from my_depthsplat_amd import _build  # noqa: E402

PATCHES = [
    ("// One chunk of the walk: keep the entries",
     "__shared__ uint64_t s_prof[4][4];\n// One chunk of the walk: keep the entries"),
    ("  const uint32_t e = base + lane;\n  const bool mine = e < end && rect_hit(q, r, lx0, ly0, lx1, ly1);",
     "  const uint64_t pt0 = __builtin_amdgcn_s_memtime();\n"
     "  const uint32_t e = base + lane;\n  const bool mine = e < end && rect_hit(q, r, lx0, ly0, lx1, ly1);"),
    ("  const PairRec* pp = plist;\n  PairRec a0",
     "  const uint64_t pt1 = __builtin_amdgcn_s_memtime();\n  const PairRec* pp = plist;\n  PairRec a0"),
    ("  __builtin_amdgcn_wave_barrier();  // list reads of this chunk before the next chunk's writes\n}",
     "  __builtin_amdgcn_wave_barrier();  // list reads of this chunk before the next chunk's writes\n"
     "  const uint64_t pt2 = __builtin_amdgcn_s_memtime();\n"
     "  if (lane == 0) { const int w = threadIdx.x >> 6; s_prof[w][0] += pt1 - pt0; s_prof[w][1] += pt2 - pt1;"
     " s_prof[w][2] += 1; s_prof[w][3] += cnt; }\n}"),
    ("  uint32_t b, e;\n  seg_bounds(seg_start, seg_count, stride, seg, b, e);\n  const uint32_t n = e - b;\n"
     "  const bool in_lds",
     "  const uint64_t t_0 = __builtin_amdgcn_s_memrealtime();\n"
     "  if (lane == 0) { s_prof[w][0] = 0; s_prof[w][1] = 0; s_prof[w][2] = 0; s_prof[w][3] = 0; }\n"
     "  uint32_t b, e;\n  seg_bounds(seg_start, seg_count, stride, seg, b, e);\n  const uint32_t n = e - b;\n"
     "  const bool in_lds"),
    ("  const bool inside = px < W && py < H;\n  const float* gv = geom + (size_t)v * G * GS;\n"
     "  const uint64_t lt = dsplat::lanemask_lt(lane);\n  PairRec* plist = reinterpret_cast<PairRec*>(aux)",
     "  const bool inside = px < W && py < H;\n  const float* gv = geom + (size_t)v * G * GS;\n"
     "  const uint64_t lt = dsplat::lanemask_lt(lane);\n  const uint64_t t_1 = __builtin_amdgcn_s_memrealtime();\n"
     "  PairRec* plist = reinterpret_cast<PairRec*>(aux)"),
    ("  if (clear_counts && tid == 0) seg_count[seg] = 0u;",
     "  if (clear_counts && tid == 0) seg_count[seg] = 0u;\n"
     "  const uint64_t t_2 = __builtin_amdgcn_s_memrealtime();\n"
     "  if (lane == 0) { uint64_t* o = scratch + ((size_t)seg * 4 + w) * 8; o[0] = t_0; o[1] = t_1; o[2] = t_2;"
     " o[3] = n | ((uint64_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) << 32); o[4] = s_prof[w][0];"
     " o[5] = s_prof[w][1]; o[6] = s_prof[w][2] | ((uint64_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);"
     " o[7] = s_prof[w][3]; }"),
]


def main():
    out = _build.PKG / "lib" / "variants" / "libdsplat_timing.so"
    with tempfile.TemporaryDirectory() as td:
        d = Path(td) / "pkg" / "csrc"  # same relative layout as the tree (../../include)
        d.mkdir(parents=True)
        shutil.copytree(_build.ROOT / "include", Path(td) / "include")
        for f in list(_build.CSRC.glob("*.hip")) + list(_build.CSRC.glob("*.h")):
            shutil.copy(f, d / f.name)
        src = (d / "dsr_raster.hip").read_text()
        for old, new in PATCHES:
            assert src.count(old) == 1, f"patch anchor not unique / missing: {old[:60]!r}"
            src = src.replace(old, new)
        (d / "dsr_raster.hip").write_text(src)
        objs = []
        for s in sorted(d.glob("*.hip")):
            o = d / (s.stem + ".o")
            r = subprocess.run([_build.HIPCC, *_build.CFLAGS, *_build.FILE_FLAGS.get(s.name, []), "-c", str(s), "-o", str(o)],
                               capture_output=True, text=True)
            if r.returncode:
                raise SystemExit(r.stderr)
            objs.append(str(o))
        subprocess.run([_build.HIPCC, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", str(out), *objs],
                       check=True)
    print(out)


if __name__ == "__main__":
    main()
