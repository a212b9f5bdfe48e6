"""Build the HIP extension libdsplat_hip.so in-tree (gfx950 only) and the CPU oracle.

Plain hipcc, no torch JIT cache: the .so lands in my_depthsplat_amd/lib/ so it travels
with the repository snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "lib" / "libdsplat_hip.so"
OBJ = PKG / "lib" / "obj"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -ffp-contract=off: the preprocess arithmetic must match the oracle bit for bit (sort keys,
# radii, tile rects). -munsafe-fp-atomics: native global_atomic_add_f32 (no CAS loop).
CFLAGS = [
    "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-ffp-contract=off",
    "-munsafe-fp-atomics", "-Wall", "-Wno-unused-function", "-I", str(ROOT / "include"),
]


# Per-file extra flags. The rasterizer's per-lane pixel math is scalar by design (its packed
# FP32 is written out with explicit vector types); the SLP vectorizer re-packs the scalar
# parts with register shuffles that cost more than they save (k_render_bwd 119 -> 109 us
# without it at config B).
FILE_FLAGS = {"dsr_raster.hip": ["-fno-slp-vectorize"]}


def _sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _needs(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_hip(force: bool = False, verbose: bool = False) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    headers = list(CSRC.glob("*.h")) + [ROOT / "include" / "dsplat_hip.h", Path(__file__)]
    srcs = _sources()
    jobs = []
    for s in srcs:
        o = OBJ / (s.stem + ".o")
        if force or _needs(o, [s] + headers):
            jobs.append((s, o))

    def compile_one(job):
        s, o = job
        cmd = [HIPCC, *CFLAGS, *FILE_FLAGS.get(s.name, []), "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {s.name}:\n{r.stderr}")
        return o

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(compile_one, jobs))
    objs = [OBJ / (s.stem + ".o") for s in srcs]
    if force or jobs or _needs(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc link failed:\n{r.stderr}")
    return LIB


def build_oracle() -> Path:
    r = subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"oracle build failed:\n{r.stdout}\n{r.stderr}")
    return ROOT / "oracle" / "build" / "libdsr_oracle.so"


if __name__ == "__main__":
    print(build_hip(force="--force" in sys.argv, verbose=True))
    print(build_oracle())
