"""Build A/B variants of libdsplat_hip.so from alternative copies of one source file.

usage: python tools/ab_build.py NAME=path/to/dsr_raster.hip [NAME2=...]
Each variant replaces the csrc file of the same name; output
my_depthsplat_amd/lib/variants/libdsplat_NAME.so (travels to the GPU box; select it with
DSPLAT_LIB=... for bench.py / tests)."""
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from my_depthsplat_amd import _build  # noqa: E402

OUT = _build.PKG / "lib" / "variants"


def build(name, alt):
    alt = Path(alt).resolve()
    d = OUT / name
    d.mkdir(parents=True, exist_ok=True)
    objs = []
    for s in _build._sources():
        src = alt if s.name == alt.name else s
        o = d / (s.stem + ".o")
        r = subprocess.run([_build.HIPCC, *_build.CFLAGS, *_build.FILE_FLAGS.get(s.name, []), "-I", str(_build.CSRC),
                            "-c", str(src), "-o", str(o)], capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f"{name}: {s.name}\n{r.stderr}")
        objs.append(str(o))
    so = OUT / f"libdsplat_{name}.so"
    subprocess.run([_build.HIPCC, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", str(so), *objs], check=True)
    return so


if __name__ == "__main__":
    specs = [a.split("=", 1) for a in sys.argv[1:]]
    with ThreadPoolExecutor(4) as ex:
        for so in ex.map(lambda nf: build(*nf), specs):
            print(so)
