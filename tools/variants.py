"""Build variants of libdsplat_hip.so with extra -D flags (kernel tuning experiments).

usage: python tools/variants.py NAME="-DFOO=1 -DBAR" [NAME2="..."] ...
Output: my_depthsplat_amd/lib/variants/libdsplat_NAME.so (travels to the GPU box).
"""
import shlex
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from my_depthsplat_amd import _build  # noqa: E402

OUT = _build.PKG / "lib" / "variants"


def build(name, flags):
    d = OUT / name
    d.mkdir(parents=True, exist_ok=True)
    objs = []
    for s in _build._sources():
        o = d / (s.stem + ".o")
        r = subprocess.run([_build.HIPCC, *_build.CFLAGS, *_build.FILE_FLAGS.get(s.name, []), *flags, "-c", str(s), "-o", str(o)], capture_output=True,
                           text=True)
        if r.returncode:
            raise RuntimeError(f"{name}: {s.name}\n{r.stderr}")
        objs.append(str(o))
    so = OUT / f"libdsplat_{name}.so"
    subprocess.run([_build.HIPCC, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", str(so), *objs],
                   check=True)
    return so


if __name__ == "__main__":
    specs = [a.split("=", 1) for a in sys.argv[1:]]
    with ThreadPoolExecutor(8) as ex:
        for so in ex.map(lambda nf: build(nf[0], shlex.split(nf[1])), specs):
            print(so)
