"""Materialise an A/B variant kernel source from its patch.

Each tools/variants/NAME.patch is a unified diff of one csrc file against the commit named on
its "# base" line (the product source the variant was measured against). This writes the
patched file to tools/variants/_src/NAME/<file> (git-ignored) and prints the path, ready for
tools/ab_build.py:

    python tools/ab_build.py NAME=$(python tools/variants/apply.py NAME)

pb_pref and pb_uni were adopted into the product (their sources equal commit 047f52e), so
they have no patch."""
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
HERE = Path(__file__).resolve().parent


def materialise(name: str) -> Path:
    patch = HERE / f"{name}.patch"
    lines = patch.read_text().splitlines()
    rel = lines[0].split(" of ", 1)[1].strip()
    base = lines[1].split()[-1]
    src = subprocess.run(["git", "-C", str(ROOT), "show", f"{base}:{rel}"], check=True,
                         capture_output=True, text=True).stdout
    out = HERE / "_src" / name / Path(rel).name
    out.parent.mkdir(parents=True, exist_ok=True)
    with tempfile.NamedTemporaryFile("w", suffix=".hip", delete=False) as t:
        t.write(src)
    subprocess.run(["patch", "-s", "-o", str(out), t.name, str(patch)], check=True)
    Path(t.name).unlink()
    return out


if __name__ == "__main__":
    names = sys.argv[1:] or sorted(p.stem for p in HERE.glob("*.patch"))
    for n in names:
        print(materialise(n))
