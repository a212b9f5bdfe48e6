"""Per-kernel register / LDS / occupancy table of one HIP source (hipcc -Rpass-analysis).

usage: python tools/kres.py [path/to/file.hip] [name-filter]"""
import re
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from my_depthsplat_amd import _build  # noqa: E402

src = Path(sys.argv[1] if len(sys.argv) > 1 else _build.CSRC / "dsr_raster.hip")
filt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run([_build.HIPCC, *_build.CFLAGS, *_build.FILE_FLAGS.get(src.name, []), "-I", str(_build.CSRC), "-c",
                    str(src), "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s+(.*?):\s+(.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for d in rows:
    if filt in d["name"]:
        n = re.sub(r"\(anonymous namespace\)::", "", d["name"]).split("(")[0]
        print(f"{n:60s} vgpr {d.get('VGPRs','?'):>4} sgpr {d.get('TotalSGPRs','?'):>4} occ {d.get('Occupancy [waves/SIMD]','?'):>2}"
              f" lds {d.get('LDS Size [bytes/block]','?'):>6} scratch {d.get('ScratchSize [bytes/lane]','?'):>4}"
              f" vspill {d.get('VGPRs Spill','?')}")
