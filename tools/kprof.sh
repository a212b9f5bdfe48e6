#!/bin/bash
# Device-side kernel times of kbench runs, one rocprofv3 process per library variant
# (host launch overhead does not enter). usage: tools/kprof.sh KERNEL "KBENCH ARGS" VARIANT...
set -e
export TMPDIR=/tmp
kern=$1; shift
args=$1; shift
for v in "$@"; do
  d=gpurun_out/kprof_$v
  rm -rf $d
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python3 tools/kbench.py --kernel $kern $args $v > $d.log 2>&1
  python3 - "$d/run_kernel_stats.csv" "$v" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    m = re.search(r"(k_\w+(?:<[^>]*>)?)\(", r["Name"])
    if m and int(r["Calls"]) >= 50:
        out.append(f"{m.group(1)}={float(r['AverageNs']) / 1e3:.2f}us")
print(f"{sys.argv[2]:>10s}: " + "  ".join(out))
PY
done
