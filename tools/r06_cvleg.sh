#!/bin/bash
# Cost-volume bench leg (configs A / B / D) and its rocprofv3 kernel stats.
# usage: bash tools/r06_cvleg.sh TAG
set -u
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --skip-headline --no-cpu-baseline --extra costvol --detail="
timeout -k 10 300 $B > gpurun_out/cvleg_$tag.log 2>&1 || { echo "leg failed"; tail -5 gpurun_out/cvleg_$tag.log; exit 1; }
python3 - gpurun_out/cvleg_$tag.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
for k, v in d["cost_volume"].items():
    if isinstance(v, dict):
        print(f"{k:32s} fwd {v['ms_per_call']:.4f} ms  fwd+bwd {v['ms_fwd_bwd']:.4f} ms  frac {v['frac']}")
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cvleg_${tag}_stats -o run -- $B \
  > gpurun_out/cvleg_${tag}_stats.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/kstats.py $(find gpurun_out/cvleg_${tag}_stats -name '*kernel_stats.csv' | head -1) 30
