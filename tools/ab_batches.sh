#!/bin/bash
# Headline with different calibration batch sets, same box: usage bash tools/ab_batches.sh TAG STEPS SET...
# (SET = comma list for DSPLAT_BENCH_BATCHES)
set -u
TAG=${1:?tag}; K=${2:?steps}; shift 2
mkdir -p gpurun_out
out=gpurun_out/abb_${TAG}.log; : > $out
for s in "$@"; do
  DSPLAT_BENCH_BATCHES=$s timeout -k 10 300 python -u bench.py --steps $K --warmup 5 --extra "" --no-cpu-baseline \
    --no-reference-binning > gpurun_out/abb_${TAG}_${s//,/_}.log 2>&1 || { echo "$s failed"; exit 1; }
  python - "$s" gpurun_out/abb_${TAG}_${s//,/_}.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)
        print(sys.argv[1], 'value', d['value'], 'mode', d['launch_mode'], 'B', d['config']['global_batch'],
              {k: v for k, v in d['launch_calibration_ms_per_step'].items() if k.startswith(('b16', 'b32'))})
PY
done
cat $out
