#!/bin/bash
# Headline throughput at 16 scenes per launch pair with N captures replayed on N HIP streams.
# usage: bash tools/ab_lanes.sh TAG N...
set -u
TAG=${1:?tag}; shift
out=gpurun_out/ablanes_${TAG}.log; : > $out
for round in 1 2; do
  for n in "$@"; do
    mode=hipgraph$n; [ "$n" = 1 ] && mode=hipgraph
    DSPLAT_BENCH_MAX_LANES=$n timeout -k 10 200 python -u bench.py --batch 16 --launch $mode --steps 500 --warmup 20 \
      --extra "" --no-cpu-baseline --no-reference-binning > gpurun_out/ablanes_${TAG}_$n.log 2>&1 || { echo "$n failed"; exit 1; }
    python3 - "$n" gpurun_out/ablanes_${TAG}_$n.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)
        print('lanes', sys.argv[1], 'value', d['value'], 'ms', d['ms_per_step'])
PY
  done
done
cat $out
