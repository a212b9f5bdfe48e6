#!/bin/bash
# Same-box A/B of library variants on the headline workload: eager B-scene launches, per-kernel
# HIP-event averages (bench.py roofline probe). usage: bash tools/ab_bench.sh TAG BATCH NAME...
# (NAME = main or a lib/variants/libdsplat_NAME.so); two rounds in alternating order.
set -u
TAG=${1:?tag}; B=${2:?batch}; shift 2
mkdir -p gpurun_out
out=gpurun_out/ab_${TAG}.log; : > $out
for round in 1 2; do
  for n in "$@"; do
    lib=""; [ "$n" != main ] && lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so
    DSPLAT_LIB=$lib timeout -k 10 200 python -u bench.py --batch $B --launch eager --steps 200 --warmup 10 --extra "" \
      --no-cpu-baseline --no-reference-binning > gpurun_out/ab_${TAG}_${n}.log 2>&1 || { echo "$n failed"; exit 1; }
    python - "$n" gpurun_out/ab_${TAG}_${n}.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l); r = d['roofline']
        print(sys.argv[1], 'value', d['value'], 'ms', d['ms_per_step'], 'probe', r['per_kernel_avg_ms_probe'], 'avg', r['avg_ms'])
PY
  done
done
cat $out
