#!/bin/bash
# Same-box A/B of library variants on secondary bench legs (bench.py --skip-headline).
# usage: bash tools/ab_legs.sh TAG LEG NAME...   (NAME = main or lib/variants/libdsplat_NAME.so)
set -u
TAG=${1:?tag}; LEG=${2:?leg}; shift 2
mkdir -p gpurun_out
out=gpurun_out/abl_${TAG}.log; : > $out
for round in 1 2; do
  for n in "$@"; do
    lib=""; [ "$n" != main ] && lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so
    DSPLAT_LIB=$lib timeout -k 10 300 python -u bench.py --skip-headline --no-cpu-baseline --extra $LEG --extra-steps 10 \
      > gpurun_out/abl_${TAG}_${n}.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abl_${TAG}_${n}.log; exit 1; }
    python - "$n" gpurun_out/abl_${TAG}_${n}.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)
        for k, v in d.items():
            if isinstance(v, dict) and 'workload' in v:
                r = v.get('roofline') or {}
                print(sys.argv[1], k, 'ms', v.get('ms_per_step', v.get('ms_per_scene')), 'kernels', r.get('per_step_ms_by_kernel'))
PY
  done
done
cat $out
