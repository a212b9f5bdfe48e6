#!/bin/bash
# Same-box A/B of library variants on the config-C training step (bench.py train leg).
# usage: bash tools/ab_train.sh TAG NAME...   (NAME = main or lib/variants/libdsplat_NAME.so)
set -u
TAG=${1:?tag}; shift
mkdir -p gpurun_out
out=gpurun_out/abt_${TAG}.log; : > $out
for round in 1 2; do
  for n in "$@"; do
    lib=""; [ "$n" != main ] && lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so
    DSPLAT_LIB=$lib timeout -k 10 200 python -u bench.py --batch 1 --launch eager --steps 20 --warmup 3 --extra train \
      --extra-steps 20 --no-cpu-baseline --no-reference-binning > gpurun_out/abt_${TAG}_${n}.log 2>&1 || { echo "$n failed"; exit 1; }
    python - "$n" gpurun_out/abt_${TAG}_${n}.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)
        t = d['train_config_c']
        k = (t.get('roofline') or {}).get('per_step_ms_by_kernel') or {}
        print(sys.argv[1], 'train_config_c ms', t['ms_per_step'], ' '.join(f'{n}={v}' for n, v in k.items()))
PY
  done
done
cat $out
