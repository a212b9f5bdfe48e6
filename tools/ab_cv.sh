#!/bin/bash
# Same-box A/B of library variants on the cost-volume bench leg (4 shapes, fwd and fwd+bwd).
# usage: bash tools/ab_cv.sh TAG NAME...   (NAME = main or lib/variants/libdsplat_NAME.so)
set -u
TAG=${1:?tag}; shift
mkdir -p gpurun_out
out=gpurun_out/abcv_${TAG}.log; : > $out
for round in 1 2; do
  for n in "$@"; do
    lib=""; [ "$n" != main ] && lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so
    DSPLAT_LIB=$lib timeout -k 10 200 python -u bench.py --batch 1 --launch eager --steps 5 --warmup 2 --extra costvol \
      --no-cpu-baseline --no-reference-binning > gpurun_out/abcv_${TAG}_${n}.log 2>&1 || { echo "$n failed"; exit 1; }
    python - "$n" gpurun_out/abcv_${TAG}_${n}.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)['cost_volume']
        print(sys.argv[1], ' '.join(f"{k[:14]}: {v['ms_per_call']:.4f}/{v['ms_fwd_bwd']:.4f}" for k, v in d.items() if isinstance(v, dict)))
PY
  done
done
cat $out
