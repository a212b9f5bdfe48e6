#!/bin/bash
# Cost-volume tests (main library), then a same-box A/B of the cost-volume leg: main vs
# lib/variants/libdsplat_NAME.so, 3 rounds.
# usage: bash tools/r06_abcv.sh TAG NAME...
set -u
tag=${1:?tag}; shift; vars="$*"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cost_volume.py -x -q --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/abcvtest_$tag.log 2>&1
rc=$?
tail -2 gpurun_out/abcvtest_$tag.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/abcvtest_$tag.log | head -20; exit $rc; fi
for r in 1 2 3; do
  for n in main $vars; do
    lib=""; [ "$n" != main ] && lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so
    DSPLAT_LIB=$lib timeout -k 10 300 python3 bench.py --skip-headline --no-cpu-baseline --extra costvol --detail= \
      > gpurun_out/abcv_${tag}_${n}_$r.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/abcv_${tag}_${n}_$r.log; exit 1; }
    python3 - gpurun_out/abcv_${tag}_${n}_$r.log $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])["cost_volume"]
print(sys.argv[2], " ".join(f"{k[9:20]}: {v['ms_per_call']:.4f}/{v['ms_fwd_bwd']:.4f}" for k, v in d.items() if isinstance(v, dict)))
PY
  done
done
