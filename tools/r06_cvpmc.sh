#!/bin/bash
# Cost-volume tests + leg timing (tools/r06_cvviews.sh), then the config-D scale-1 forward +
# backward PMC passes (tools/prof_cv.sh --bwd: SQ, GRBM, FETCH, WRITE and the EA atomic count).
# usage: bash tools/r06_cvpmc.sh TAG
set -u
tag=${1:?tag}
bash tools/r06_cvviews.sh $tag || exit $?
# A/B: the grouping on st itself (no helper stream), same box
B="python3 bench.py --skip-headline --no-cpu-baseline --extra costvol --detail="
for fk in 0 1 0 1; do
  DSPLAT_CV_FORK=$fk timeout -k 10 300 $B > gpurun_out/cvfork_${tag}_$fk.log 2>&1 || { echo "fork A/B failed"; exit 1; }
  python3 - gpurun_out/cvfork_${tag}_$fk.log $fk <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
for k, v in d["cost_volume"].items():
    if isinstance(v, dict) and k.startswith("config_d"):
        print(f"fork {sys.argv[2]} {k:30s} fwd {v['ms_per_call']:.4f} ms  fwd+bwd {v['ms_fwd_bwd']:.4f} ms")
PY
done
bash tools/prof_cv.sh ${tag}_d1bwd config_d_scale1_112x192 --bwd > gpurun_out/cvpmc_${tag}_d1bwd.log 2>&1
rc=$?
cat gpurun_out/cvpmc_${tag}_d1bwd.log
exit $rc
