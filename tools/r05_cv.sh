#!/bin/bash
# Cost-volume round-5 check on the GPU box: the cost-volume GPU tests, the bench's cost-volume
# leg alone, then rocprofv3 kernel stats + SQ PMC of config-D scale 1 (stops at the first
# step that ends by a signal / timeout).  usage: bash tools/r05_cv.sh TAG
set -u
TAG=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cost_volume.py -m gpu -q --timeout 120 --timeout-method thread \
    > gpurun_out/cvtest_${TAG}.log 2>&1
rc=$?
tail -6 gpurun_out/cvtest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --skip-headline --extra costvol --no-cpu-baseline > gpurun_out/cvbench_${TAG}.log 2>&1 \
    || { echo "bench failed"; tail -5 gpurun_out/cvbench_${TAG}.log; exit 1; }
python - gpurun_out/cvbench_${TAG}.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        for k, v in d.get('cost_volume', {}).items():
            if isinstance(v, dict):
                print(k, 'fwd', v['ms_per_call'], 'frac', v['frac'], 'fwd+bwd', v['ms_fwd_bwd'], 'frac_fb', v['frac_fwd_bwd'])
PY
export TMPDIR=/tmp
bash tools/prof_cv.sh ${TAG}_d1 config_d_scale1_112x192 > gpurun_out/cvprof_${TAG}_d1.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/cvprof_${TAG}_d1.log; exit 1; }
tail -14 gpurun_out/cvprof_${TAG}_d1.log
exit $rc
