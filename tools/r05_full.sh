#!/bin/bash
# Round-5 combined GPU pass: the whole -m gpu suite, then the bench's cost-volume and config-C
# training legs (no headline). Stops at the first step that ends by a signal / timeout.
# usage: bash tools/r05_full.sh TAG
set -u
TAG=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 240 --timeout-method thread \
    > gpurun_out/gputest_${TAG}.log 2>&1
rc=$?
tail -12 gpurun_out/gputest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u bench.py --skip-headline --extra costvol,train --no-cpu-baseline > gpurun_out/legbench_${TAG}.log 2>&1 \
    || { echo "bench failed"; tail -5 gpurun_out/legbench_${TAG}.log; exit 1; }
python - gpurun_out/legbench_${TAG}.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        for k, v in d.get('cost_volume', {}).items():
            if isinstance(v, dict):
                print(k, 'fwd', v['ms_per_call'], 'frac', v['frac'], 'fwd+bwd', v['ms_fwd_bwd'], 'frac_fb', v['frac_fwd_bwd'])
        t = d.get('train_config_c', {})
        print('train_config_c', {x: t.get(x) for x in ('ms_per_step', 'value', 'unit')},
              (t.get('roofline') or {}).get('per_step_ms_by_kernel'))
PY
exit $rc
