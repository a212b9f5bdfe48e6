#!/bin/bash
# Fused head backward: its tests + the adapter / training tests, then the config C and config D
# training legs (and their kernel stats).
# usage: bash tools/r06_headbwd.sh TAG
set -u
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_head_render.py tests/test_adapter_gpu.py tests/test_training_parity.py \
  tests/test_loss_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/headtest_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/headtest_$tag.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/headtest_$tag.log | head -20; exit $rc; fi
timeout -k 10 300 python3 bench.py --skip-headline --no-cpu-baseline --extra train,train_d --extra-steps 10 --detail= \
  > gpurun_out/trainleg_$tag.log 2>&1 || { echo "legs failed"; tail -5 gpurun_out/trainleg_$tag.log; exit 1; }
python3 - gpurun_out/trainleg_$tag.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
c = d["train_config_c"]
print("config C ms", c["ms_per_step"], json.dumps(c["roofline"]["per_step_ms_by_kernel"]))
print("config D DP ms", d["train_config_d_dp"]["ms_per_step"])
PY
