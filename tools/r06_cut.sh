#!/bin/bash
# Raster GPU tests (depth cut included), then the config D render / config E legs.
# usage: bash tools/r06_cut.sh TAG
set -u
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_raster_gpu.py tests/test_fullsize_parity.py tests/test_bounded_keys.py \
  -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/cuttest_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/cuttest_$tag.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/cuttest_$tag.log | head -20; exit $rc; fi
for r in 1 2; do
timeout -k 10 300 python3 bench.py --skip-headline --no-cpu-baseline --extra dl3dv,recon12 --extra-steps 10 --detail= \
  > gpurun_out/cutleg_${tag}_$r.log 2>&1 || { echo "legs failed"; tail -5 gpurun_out/cutleg_${tag}_$r.log; exit 1; }
python3 - gpurun_out/cutleg_${tag}_$r.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
r = d["render_config_d"]
print("config D ms", r["ms_per_step"], json.dumps(r["roofline"]["per_step_ms_by_kernel"]))
print("config E ms/scene", d["recon_config_e"]["ms_per_scene"])
PY
done
