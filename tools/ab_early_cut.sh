#!/bin/bash
# Same-box A/B of the early depth-cut scatter (DSPLAT_EARLY_CUT_SCATTER=1 / 0) on the config D
# render and config E legs, plus the early-scatter tests.
# usage: bash tools/ab_early_cut.sh TAG
set -u
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_raster_gpu.py -k "depth_cut" -x -q --timeout 240 --timeout-method thread \
  -m gpu > gpurun_out/earlytest_$tag.log 2>&1
rc=$?
tail -2 gpurun_out/earlytest_$tag.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/earlytest_$tag.log | head -20; exit $rc; fi
for r in 1 2 3; do
  for e in 1 0; do
    DSPLAT_EARLY_CUT_SCATTER=$e timeout -k 10 300 python3 bench.py --skip-headline --no-cpu-baseline --extra dl3dv,recon12 \
      --extra-steps 20 --detail= > gpurun_out/abearly_${tag}_${e}_$r.log 2>&1 || { echo "leg failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('early', sys.argv[2], 'D ms', d['render_config_d']['ms_per_step'], 'E ms/scene', d['recon_config_e']['ms_per_scene'])" gpurun_out/abearly_${tag}_${e}_$r.log $e
  done
done
