#!/bin/bash
# Helper-stream accumulator fill: raster backward / head / training tests, then a same-box A/B of
# the config C leg: side (default, DSPLAT_SIDE_FILL=1) vs inorder (DSPLAT_SIDE_FILL=0), 3 rounds.
# (DSPLAT_SIDE_FILL was dropped after this A/B, profiles/r06ar_side_fill_ab.txt; kept as its recipe)
# usage: bash tools/r06_abside.sh TAG
set -u
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_raster_gpu.py tests/test_head_render.py tests/test_training_parity.py \
  tests/test_rasterizer_module.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/abside_test_$tag.log 2>&1
rc=$?
tail -2 gpurun_out/abside_test_$tag.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/abside_test_$tag.log | head -20; exit $rc; fi
for r in 1 2 3; do
  for n in side inorder; do
    sf=1; [ "$n" = inorder ] && sf=0
    DSPLAT_SIDE_FILL=$sf timeout -k 10 200 python3 bench.py --skip-headline --no-cpu-baseline \
      --extra train --extra-steps 20 --detail= > gpurun_out/abside_${tag}_${n}_$r.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/abside_${tag}_${n}_$r.log; exit 1; }
    python3 -c "import json,sys; t=json.loads(open(sys.argv[1]).read().splitlines()[-1])['train_config_c']; print(sys.argv[2], 'C ms', t['ms_per_step'], json.dumps(t['roofline']['per_step_ms_by_kernel']))" gpurun_out/abside_${tag}_${n}_$r.log $n
  done
done
