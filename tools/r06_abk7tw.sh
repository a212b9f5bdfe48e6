#!/bin/bash
# K7 tile-wave form: raster backward / head / training tests, then a same-box A/B of the config C
# leg: main (tile wave, WPE 4), tw3 (tile wave, WPE 3 variant library), sub (DSPLAT_K7_SUBTILE=1:
# the sub-tile waves of k_render_bwd), 3 rounds.
# usage: bash tools/r06_abk7tw.sh TAG [VARIANT...]   (default: tw3)
set -u
tag=${1:?tag}; shift; vars=${*:-tw3}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_raster_gpu.py tests/test_head_render.py tests/test_training_parity.py \
  tests/test_rasterizer_module.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/k7twtest_$tag.log 2>&1
rc=$?
tail -2 gpurun_out/k7twtest_$tag.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/k7twtest_$tag.log | head -20; exit $rc; fi
for r in 1 2 3; do
  for n in main $vars sub; do
    lib=""; [ "$n" != main ] && [ "$n" != sub ] && lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so
    sub=""; [ "$n" = sub ] && sub=1
    DSPLAT_K7_SUBTILE=$sub DSPLAT_LIB=$lib timeout -k 10 200 python3 bench.py --skip-headline --no-cpu-baseline \
      --extra train --extra-steps 20 --detail= > gpurun_out/abk7tw_${tag}_${n}_$r.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/abk7tw_${tag}_${n}_$r.log; exit 1; }
    python3 -c "import json,sys; t=json.loads(open(sys.argv[1]).read().splitlines()[-1])['train_config_c']; print(sys.argv[2], 'C ms', t['ms_per_step'], json.dumps(t['roofline']['per_step_ms_by_kernel']))" gpurun_out/abk7tw_${tag}_${n}_$r.log $n
  done
done
