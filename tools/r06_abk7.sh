#!/bin/bash
# K7 cross-wave combine: the raster backward / training / head tests, then a same-box A/B of
# the config C training leg (main vs lib/variants/libdsplat_k7old.so), 3 rounds.
# usage: bash tools/r06_abk7.sh TAG [VARIANT...]   (default variant: k7old)
set -u
tag=${1:?tag}; shift; vars=${*:-k7old}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_raster_gpu.py tests/test_head_render.py tests/test_training_parity.py \
  tests/test_rasterizer_module.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/k7test_$tag.log 2>&1
rc=$?
tail -2 gpurun_out/k7test_$tag.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/k7test_$tag.log | head -20; exit $rc; fi
for r in 1 2 3; do
  for n in main $vars; do
    lib=""; [ "$n" != main ] && lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so
    ag=""; [ "$n" = bwdrec ] && ag=1  # (that variant takes the geometry records: the pre-ABI-21 backward)
    DSPLAT_AB_GEOM=$ag DSPLAT_LIB=$lib timeout -k 10 200 python3 bench.py --skip-headline --no-cpu-baseline --extra train --extra-steps 20 \
      --detail= > gpurun_out/abk7_${tag}_${n}_$r.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/abk7_${tag}_${n}_$r.log; exit 1; }
    python3 -c "import json,sys; t=json.loads(open(sys.argv[1]).read().splitlines()[-1])['train_config_c']; print(sys.argv[2], 'C ms', t['ms_per_step'], json.dumps(t['roofline']['per_step_ms_by_kernel']))" gpurun_out/abk7_${tag}_${n}_$r.log $n
  done
done
