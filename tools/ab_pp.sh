#!/bin/bash
# adapter GPU tests on the main library, raster/training GPU tests on variant pb_pref, then A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_adapter_gpu.py \
  > gpurun_out/abpp_adapter_tests.log 2>&1 || { echo "adapter tests failed"; tail -30 gpurun_out/abpp_adapter_tests.log; exit 1; }
tail -1 gpurun_out/abpp_adapter_tests.log
DSPLAT_LIB=my_depthsplat_amd/lib/variants/libdsplat_pb_pref.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_raster_gpu.py tests/test_training_parity.py tests/test_rasterizer_module.py \
  > gpurun_out/abpp_raster_tests.log 2>&1 || { echo "pb_pref tests failed"; tail -30 gpurun_out/abpp_raster_tests.log; exit 1; }
tail -1 gpurun_out/abpp_raster_tests.log
bash tools/ab_train.sh pp main pb_pref
