#!/bin/bash
# Adapter variants: GPU parity (adapter tests) under each variant library, then the config-C
# training A/B. usage: bash tools/ab_adapter.sh TAG NAME...
set -u
TAG=${1:?tag}; shift
mkdir -p gpurun_out
for n in "$@"; do
  [ "$n" = main ] && continue
  DSPLAT_LIB=my_depthsplat_amd/lib/variants/libdsplat_$n.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_adapter_gpu.py tests/test_golden_adapter.py tests/test_training_parity.py \
    > gpurun_out/abad_${TAG}_${n}_tests.log 2>&1 || { echo "$n tests failed"; tail -30 gpurun_out/abad_${TAG}_${n}_tests.log; exit 1; }
  tail -2 gpurun_out/abad_${TAG}_${n}_tests.log
done
bash tools/ab_train.sh $TAG "$@"
