set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_raster_gpu.py tests/test_training_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pool_tests.log 2>&1 || { tail -30 gpurun_out/pool_tests.log; exit 1; }
tail -2 gpurun_out/pool_tests.log
: > gpurun_out/abt_pool.log
for r in 1 2; do for v in 0 1; do
DSPLAT_REUSE_DGEOM=$v timeout -k 10 200 python -u bench.py --batch 1 --launch eager --steps 20 --warmup 3 --extra train --extra-steps 20 --no-cpu-baseline --no-reference-binning > gpurun_out/abt_pool_$v.log 2>&1 || { echo "fail $v"; exit 1; }
python -c "
import json,sys
for l in open('gpurun_out/abt_pool_$v.log'):
    if l.startswith('{'): print('reuse=$v', json.loads(l)['train_config_c']['ms_per_step'])
" >> gpurun_out/abt_pool.log
done; done
cat gpurun_out/abt_pool.log
