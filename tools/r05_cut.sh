#!/bin/bash
# Depth-cut check on the GPU box: the depth-cut GPU tests, the config D / E bench legs, and a
# stats + SQ PMC pass of the config-E leg (k_preprocess_cut LDS conflicts); stops at the first
# step that ends by a signal / timeout.  usage: bash tools/r05_cut.sh TAG
set -u
TAG=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_raster_gpu.py tests/test_fullsize_parity.py tests/test_training_parity.py -m gpu -q -k "cut or config_d or dl3dv" \
    --timeout 200 --timeout-method thread > gpurun_out/cuttest_${TAG}.log 2>&1
rc=$?
tail -4 gpurun_out/cuttest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --skip-headline --extra dl3dv,recon12 --no-cpu-baseline > gpurun_out/cutbench_${TAG}.log 2>&1 \
    || { echo "bench failed"; tail -5 gpurun_out/cutbench_${TAG}.log; exit 1; }
python - gpurun_out/cutbench_${TAG}.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        for k in ('render_config_d', 'recon_config_e'):
            v = d.get(k, {})
            print(k, {x: v.get(x) for x in ('ms_per_step', 'ms_per_scene', 'views_per_s', 'value')},
                  'kernels', v.get('roofline', {}).get('per_step_ms_by_kernel'))
PY
export TMPDIR=/tmp
out=gpurun_out/prof_cut_${TAG}
mkdir -p $out
B="python3 bench.py --skip-headline --no-cpu-baseline --extra recon12 --extra-steps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- $B > $out/stats.log 2>&1 \
    || { echo "stats failed"; exit 1; }
python3 tools/kstats.py $(find $out/stats -name '*kernel_stats.csv' | head -1) 10
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY \
    --output-format csv -d $out/pmc_sq -o run -- $B > $out/pmc_sq.log 2>&1 || { echo "pmc failed"; exit 1; }
python3 tools/pmc_raw.py $out/pmc_sq k_preprocess_cut | head -3
python3 tools/pmc_raw.py $out/pmc_sq k_scatter_cut | head -3
exit 0
