#!/bin/bash
# Cost-volume profile (GPU box): kernel stats, MFMA busy cycles, HBM bytes (separate passes).
set -e
export TMPDIR=/tmp
out=gpurun_out/prof_cv
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- python3 tools/cv_bench.py > $out/stats.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES --output-format csv -d $out/mfma -o run -- python3 tools/cv_bench.py > $out/mfma.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 tools/cv_bench.py > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 tools/cv_bench.py > $out/write.log 2>&1
python3 tools/pmc_summary.py $out/mfma $out/fetch $out/write > $out/pmc_summary.json
echo done
