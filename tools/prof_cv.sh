#!/bin/bash
# Cost-volume profile on the GPU box (repo root): kernel stats + PMC passes for one bench shape.
# usage: bash tools/prof_cv.sh TAG SHAPE [--bwd]   (SHAPE: a bench._costvol_case tag)
set -u
tag=${1:?tag}; shape=${2:?shape}; shift 2
export TMPDIR=/tmp
out=gpurun_out/prof_cv_$tag
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 120 "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/$name.log; exit $rc; fi
}
run stats rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- python3 tools/cv_case.py $shape 20 "$@"
run pmc_sq rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT --output-format csv -d $out/pmc_sq -o run -- python3 tools/cv_case.py $shape 5 "$@"
run pmc_grbm rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES --output-format csv -d $out/pmc_grbm -o run -- python3 tools/cv_case.py $shape 5 "$@"
run fetch rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 tools/cv_case.py $shape 5 "$@"
run atomic rocprofv3 --kernel-trace --pmc TCC_EA0_ATOMIC_sum TCC_EA0_WRREQ_sum --output-format csv -d $out/atomic -o run -- python3 tools/cv_case.py $shape 5 "$@"
run write rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 tools/cv_case.py $shape 5 "$@"
python3 tools/kstats.py $(find $out/stats -name '*kernel_stats.csv' | head -1) 8
python3 tools/pmc_raw.py $out/pmc_sq k_cost_ | head -4
python3 tools/pmc_raw.py $out/pmc_grbm k_cost_ | head -4
python3 tools/pmc_raw.py $out/fetch k_cost_epi | head -2
python3 tools/pmc_raw.py $out/write k_cost_epi | head -2
python3 tools/pmc_raw.py $out/fetch k_to_hwc | head -2
python3 tools/pmc_raw.py $out/write k_to_hwc | head -2
python3 tools/pmc_raw.py $out/atomic k_cost_epi | head -3
python3 tools/pmc_raw.py $out/pmc_sq k_cost_epi_bwd | head -3
python3 tools/pmc_raw.py $out/fetch k_cost_epi_bwd | head -2
python3 tools/pmc_raw.py $out/write k_cost_epi_bwd | head -2
