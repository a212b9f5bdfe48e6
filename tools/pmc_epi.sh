#!/bin/bash
# k_epi_groups counters at config D scale 1 (one SQ pass, kernel stats).
set -u
mkdir -p gpurun_out/pmc_epi
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc_epi/stats -o run -- python3 $R/tools/cv_case.py config_d_scale1_112x192 10 > $R/gpurun_out/pmc_epi/stats.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/pmc_epi/sq -o run -- python3 $R/tools/cv_case.py config_d_scale1_112x192 3 > $R/gpurun_out/pmc_epi/sq.log 2>&1 || exit 1
echo done
