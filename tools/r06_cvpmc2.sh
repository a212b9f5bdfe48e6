#!/bin/bash
# Config-D scale-1 forward + backward PMC passes only (tools/prof_cv.sh --bwd).
# usage: bash tools/r06_cvpmc2.sh TAG [SHAPE]
set -u
tag=${1:?tag}; shape=${2:-config_d_scale1_112x192}
mkdir -p gpurun_out
bash tools/prof_cv.sh ${tag}_bwd $shape --bwd > gpurun_out/cvpmc_${tag}_bwd.log 2>&1
rc=$?
cat gpurun_out/cvpmc_${tag}_bwd.log
python3 tools/pmc_raw.py gpurun_out/prof_cv_${tag}_bwd/atomic k_dtgt_sum | head -2
python3 tools/pmc_raw.py gpurun_out/prof_cv_${tag}_bwd/fetch k_dtgt_sum | head -2
python3 tools/pmc_raw.py gpurun_out/prof_cv_${tag}_bwd/write k_dtgt_sum | head -2
exit $rc
