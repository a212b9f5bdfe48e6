#!/bin/bash
# Round-6 cost-volume PMC refresh: tools/prof_cv.sh per bench shape (stats + SQ / GRBM / FETCH /
# WRITE passes), then gpurun_out/pmc_costvol.json (the bench's mfma_busy source).
# usage: bash tools/r06_pmc_cv.sh TAG
set -u
tag=${1:?tag}
specs=""
for shp in config_a_32x32 config_b_scale0_64x64 config_d_scale0_56x96 config_d_scale1_112x192; do
  bash tools/prof_cv.sh ${tag}_$shp $shp > gpurun_out/cvpmc_${tag}_$shp.log 2>&1 || { echo "cv $shp failed"; tail -5 gpurun_out/cvpmc_${tag}_$shp.log; exit 1; }
  specs="$specs $shp=gpurun_out/prof_cv_${tag}_$shp"
done
python3 tools/cv_pmc_json.py gpurun_out/pmc_costvol.json "rocprofv3 --pmc (tools/r06_pmc_cv.sh, $tag), python tools/cv_case.py" $specs
