#!/bin/bash
# Round-6 cost-volume GPU check: the cost-volume / context test files, then (only if pytest
# itself ended normally: 0 = green, 1 = failures) the headline profile.
# usage: bash tools/r06_cv.sh TAG
set -u
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cost_volume.py tests/test_contexts.py -x -v --timeout 120 \
  --timeout-method thread -m gpu > gpurun_out/cv_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/cv_$tag.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash tools/r06_headline.sh $tag
