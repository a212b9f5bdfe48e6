#!/bin/bash
# Cost-volume tests (views mode included), then the cost-volume bench leg + its kernel stats.
# usage: bash tools/r06_cvviews.sh TAG
set -u
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cost_volume.py -x -v --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/cvtest_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/cvtest_$tag.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|error" gpurun_out/cvtest_$tag.log | head -20; exit $rc; fi
bash tools/r06_cvleg.sh $tag
