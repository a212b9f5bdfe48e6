#!/bin/bash
# Round-5 iteration step on the GPU box: one GPU test file (or "none"), then rocprofv3 kernel
# stats (no counters) of cost-volume shapes fwd+bwd. Stops at the first failing GPU step.
# usage: bash tools/r05_step.sh TAG TESTFILE|none SHAPE...
set -u
TAG=${1:?tag}; TF=${2:?testfile}; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$TF" != none ]; then
  timeout -k 10 400 python -u -m pytest $TF -m gpu -q --timeout 200 --timeout-method thread \
      > gpurun_out/steptest_${TAG}.log 2>&1
  rc=$?
  tail -8 gpurun_out/steptest_${TAG}.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
for shape in "$@"; do
  out=gpurun_out/prof_cvb_${TAG}_$shape
  mkdir -p $out
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
      python3 tools/cv_case.py $shape 20 --bwd > $out/run.log 2>&1 || { echo "prof $shape failed"; tail -5 $out/run.log; exit 1; }
  echo "== $shape fwd+bwd x20"
  python3 tools/kstats.py $(find $out -name '*kernel_stats.csv' | head -1) 12
done
