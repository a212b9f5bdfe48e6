#!/bin/bash
# The whole -m gpu suite, then kernel traces (per-dispatch start / end) of the config D render
# and config C training legs: where the step's time goes between the kernels.
# usage: bash tools/r06_legtrace.sh TAG
set -u
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/gputest_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/gputest_$tag.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/gputest_$tag.log | head -20; exit $rc; fi
for leg in dl3dv train; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/legtrace_${tag}_$leg -o run -- \
    python3 bench.py --skip-headline --no-cpu-baseline --extra $leg --extra-steps 5 --detail= \
    > gpurun_out/legtrace_${tag}_$leg.log 2>&1 || { echo "$leg trace failed"; tail -5 gpurun_out/legtrace_${tag}_$leg.log; exit 1; }
  echo "$leg traced"
done
