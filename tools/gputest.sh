#!/bin/bash
# The -m gpu suite alone on the GPU box (parity report + per-test durations).
# Usage (repo root on the box): bash tools/gputest.sh TAG [pytest selectors...]
set -u
TAG=${1:?tag}; shift
mkdir -p gpurun_out
export DSPLAT_PARITY_REPORT=gpurun_out/parity_${TAG}.jsonl
rm -f "$DSPLAT_PARITY_REPORT"
sel=("$@"); [ ${#sel[@]} -eq 0 ] && sel=(tests)
timeout -k 10 900 python -u -m pytest "${sel[@]}" -m gpu -v --maxfail=20 --timeout 300 --timeout-method thread \
    --durations=15 > gpurun_out/gputest_${TAG}.log 2>&1
rc=$?
tail -25 gpurun_out/gputest_${TAG}.log
exit $rc
