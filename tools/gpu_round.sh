#!/bin/bash
# One GPU-box session: the -m gpu suite (with the full-size parity report), then the bench.
# Usage (from the repo root on the box): bash tools/gpu_round.sh TAG [bench args...]
# Stops before the bench when pytest ended by a signal / timeout (exit >= 2 other than a
# plain test failure), so a faulted GPU is not touched again.
set -u
TAG=${1:?tag}; shift
mkdir -p gpurun_out
export DSPLAT_PARITY_REPORT=gpurun_out/parity_${TAG}.jsonl
rm -f "$DSPLAT_PARITY_REPORT"
timeout -k 10 780 python -u -m pytest tests -m gpu -v --maxfail=15 --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_${TAG}.log 2>&1
rc=$?
tail -5 gpurun_out/gputest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 360 python -u bench.py "$@" > gpurun_out/bench_${TAG}.log 2>&1
brc=$?
tail -c 3000 gpurun_out/bench_${TAG}.log
exit $(( rc > brc ? rc : brc ))
