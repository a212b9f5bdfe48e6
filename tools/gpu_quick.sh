#!/bin/bash
# GPU tests (optionally a subset) + the headline bench leg only, for quick A/B on the box.
# usage: bash tools/gpu_quick.sh TAG [pytest selectors...]
set -u
TAG=${1:?tag}; shift
mkdir -p gpurun_out
sel=("$@"); [ ${#sel[@]} -eq 0 ] && sel=(tests)
timeout -k 10 600 python -u -m pytest "${sel[@]}" -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_${TAG}.log 2>&1
rc=$?
tail -15 gpurun_out/gputest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --extra "" --no-cpu-baseline > gpurun_out/bench_${TAG}.log 2>&1
brc=$?
tail -c 1500 gpurun_out/bench_${TAG}.log
exit $(( rc > brc ? rc : brc ))
