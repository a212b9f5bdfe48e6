#!/bin/bash
# Round-5 GPU check: the -m gpu suite, then the headline bench leg (eager roofline probe
# included), each under its own time limit; stops at the first step that ends by a signal.
# usage: bash tools/r05_check.sh TAG [pytest selectors...]
set -u
TAG=${1:?tag}; shift
mkdir -p gpurun_out
sel=("$@"); [ ${#sel[@]} -eq 0 ] && sel=(tests)
timeout -k 10 600 python -u -m pytest "${sel[@]}" -m gpu -q --maxfail=10 --timeout 240 --timeout-method thread \
    > gpurun_out/gputest_${TAG}.log 2>&1
rc=$?
tail -12 gpurun_out/gputest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --extra "" --no-cpu-baseline > gpurun_out/bench_${TAG}.log 2>&1
brc=$?
tail -c 1200 gpurun_out/bench_${TAG}.log
exit $(( rc > brc ? rc : brc ))
