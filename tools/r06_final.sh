#!/bin/bash
# Round-6 end-of-round pass on the GPU box: the whole -m gpu suite, the default bench (all
# legs, CPU baseline) after smoke(), then rocprofv3 kernel stats of a short headline run. Each step has its
# own time limit; stops at the first step that ends by a signal / timeout.
# usage: bash tools/r06_final.sh TAG
set -u
TAG=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 240 --timeout-method thread \
    > gpurun_out/gputest_${TAG}.log 2>&1
rc=$?
tail -6 gpurun_out/gputest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_${TAG}.log 2>&1
src=$?
tail -2 gpurun_out/smoke_${TAG}.log
if [ $src -ne 0 ]; then echo "smoke rc=$src: stopping"; exit $src; fi
timeout -k 10 900 python -u bench.py > gpurun_out/bench_${TAG}.log 2>&1
brc=$?
echo "bench rc=$brc"
if [ $brc -ne 0 ]; then tail -5 gpurun_out/bench_${TAG}.log; exit $brc; fi
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
    python3 bench.py --steps 50 --warmup 5 --extra "" --no-cpu-baseline --no-reference-binning \
    > gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/kstats.py $(find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' | head -1) 8
exit $rc
