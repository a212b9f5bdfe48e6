#!/bin/bash
# Config-D DP training leg: whole-step kernel trace (rocprofv3 --kernel-trace --stats).
# usage: bash tools/r06_tdprof.sh TAG
set -u
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tdprof_$tag -o run -- \
  python3 bench.py --skip-headline --no-cpu-baseline --extra train_d --extra-steps 5 --detail= \
  > gpurun_out/tdprof_$tag.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/tdprof_$tag.log; exit 1; }
python3 tools/kstats.py $(find gpurun_out/tdprof_$tag -name '*kernel_stats.csv' | head -1) 40
