#!/bin/bash
# Kernel stats of one secondary bench leg (run on the GPU box): tools/prof_extra.sh train|dl3dv
set -e
export TMPDIR=/tmp
leg=$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$leg -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --extra $leg --extra-steps 5 > gpurun_out/prof_$leg.log 2>&1
