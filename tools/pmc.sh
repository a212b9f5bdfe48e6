#!/bin/bash
# usage: tools_pmc.sh OUTDIR COUNTERS...   (run on the GPU box)
out=$1; shift
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d gpurun_out/$out -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/$out.log 2>&1
