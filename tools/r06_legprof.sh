#!/bin/bash
# Whole-step kernel traces of the config C training leg and the config D render leg (every
# kernel of a step, not only the dominant ones): rocprofv3 --kernel-trace --stats.
# usage: bash tools/r06_legprof.sh TAG
set -u
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
for leg in train dl3dv; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/legprof_${tag}_$leg -o run -- \
    python3 bench.py --skip-headline --no-cpu-baseline --extra $leg --extra-steps 10 --detail= \
    > gpurun_out/legprof_${tag}_$leg.log 2>&1 || { echo "$leg prof failed"; tail -5 gpurun_out/legprof_${tag}_$leg.log; exit 1; }
  echo "== $leg"
  python3 tools/kstats.py $(find gpurun_out/legprof_${tag}_$leg -name '*kernel_stats.csv' | head -1) 40
done
