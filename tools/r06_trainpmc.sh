#!/bin/bash
# Config C training leg: the EA atomic request count per kernel (rocprofv3 --pmc, own pass).
# usage: bash tools/r06_trainpmc.sh TAG
set -u
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc TCC_EA0_ATOMIC_sum TCC_EA0_WRREQ_sum --output-format csv \
  -d gpurun_out/trainpmc_$tag -o run -- python3 bench.py --skip-headline --no-cpu-baseline --extra train \
  --extra-steps 3 --detail= > gpurun_out/trainpmc_$tag.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/trainpmc_$tag.log; exit 1; }
for k in k_render_bwd k_head_bwd k_project_emit k_sort_render; do
  python3 tools/pmc_raw.py gpurun_out/trainpmc_$tag $k | head -2
done
