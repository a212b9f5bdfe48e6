#!/bin/bash
# Kernel-trace stats of each extra bench leg (config C training, D 960x540, E recon12), run
# on the GPU box from the repo root. The main config-B leg runs too (few steps) and shows up
# in the same stats; the leg's kernels are the ones the leg names in DESIGN.md.
# usage: tools/profile_legs.sh TAG
set -e
tag=${1:-r01}
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
for leg in train dl3dv recon12; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/leg_$leg -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --extra $leg --extra-steps 10 > $out/leg_$leg.log 2>&1
done
echo done
