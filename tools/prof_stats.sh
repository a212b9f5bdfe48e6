#!/bin/bash
# rocprofv3 kernel-trace stats of one bench leg on the GPU box (repo root).
# usage: bash tools/prof_stats.sh TAG LEG [bench args...]   (LEG: train, dl3dv, recon12, costvol, train_d, "")
set -u
tag=${1:?tag}; leg=${2?leg}; shift 2
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- \
  python3 bench.py --no-cpu-baseline --no-reference-binning --steps 3 --warmup 2 --batch 1 --launch eager \
  --extra "$leg" --extra-steps 10 "$@" > $out/stats.log 2>&1
rc=$?
f=$(find $out/stats -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && head -25 "$f" | cut -d, -f1-8
exit $rc
