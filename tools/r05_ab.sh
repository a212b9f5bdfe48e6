#!/bin/bash
# Same-box A/B of variant libraries: image digests (bit-identity with main), then the eager
# 16-scene headline probe (tools/ab_bench.sh, two rounds in alternating order).
# usage: bash tools/r05_ab.sh TAG [--cut] NAME...   (NAME = main or lib/variants/libdsplat_NAME.so)
set -u
TAG=${1:?tag}; shift
CUT=""; [ "${1:-}" = "--cut" ] && { CUT=--cut; shift; }
mkdir -p gpurun_out
for n in "$@"; do
  lib=""; [ "$n" != main ] && lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so
  d=$(DSPLAT_LIB=$lib timeout -k 10 240 python -u tools/img_digest.py $CUT 2>&1 | tail -1) || { echo "$n digest failed: $d"; exit 1; }
  echo "digest $n $d" | tee -a gpurun_out/ab_${TAG}_digest.log
done
bash tools/ab_bench.sh $TAG 16 "$@"
