#!/bin/bash
# SQ_INSTS_VALU / LDS / wave counts of the headline kernels for main and variant libraries
# (separate --pmc pass per library). usage: bash tools/pmc_split.sh TAG NAME...
set -u
TAG=${1:?tag}; shift
cd /tmp && export TMPDIR=/tmp; cd - > /dev/null
for n in "$@"; do
  lib=""; [ "$n" != main ] && lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so
  d=gpurun_out/pmc_${TAG}_$n
  DSPLAT_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU} --output-format csv -d $d -o run \
    -- python3 bench.py --batch 16 --launch eager --steps 5 --warmup 2 --extra "" --no-cpu-baseline \
    --no-reference-binning > $d.log 2>&1 || { echo "$n pmc failed"; exit 1; }
  echo "== $n"; python3 tools/pmc_raw.py $d k_sort_render | tail -3
done
