#!/bin/bash
# PMC pass (SQ counters) of one kbench kernel per library variant:
#   KB_KERNEL=sort_render KB_ARGS=--exact tools/pmc_variants.sh main VARIANT...
set -e
export TMPDIR=/tmp
for v in "$@"; do
  d=gpurun_out/pmcv_$v; rm -rf $d
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $d -o run -- \
    python3 tools/kbench.py --kernel $KB_KERNEL ${KB_ARGS:-} --views 3 --iters 5 $v > $d.log 2>&1
  python3 tools/pmc_summary.py $d > $d.json
done
