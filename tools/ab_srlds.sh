#!/bin/bash
# Same-box A/B of the sort_render LDS request (DSPLAT_SR_LDS) in the headline's multi-lane mode:
# does leaving room for one k_project_emit workgroup per CU let the lanes' kernels overlap?
# usage: bash tools/ab_srlds.sh TAG BYTES [MODE]
set -u
tag=${1:?tag}; bytes=${2:?bytes}; mode=${3:-hipgraph7}
mkdir -p gpurun_out
B="python3 bench.py --no-cpu-baseline --no-reference-binning --extra= --batch 16 --launch $mode --steps 300 --warmup 20 --detail="
for r in 1 2; do
  for v in main pad; do
    if [ $v = pad ]; then export DSPLAT_SR_LDS=$bytes; else unset DSPLAT_SR_LDS; fi
    timeout -k 10 240 $B > gpurun_out/ab_srlds_${tag}_${v}_$r.log 2>&1 || { echo "$v $r failed"; tail -3 gpurun_out/ab_srlds_${tag}_${v}_$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_ms'])" gpurun_out/ab_srlds_${tag}_${v}_$r.log "$v $r"
  done
done
export DSPLAT_SR_LDS=$bytes
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_srlds_${tag}_trace -o run -- $B > gpurun_out/ab_srlds_${tag}_trace.log 2>&1
echo "trace rc=$?"
