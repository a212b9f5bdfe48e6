#!/bin/bash
# One PMC pass over a bench leg (run on the GPU box), eager launches:
#   tools/pmc_leg.sh LEG OUTNAME COUNTER...     LEG: main | train | dl3dv
set -e
export TMPDIR=/tmp
leg=$1; name=$2; shift 2
extra=""; [ "$leg" != "main" ] && extra="$leg"
out=gpurun_out/$name
rm -rf $out
timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $out -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --eager --extra "$extra" --extra-steps 2 > $out.log 2>&1
python3 tools/pmc_summary.py $out > $out.json
