#!/bin/bash
# Round profile of the default bench (run on the GPU box from the repo root):
#   1. kernel-trace stats of the bench command itself (hipGraph replays + eager timed region)
#   2. separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ), eager launches, fewer steps
#   3. pmc_traffic.json: HBM bytes per launch per kernel (FETCH x2 gfx950 correction + WRITE)
# usage: tools/profile_round.sh TAG
set -e
tag=${1:-r01}
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
# (--launch hipgraph: one scene in flight, so the per-kernel averages are the kernels' own
# durations, comparable with the roofline's eager single-stream HIP-event timing; with N
# scenes in flight the kernels share the chip and their durations stretch)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- \
  python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --extra "" --launch hipgraph > $out/stats.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats_default -o run -- \
  python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --extra "" > $out/stats_default.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --eager --extra "" > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --eager --extra "" > $out/write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $out/sq -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --eager --extra "" > $out/sq.log 2>&1
python3 tools/pmc_summary.py --json $out/pmc_traffic.json 2v256x256x3b1 "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ, $tag" \
  $out/fetch $out/write $out/sq
python3 tools/pmc_summary.py $out/fetch $out/write $out/sq > $out/pmc_summary.json
echo done
