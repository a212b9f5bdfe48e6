#!/bin/bash
# Round-6 headline evidence on the GPU box (repo root): rocprofv3 kernel trace + stats of the
# bench's eager 16-scene launches (the roofline's avg_ms comes from these launches), a kernel
# trace of the hipgraph7 mode (per-dispatch start / end: how much the lanes overlap), and the
# PMC passes (FETCH_SIZE / WRITE_SIZE / SQ group) summarised into
# gpurun_out/prof_TAG/pmc_traffic_2v256x256x3b16.json (copied to profiles/ by hand).
# usage: bash tools/r06_headline.sh TAG
set -u
tag=${1:?tag}
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
run() {  # run NAME TIMEOUT CMD...: stop the whole script on any failure
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/$name.log; echo "stopping after $name"; exit $rc; fi
}
B="python3 bench.py --no-cpu-baseline --no-reference-binning --extra="
run stats_b16_eager 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats_b16_eager -o run -- \
  $B --steps 50 --warmup 5 --batch 16 --launch eager
run trace_b16_hipgraph7 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace_b16_hipgraph7 -o run -- \
  $B --steps 50 --warmup 5 --batch 16 --launch hipgraph7
for pass in FETCH_SIZE WRITE_SIZE \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"; do
  n=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  run pmc_b16_$n 240 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $out/pmc_b16_$n -o run -- \
    $B --steps 10 --warmup 3 --eager --batch 16
done
python3 tools/pmc_summary.py --json $out/pmc_traffic_2v256x256x3b16.json 2v256x256x3b16 \
  "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ (tools/r06_headline.sh, $tag)" $out/pmc_b16_fetch_size \
  $out/pmc_b16_write_size $out/pmc_b16_sq_waves
python3 tools/kstats.py $(find $out/stats_b16_eager -name '*kernel_stats.csv' | head -1) 6
echo done
