#!/bin/bash
# Round-2 profile on the GPU box (repo root): GPU tests, kernel-trace stats of the bench (the
# calibrated headline configuration: 4 scenes per step on 4 streams, and one scene per step on
# one graph), separate PMC passes per counter group for the headline (exact binning only, one
# and four scenes per launch), the config C training step, the config E reconstruction and
# the cost volume, then JSON summaries.
# usage: bash tools/profile_legs2.sh TAG  (second half of tools/profile_r02.sh)
set -u
tag=${1:?tag}
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
run() {  # run NAME TIMEOUT CMD...: stop the whole script on a timeout / signal / crash
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit $rc; fi
}
B="python3 bench.py --no-cpu-baseline --no-reference-binning"
export DSPLAT_PARITY_REPORT=$out/parity.jsonl
# config C training step and config E reconstruction (the headline runs too, 3 steps)
for leg in train recon12; do
  for pass in FETCH_SIZE WRITE_SIZE \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"; do
    n=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    run ${leg}_$n 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $out/${leg}_$n -o run -- \
      $B --steps 3 --warmup 2 --eager --batch 1 --extra $leg --extra-steps 3
  done
  python3 tools/pmc_summary.py --json $out/pmc_$leg.json $leg "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ, $tag" \
    $out/${leg}_fetch_size $out/${leg}_write_size $out/${leg}_sq_waves
done
run stats_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats_train -o run -- \
  $B --steps 5 --warmup 2 --batch 1 --launch hipgraph --extra train --extra-steps 10
# cost volume, per shape (config A and config B scale 0, the bench's costvol leg)
for shp in a b0; do
  run cv_stats_$shp 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cv_stats_$shp -o run -- \
    python3 tools/cv_bench.py $shp
  run cv_sq_$shp 240 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/cv_sq_$shp -o run -- \
    python3 tools/cv_bench.py $shp
  run cv_fetch_$shp 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/cv_fetch_$shp -o run -- \
    python3 tools/cv_bench.py $shp
  python3 tools/pmc_summary.py $out/cv_sq_$shp $out/cv_fetch_$shp > $out/pmc_costvol_$shp.json
done
echo done
