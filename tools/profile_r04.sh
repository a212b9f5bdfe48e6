#!/bin/bash
# Round-4 profile on the GPU box (repo root): rocprofv3 kernel-trace stats of the headline (the
# bench's 16-scene eager roofline launches, and the calibrated multi-stream mode), separate PMC
# passes per counter group for the 16-scene headline, the cost volume at its four bench shapes
# (stats + PMC: MFMA busy), the secondary legs (tools/profile_legs.sh: config C / D / E, stats +
# PMC), then the JSON summaries the bench reads. (The GPU tests and the full bench run apart:
# tools/gpu_round.sh.)
# usage: bash tools/profile_r04.sh TAG
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
run stats_b16_eager 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats_b16_eager -o run -- \
  $B --steps 50 --warmup 5 --extra "" --batch 16 --launch eager
run stats_b16_hipgraph3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats_b16_hipgraph3 -o run -- \
  $B --steps 50 --warmup 5 --extra "" --batch 16 --launch hipgraph3
for pass in FETCH_SIZE WRITE_SIZE \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"; do
  n=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  run pmc_b16_$n 240 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $out/pmc_b16_$n -o run -- \
    $B --steps 10 --warmup 3 --eager --batch 16 --extra ""
done
python3 tools/pmc_summary.py --json $out/pmc_traffic_2v256x256x3b16.json 2v256x256x3b16 \
  "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ, $tag" $out/pmc_b16_fetch_size $out/pmc_b16_write_size \
  $out/pmc_b16_sq_waves
specs=""
for shp in config_a_32x32 config_b_scale0_64x64 config_d_scale0_56x96 config_d_scale1_112x192; do
  bash tools/prof_cv.sh ${tag}_$shp $shp > $out/cv_$shp.log 2>&1 || { echo "cv $shp failed"; tail -5 $out/cv_$shp.log; exit 1; }
  specs="$specs $shp=gpurun_out/prof_cv_${tag}_$shp"
done
python3 tools/cv_pmc_json.py $out/pmc_costvol.json "rocprofv3 --pmc (tools/profile_r03.sh, $tag), python tools/cv_case.py" $specs > /dev/null
bash tools/profile_legs.sh $tag train dl3dv recon12 > $out/legs.log 2>&1 || { echo "legs failed"; tail -5 $out/legs.log; exit 1; }
tail -3 $out/legs.log
echo done
