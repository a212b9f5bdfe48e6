#!/bin/bash
# Round-4 profile of the secondary bench legs (config C training step, config D 6-view 448x768
# render, config E 12-view 512x960 reconstruction): per leg a rocprofv3 kernel-trace --stats pass
# and separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ group), each running ONLY that leg
# (bench.py --skip-headline), then the JSON summaries bench.py reads for the legs' roofline
# traffic / VALU issue (profiles/pmc_traffic_<workload>.json).
# usage (GPU box, repo root): bash tools/profile_legs.sh TAG [leg ...]   (legs: train dl3dv recon12)
set -u
tag=${1:?tag}; shift
legs=("$@"); [ ${#legs[@]} -eq 0 ] && legs=(train dl3dv recon12)
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
run() {  # run NAME TIMEOUT CMD...: stop the whole script on a timeout / signal / crash
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/$name.log; echo "stopping after $name"; exit $rc; fi
}
declare -A WL=([train]=train_c_2v256x256b16x4 [dl3dv]=render_d_6v448x768x8 [recon12]=recon_e_12v512x960x100c10)
for leg in "${legs[@]}"; do
  B="python3 bench.py --skip-headline --no-cpu-baseline --extra $leg --extra-steps 2"
  run ${leg}_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${leg}_stats -o run -- $B
  dirs=""
  for pass in FETCH_SIZE WRITE_SIZE \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"; do
    n=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    run ${leg}_pmc_$n 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $out/${leg}_pmc_$n -o run -- $B
    dirs="$dirs $out/${leg}_pmc_$n"
  done
  python3 tools/pmc_summary.py --json $out/pmc_traffic_${WL[$leg]}.json ${WL[$leg]} \
    "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ (tools/profile_legs.sh, $tag)" $dirs
done
echo done
