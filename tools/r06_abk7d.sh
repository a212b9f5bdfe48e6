#!/bin/bash
# K7 tile-wave vs sub-tile waves (DSPLAT_K7_SUBTILE=1) on the config-D DP training leg and config C.
# usage: bash tools/r06_abk7d.sh TAG
set -u
tag=${1:?tag}
mkdir -p gpurun_out
for r in 1 2; do
  for sub in "" 1; do
    DSPLAT_K7_SUBTILE=$sub timeout -k 10 300 python3 bench.py --skip-headline --no-cpu-baseline --extra train,train_d \
      --extra-steps 10 --detail= > gpurun_out/abk7d_${tag}_${sub:-tw}_$r.log 2>&1 || { echo "failed"; tail -3 gpurun_out/abk7d_${tag}_${sub:-tw}_$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], 'C ms', d['train_config_c']['ms_per_step'], 'k7', d['train_config_c']['roofline']['per_step_ms_by_kernel']['k_render_bwd'], 'D DP ms', d['train_config_d_dp']['ms_per_step'])" gpurun_out/abk7d_${tag}_${sub:-tw}_$r.log ${sub:-tw}
  done
done
