#!/bin/bash
# Config C / D training legs only (no tests): per-kernel ms per step.
# usage: bash tools/r06_trainleg.sh TAG [legs]
set -u
tag=${1:?tag}; legs=${2:-train,train_d}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --skip-headline --no-cpu-baseline --extra $legs --extra-steps 10 --detail= \
  > gpurun_out/trainleg_$tag.log 2>&1 || { echo "legs failed"; tail -5 gpurun_out/trainleg_$tag.log; exit 1; }
python3 - gpurun_out/trainleg_$tag.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
if "train_config_c" in d:
    c = d["train_config_c"]
    print("config C ms", c["ms_per_step"], json.dumps(c["roofline"]["per_step_ms_by_kernel"]))
if "train_config_d_dp" in d:
    print("config D DP ms", d["train_config_d_dp"]["ms_per_step"])
PY
