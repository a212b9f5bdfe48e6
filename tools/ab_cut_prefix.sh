#!/bin/bash
# Same-box A/B of the depth cut's per-tile prefix (DSPLAT_CUT_PREFIX) on the config D / E legs.
# usage: bash tools/ab_cut_prefix.sh TAG PREFIX...
set -u
TAG=${1:?tag}; shift
mkdir -p gpurun_out
out=gpurun_out/abcp_${TAG}.log; : > $out
for round in 1 2; do
  for pf in "$@"; do
    DSPLAT_CUT_PREFIX=$pf timeout -k 10 300 python -u bench.py --skip-headline --extra dl3dv,recon12 --no-cpu-baseline \
      > gpurun_out/abcp_${TAG}_${pf}.log 2>&1 || { echo "$pf failed"; tail -5 gpurun_out/abcp_${TAG}_${pf}.log; exit 1; }
    python - $pf gpurun_out/abcp_${TAG}_${pf}.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)
        rd, re = d.get('render_config_d', {}), d.get('recon_config_e', {})
        print('prefix', sys.argv[1], '| D', rd.get('ms_per_step'), (rd.get('roofline') or {}).get('per_step_ms_by_kernel'), '| E', re.get('ms_per_scene'), (re.get('roofline') or {}).get('per_step_ms_by_kernel'))
PY
  done
done
cat $out
