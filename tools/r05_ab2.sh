#!/bin/bash
# Same-box A/B of library variants on the cost-volume leg and the config D / E legs.
# usage: bash tools/r05_ab2.sh TAG NAME...   (NAME = main or a lib/variants/libdsplat_NAME.so)
set -u
TAG=${1:?tag}; shift
mkdir -p gpurun_out
out=gpurun_out/ab2_${TAG}.log; : > $out
for round in 1 2; do
  for n in "$@"; do
    lib=""; [ "$n" != main ] && lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so
    DSPLAT_LIB=$lib timeout -k 10 300 python -u bench.py --skip-headline --extra costvol,dl3dv,recon12 --no-cpu-baseline \
      > gpurun_out/ab2_${TAG}_${n}.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab2_${TAG}_${n}.log; exit 1; }
    python - "$n" gpurun_out/ab2_${TAG}_${n}.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)
        cv = d.get('cost_volume', {})
        s = ' '.join(f"{k[:14]}: {v['ms_per_call']:.4f}/{v['ms_fwd_bwd']:.4f}" for k, v in cv.items() if isinstance(v, dict))
        rd, re = d.get('render_config_d', {}), d.get('recon_config_e', {})
        print(sys.argv[1], s, '| D', rd.get('ms_per_step'), '| E', re.get('ms_per_scene'),
              (re.get('roofline') or {}).get('per_step_ms_by_kernel', {}).get('k_preprocess_cut'))
PY
  done
done
cat $out
