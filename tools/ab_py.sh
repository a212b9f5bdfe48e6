#!/bin/bash
# Same-box A/B of a host-side (Python) change on the config D / E legs: the tree as sent vs a
# copy with OLD_FILE put back at PKG_PATH. usage: bash tools/ab_py.sh TAG OLD_FILE PKG_PATH
set -u
TAG=${1:?tag}; OLD=${2:?old file}; DST=${3:?package path}
mkdir -p gpurun_out
rm -rf /tmp/ab_old && cp -r "$PWD" /tmp/ab_old && cp "$OLD" "/tmp/ab_old/$DST"
out=$PWD/gpurun_out/abpy_${TAG}.log; : > $out
for round in 1 2; do
  for tree in new old; do
    d=$PWD; [ $tree = old ] && d=/tmp/ab_old
    (cd $d && timeout -k 10 300 python -u bench.py --skip-headline --extra dl3dv,recon12 --no-cpu-baseline) \
      > gpurun_out/abpy_${TAG}_${tree}.log 2>&1 || { echo "$tree failed"; tail -5 gpurun_out/abpy_${TAG}_${tree}.log; exit 1; }
    python - $tree gpurun_out/abpy_${TAG}_${tree}.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)
        rd, re = d.get('render_config_d', {}), d.get('recon_config_e', {})
        print(sys.argv[1], '| D', rd.get('ms_per_step'), (rd.get('roofline') or {}).get('per_step_ms_by_kernel'), '| E', re.get('ms_per_scene'), (re.get('roofline') or {}).get('per_step_ms_by_kernel'))
PY
  done
done
cat $out
