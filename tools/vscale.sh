set -u
mkdir -p gpurun_out/vscale
for v in 1 3 6; do
  timeout -k 10 200 python -u bench.py --batch 16 --launch eager --views $v --steps 100 --warmup 10 --extra "" --no-cpu-baseline --no-reference-binning > gpurun_out/vscale/v$v.log 2>&1 || exit 1
  python - $v gpurun_out/vscale/v$v.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l); r = d['roofline']
        print('views', sys.argv[1], 'ms', d['ms_per_step'], 'probe', r['per_kernel_avg_ms_probe'], 'N', d['config']['num_rendered_per_step'])
PY
done
