set -u
mkdir -p gpurun_out
out=gpurun_out/abch_r05w.log; : > $out
for round in 1 2; do
  for h in 4096 3072 2048; do
    timeout -k 10 300 python -u tools/ab_cut_hint.py $h --skip-headline --extra dl3dv,recon12 --no-cpu-baseline > gpurun_out/abch_r05w_$h.log 2>&1 || { echo "$h failed"; tail -5 gpurun_out/abch_r05w_$h.log; exit 1; }
    python - $h gpurun_out/abch_r05w_$h.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)
        rd, re = d.get('render_config_d', {}), d.get('recon_config_e', {})
        print('hint', sys.argv[1], '| D', rd.get('ms_per_step'), (rd.get('roofline') or {}).get('per_step_ms_by_kernel'), '| E', re.get('ms_per_scene'), (re.get('roofline') or {}).get('per_step_ms_by_kernel'))
PY
  done
done
cat $out
