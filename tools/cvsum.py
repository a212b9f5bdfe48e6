"""Print the cost_volume leg of a bench log (last JSON line)."""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(line)
for k, v in d["cost_volume"].items():
    if k == "note":
        continue
    s = v["shape"]
    print(f"{k:26s} BV={s['BV']:2d} J={s['J']} C={s['C']:3d} {s['H']}x{s['W']} D={s['D']:3d} | fwd {v['ms_per_call']*1e3:8.1f} us "
          f"{v['tflops']:6.2f} TF frac {v['frac']:.4f} | fwd+bwd {v['ms_fwd_bwd']*1e3:9.1f} us {v['tflops_fwd_bwd']:6.2f} TF")
