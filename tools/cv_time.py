"""Time the bench's cost-volume shapes (bench.costvol_leg, no CPU sample) on cuda:0 and print
one line per shape. usage: python tools/cv_time.py"""
import json
import sys
import types
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402

args = types.SimpleNamespace(no_cpu_baseline=True)
res = bench.costvol_leg(args, torch.device("cuda:0"), 0, 1, lambda *v: v)
for k, v in res.items():
    if k == "note":
        continue
    s = v["shape"]
    print(f"{k:26s} BV={s['BV']:2d} J={s['J']} C={s['C']:3d} {s['H']}x{s['W']} D={s['D']:3d} | fwd "
          f"{v['ms_per_call'] * 1e3:8.1f} us {v['tflops']:6.2f} TF frac {v['frac']:.4f} | fwd+bwd "
          f"{v['ms_fwd_bwd'] * 1e3:9.1f} us {v['tflops_fwd_bwd']:6.2f} TF")
print(json.dumps(res))
