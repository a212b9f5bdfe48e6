"""Config B throughput with scenes batched into one decoder call (B scenes x 3 views per
launch pair) vs one scene per call, each replayed as hipGraphs on 1..4 streams (GPU box).
usage: python tools/batch_exp.py [steps] [B,B,...]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from my_depthsplat_amd import _lib  # noqa: E402
from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg  # noqa: E402
from my_depthsplat_amd.graphs import GraphedCall  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda:0")
_lib.load()
dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(dev)


def call_of(sc):
    def f():
        with torch.no_grad():
            return dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, (256, 256))
    return f


def bench(fns, n, nstreams):
    graphs = [GraphedCall(f, warmup=2) for f in fns]
    lanes = [torch.cuda.Stream(device=dev) for _ in graphs]
    for _ in range(3):
        for g, s in zip(graphs, lanes):
            with torch.cuda.stream(s):
                g()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        k = i % nstreams
        with torch.cuda.stream(lanes[k]):
            graphs[k]()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


for B in [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "2", "4"])]:
    scs = [make_scene(batch=B, n_context=2, n_targets=3, height=256, width=256, seed=1000 + 16 * i, device=dev)
           for i in range(4)]
    for ns in (1, 2, 4):
        t = bench([call_of(s) for s in scs[:ns]], steps, ns)
        print(f"B={B} streams={ns}: {t * 1e6:8.1f} us per call, {t * 1e6 / B:7.1f} us per scene, "
              f"{3 * B / t:9.0f} views/s", flush=True)
