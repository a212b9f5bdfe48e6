"""Round-6 overlap experiment: can k_sort_render of one batch share the chip with
k_project_emit of the next? The r06a hipgraph7 trace shows the lanes phase-lock (project_emit
kernels run with each other, sort_render kernels with each other, 97 % of the time). Here two
lanes (own decoders, own scenes, B = 16) run eagerly:
  serial  one stream
  free    two streams, no ordering between them
  chain   two streams, each lane's project_emit waits for the other lane's previous
          project_emit (an event recorded right after it): every sort_render is issued while the
          other lane's project_emit runs
usage: python tools/pipe_exp.py [steps]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from my_depthsplat_amd import raster  # noqa: E402
from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda:0")
B, H = 16, 256
decs = [DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(dev)
        for _ in range(2)]
scs = [make_scene(batch=B, n_context=2, n_targets=3, height=H, width=H, seed=500 + i, device=dev) for i in range(2)]
streams = [torch.cuda.Stream(device=dev) for _ in range(2)]


def call(i):
    s = scs[i]
    with torch.no_grad():
        return decs[i](s.gaussians, s.target_extrinsics, s.target_intrinsics, s.near, s.far, (H, H))


class Chain:
    """After a lane's k_project_emit launch: the OTHER lane's stream waits for it."""
    def __init__(self):
        self.lane = 0

    def start(self, name):
        return name

    def stop(self, tok):
        if tok == "k_project_emit":
            e = torch.cuda.Event()
            e.record(streams[self.lane])
            streams[1 - self.lane].wait_event(e)


def run(mode, n):
    chain = Chain() if mode == "chain" else None
    raster.set_timer(chain)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(n):
        i = k % 2
        if mode == "serial":
            call(i)
        else:
            if chain:
                chain.lane = i
            with torch.cuda.stream(streams[i]):
                call(i)
    torch.cuda.synchronize()
    raster.set_timer(None)
    return (time.perf_counter() - t0) / n * 1e3


ref = [call(i).color.clone() for i in range(2)]
for mode in ["serial", "free", "chain"] * 2:
    run(mode, 10)
    ms = run(mode, steps)
    print(f"{mode:7s} {ms:.4f} ms/step  {B * 3 / ms * 1e3:9.0f} views/s", flush=True)
torch.cuda.synchronize()
for i in range(2):
    assert torch.equal(call(i).color, ref[i])
print("images unchanged")
