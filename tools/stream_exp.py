"""Experiment: 3 views in one launch sequence vs one view per stream (hipGraph-captured)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from my_depthsplat_amd import raster  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402

dev = torch.device("cuda:0")
H = W = 256
sc = make_scene(batch=1, n_context=2, n_targets=3, height=H, width=W, seed=1000, device=dev)
g = sc.gaussians
bg = torch.zeros(3, 3, device=dev)
cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg, [0] * 3, True)
cam1 = [cams[i:i + 1].contiguous() for i in range(3)]
layout = raster.input_layout(g.harmonics, g.covariances, True, True)


def one():
    return raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, cams, 3, H, W, layout)[0]


streams = [torch.cuda.Stream() for _ in range(3)]


def split():
    cur = torch.cuda.current_stream()
    outs = []
    ev = torch.cuda.Event()
    ev.record(cur)
    for i, s in enumerate(streams):
        s.wait_event(ev)
        with torch.cuda.stream(s):
            outs.append(raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, cam1[i], 1,
                                           H, W, layout)[0])
    for s in streams:
        e = torch.cuda.Event()
        e.record(s)
        cur.wait_event(e)
    return outs


def timeit(fn, n=100):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def graphed(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        fn()
    return lambda: gr.replay()


print(f"eager 3-view launch: {timeit(one):.1f} us   eager 3 streams x 1 view: {timeit(split):.1f} us", flush=True)
print(f"graph 3-view launch: {timeit(graphed(one)):.1f} us   graph 3 streams x 1 view: {timeit(graphed(split)):.1f} us",
      flush=True)
