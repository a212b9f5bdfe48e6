"""Multi-process data-parallel helpers on CPU with gloo (world_size 2)."""
from __future__ import annotations

import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from my_depthsplat_amd.parallel import allreduce_gradients, reduce_max, shard


def test_shard_covers_everything():
    for n in (0, 1, 7, 16, 33):
        for w in (1, 2, 3, 8):
            parts = [shard(n, r, w) for r in range(w)]
            assert [i for p in parts for i in p] == list(range(n))
            assert max(len(p) for p in parts) - min(len(p) for p in parts) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(rank)
    lin = torch.nn.Linear(5, 3)
    extra = torch.nn.Parameter(torch.zeros(4))  # no grad on this rank -> contributes zeros
    x = torch.randn(8, 5)
    lin(x).square().sum().backward()
    if rank == 0:
        extra.grad = torch.ones(4)
    before = [p.grad.clone() for p in lin.parameters()]
    nbytes = allreduce_gradients(list(lin.parameters()) + [extra])
    t = reduce_max(float(rank + 1))
    q.put((rank, [b.numpy() for b in before], [p.grad.numpy() for p in lin.parameters()], extra.grad.numpy(),
           nbytes, t))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_gradients_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, b0, a0, e0, n0, t0), (_, b1, a1, e1, n1, t1) = res
    for x0, x1, y0, y1 in zip(b0, b1, a0, a1):
        avg = (x0 + x1) / 2
        assert abs(y0 - avg).max() < 1e-6 and abs(y1 - avg).max() < 1e-6
    assert (e0 == 0.5).all() and (e1 == 0.5).all()
    assert n0 == n1 == (15 + 3 + 4) * 4
    assert t0 == t1 == 2.0


# ---------------------------------------------------------------- the data-parallel training step

def _dense_render(gs, ext, K, near, far, image_shape):
    """Decoder-signature renderer on the dense torch restatement (tests/dense_raster.py):
    the per-scene Gaussians seen from each target view, reference camera set-up."""
    from dense_raster import render

    from my_depthsplat_amd.cuda_splatting import _cov6, camera_settings
    B, v = ext.shape[:2]
    H, W = image_shape
    out = []
    for b in range(B):
        st = camera_settings(ext[b], K[b], near[b], far[b])
        views = []
        for j in range(v):
            s = st["scale"][j]
            views.append(render(gs.means[b] * s, gs.harmonics[b].transpose(-1, -2), gs.opacities[b],
                                _cov6(gs.covariances[b]) * s * s, st["viewmatrix"][j].reshape(-1),
                                st["projmatrix"][j].reshape(-1), st["campos"][j], float(st["tanfovx"][j]),
                                float(st["tanfovy"][j]), torch.zeros(3), H, W))
        out.append(torch.stack(views))
    return torch.stack(out)


def _train_setup(seed_batch=5):
    from my_depthsplat_amd.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg
    from my_depthsplat_amd.training import GaussianHead, synthetic_batch
    adapter = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, 1))
    torch.manual_seed(0)  # identical head initialisation on every rank
    head = GaussianHead(3 + adapter.d_in, width=8, down=4)
    batch = synthetic_batch(4, 2, 1, 16, 16, seed=seed_batch)
    return adapter, head, batch


def _train_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from my_depthsplat_amd.training import TrainStep, rank_batch, torch_l1_mse
    adapter, head, batch = _train_setup()
    mine = rank_batch(batch, rank, world)
    step = TrainStep(head, adapter, _dense_render, torch_l1_mse, lr=1e-3, world=world)
    loss = step.forward_backward(mine)
    nbytes = allreduce_gradients(list(head.parameters()), world)
    grads = [p.grad.clone().numpy() for p in head.parameters()]
    step.opt.zero_grad(set_to_none=True)
    step(mine)  # full step: all-reduce, clip, AdamW
    params = [p.detach().clone().numpy() for p in head.parameters()]
    q.put((rank, mine.n_scenes, float(loss), grads, params, nbytes))
    dist.barrier()
    dist.destroy_process_group()


def test_training_step_gloo_world2_matches_full_batch():
    """world 2 (gloo): each rank takes its half of a 4-scene batch (parallel.shard), runs head
    -> adapter -> dense rasterizer -> loss -> backward and ONE bucketed all-reduce. The
    averaged gradient equals the single-process gradient of the whole batch, and after the
    optimizer step both ranks hold identical parameters."""
    from my_depthsplat_amd.training import TrainStep, torch_l1_mse
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, n0, l0, g0, p0, b0), (_, n1, l1, g1, p1, b1) = res
    assert n0 == n1 == 2
    adapter, head, batch = _train_setup()
    assert b0 == b1 == 4 * sum(p.numel() for p in head.parameters())
    TrainStep(head, adapter, _dense_render, torch_l1_mse, world=1).forward_backward(batch)
    for a, b, ref in zip(g0, g1, [p.grad.numpy() for p in head.parameters()]):
        assert abs(a - b).max() == 0
        assert abs(a - ref).max() <= 1e-4 * (abs(ref).max() + 1e-12) + 1e-7
    for a, b in zip(p0, p1):
        assert (a == b).all()
    assert abs((l0 + l1) / 2) > 0


# ---------------------------------------------------------------- single-scene view split

class _DenseDecoder:
    """Decoder-signature stub over the dense torch renderer (returns DecoderOutput)."""

    def __call__(self, gs, ext, K, near, far, image_shape, depth_mode=None):
        from my_depthsplat_amd.decoder import DecoderOutput
        return DecoderOutput(_dense_render(gs, ext, K, near, far, image_shape), None)


def _split_scene():
    from my_depthsplat_amd.synthetic import make_scene
    return make_scene(batch=1, n_context=2, n_targets=7, height=12, width=20, seed=31, device="cpu")


def _split_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from my_depthsplat_amd.parallel import render_view_split
    sc = _split_scene()
    color = render_view_split(_DenseDecoder(), sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near,
                              sc.far, sc.image_shape, 2, rank, world)
    q.put((rank, color.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_view_split_gloo_world2_matches_one_rank():
    """One scene, 7 target views split 4 / 3 over 2 gloo ranks (Gaussians replicated), each rank
    rendering its share in chunks of 2, then the all-gather: every rank ends with exactly the
    images of the one-rank chunked render (render_chunked over all 7 views)."""
    from my_depthsplat_amd.decoder import render_chunked
    sc = _split_scene()
    want = render_chunked(_DenseDecoder(), sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near,
                          sc.far, sc.image_shape, 2).color.numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, got in res:
        assert got.shape == want.shape == (1, 7, 3, 12, 20)
        assert (got == want).all()
