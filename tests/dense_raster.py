"""Dense, differentiable torch restatement of the 3DGS forward (tiny scenes only), used to
check the oracle's forward AND backward through torch.autograd.

Same per-Gaussian math as SURVEY.md §8a A7/A9 (cull z <= 0.2, EWA with 1.3 tanfov clamp and
+0.3 dilation, conic, SH -> RGB + 0.5 clamped, alpha = min(0.99, o e^power), skip power > 0
or alpha < 1/255, stop at T(1-alpha) < 1e-4), with the tile-rect membership of each Gaussian
(from its radius) applied as a mask so the set of (pixel, Gaussian) pairs is identical.
Discrete decisions (culling, masks, sort order, termination) carry no gradient, as in the
upstream backward. float64 by default.
"""
from __future__ import annotations

import math

import torch

C0 = 0.28209479177387814
C1 = 0.4886025119029199
C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]


def sh_rgb(sh, d):  # sh [P, M, 3], d [P, 3] unit
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    deg = math.isqrt(sh.shape[1]) - 1
    r = C0 * sh[:, 0]
    if deg > 0:
        r = r - C1 * y * sh[:, 1] + C1 * z * sh[:, 2] - C1 * x * sh[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = r + C2[0] * xy * sh[:, 4] + C2[1] * yz * sh[:, 5] + C2[2] * (2 * zz - xx - yy) * sh[:, 6] + \
            C2[3] * xz * sh[:, 7] + C2[4] * (xx - yy) * sh[:, 8]
    return r + 0.5


def render(means, shs, opac, cov6, view, proj, campos, tanx, tany, bg, H, W, ndc_offset=None):
    """means [P,3], shs [P,M,3], opac [P], cov6 [P,6], view/proj [16] column-major,
    campos [3]. ndc_offset [P,2] (zeros, requires_grad) exposes d/d(ndc xy) = means2D grad."""
    dt = means.dtype
    V = view.reshape(4, 4).T  # column-major storage -> row-major world->camera
    Pm = proj.reshape(4, 4).T
    hom = torch.cat([means, torch.ones_like(means[:, :1])], 1)
    pv = hom @ V.T
    ph = hom @ Pm.T
    vis = (pv[:, 2] > 0.2).detach()
    ndc = ph[:, :2] / (ph[:, 3:4] + 1e-7)
    if ndc_offset is not None:
        ndc = ndc + ndc_offset
    pix = torch.stack([((ndc[:, 0] + 1) * W - 1) * 0.5, ((ndc[:, 1] + 1) * H - 1) * 0.5], 1)
    fx, fy = W / (2 * tanx), H / (2 * tany)
    t = pv[:, :3]
    limx, limy = 1.3 * tanx, 1.3 * tany
    tx = torch.clamp(t[:, 0] / t[:, 2], -limx, limx) * t[:, 2]
    ty = torch.clamp(t[:, 1] / t[:, 2], -limy, limy) * t[:, 2]
    tz = t[:, 2]
    zero = torch.zeros_like(tz)
    J = torch.stack([torch.stack([fx / tz, zero, -fx * tx / tz ** 2], 1),
                     torch.stack([zero, fy / tz, -fy * ty / tz ** 2], 1)], 1)  # [P, 2, 3]
    Tm = J @ V[:3, :3]
    S = torch.stack([torch.stack([cov6[:, 0], cov6[:, 1], cov6[:, 2]], 1),
                     torch.stack([cov6[:, 1], cov6[:, 3], cov6[:, 4]], 1),
                     torch.stack([cov6[:, 2], cov6[:, 4], cov6[:, 5]], 1)], 1)
    cov = Tm @ S @ Tm.transpose(1, 2) + 0.3 * torch.eye(2, dtype=dt)
    a, b, c = cov[:, 0, 0], cov[:, 0, 1], cov[:, 1, 1]
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], 1)
    mid = 0.5 * (a + c)
    lam = mid + torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
    radius = torch.ceil(3 * torch.sqrt(lam)).detach()
    d = means - campos
    d = d / d.norm(dim=1, keepdim=True)
    rgb = torch.clamp(sh_rgb(shs, d), min=0)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    px, py = pix[:, 0].detach(), pix[:, 1].detach()
    x0 = torch.clamp(torch.trunc((px - radius) / 16), 0, gx)
    y0 = torch.clamp(torch.trunc((py - radius) / 16), 0, gy)
    x1 = torch.clamp(torch.trunc((px + radius + 15) / 16), 0, gx)
    y1 = torch.clamp(torch.trunc((py + radius + 15) / 16), 0, gy)
    vis = vis & ((x1 - x0) * (y1 - y0) > 0)
    ys, xs = torch.meshgrid(torch.arange(H, dtype=dt), torch.arange(W, dtype=dt), indexing="ij")
    xs, ys = xs.reshape(-1), ys.reshape(-1)
    tile_x, tile_y = torch.floor(xs / 16), torch.floor(ys / 16)
    order = torch.argsort(pv[:, 2].detach(), stable=True)
    Tr = torch.ones(H * W, dtype=dt)
    Cc = torch.zeros(3, H * W, dtype=dt)
    done = torch.zeros(H * W, dtype=torch.bool)
    for i in order.tolist():
        if not bool(vis[i]):
            continue
        inrect = (tile_x >= x0[i]) & (tile_x < x1[i]) & (tile_y >= y0[i]) & (tile_y < y1[i])
        dx, dy = pix[i, 0] - xs, pix[i, 1] - ys
        power = -0.5 * (conic[i, 0] * dx * dx + conic[i, 2] * dy * dy) - conic[i, 1] * dx * dy
        alpha = torch.clamp(opac[i] * torch.exp(power), max=0.99)
        ok = inrect & (power <= 0).detach() & (alpha >= 1 / 255).detach() & ~done
        testT = Tr * (1 - alpha)
        stop = ok & (testT < 1e-4).detach()
        blend = ok & ~stop
        Cc = Cc + torch.where(blend, rgb[i][:, None] * alpha * Tr, torch.zeros_like(Cc))
        Tr = torch.where(blend, testT, Tr)
        done = done | stop
    return (Cc + Tr * bg[:, None]).reshape(3, H, W)
