"""ctypes wrapper of the CPU rasterizer restatement (oracle/dsr_oracle.cpp).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). One call = one view, exactly the
upstream per-call granularity of cuda_splatting.py:112-123. numpy in, numpy out.
"""
from __future__ import annotations

import ctypes
import subprocess
from ctypes import c_float, c_int, c_void_p
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "libdsr_oracle.so"
_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
        lib = ctypes.CDLL(str(LIB))
        lib.orc_forward.restype = c_void_p
        lib.orc_forward.argtypes = [c_int, c_int, c_int, c_int, c_int] + [c_void_p] * 9 + [c_float, c_float]
        lib.orc_free.argtypes = [c_void_p]
        lib.orc_num_rendered.argtypes = [c_void_p]
        lib.orc_num_tiles.argtypes = [c_void_p]
        lib.orc_get_image.argtypes = [c_void_p] * 4
        lib.orc_get_geom.argtypes = [c_void_p] * 8
        lib.orc_get_binning.argtypes = [c_void_p] * 4
        lib.orc_backward.argtypes = [c_void_p] * 9
        lib.orc_backward_f64.argtypes = [c_void_p] * 9
        lib.orc_conic_grad.argtypes = [ctypes.c_double] * 3 + [c_void_p, c_int, c_void_p]
        _lib = lib
    return _lib


def _f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def _p(a):
    return None if a is None else a.ctypes.data_as(c_void_p)


class View:
    """Forward state of one rendered view (owns the C++ state until close())."""

    def __init__(self, means, shs, colors, opacities, cov6, viewmatrix, projmatrix, campos, tanfovx, tanfovy,
                 bg, H, W, sh_degree):
        lib = load()
        self.means, self.shs, self.colors = _f32(means), _f32(shs), _f32(colors)
        self.opac, self.cov6 = _f32(opacities).reshape(-1), _f32(cov6)
        self.view, self.proj = _f32(viewmatrix).reshape(16), _f32(projmatrix).reshape(16)
        self.campos, self.bg = _f32(campos).reshape(3), _f32(bg).reshape(3)
        self.P = self.means.shape[0]
        self.M = 0 if self.shs is None else self.shs.reshape(self.P, -1, 3).shape[1]
        self.H, self.W = int(H), int(W)
        self.h = lib.orc_forward(self.P, int(sh_degree), self.M, self.W, self.H, _p(self.bg), _p(self.means),
                                 _p(self.shs), _p(self.colors), _p(self.opac), _p(self.cov6), _p(self.view),
                                 _p(self.proj), _p(self.campos), float(tanfovx), float(tanfovy))
        self.num_rendered = lib.orc_num_rendered(self.h)
        self.num_tiles = lib.orc_num_tiles(self.h)

    def image(self):
        c = np.empty((3, self.H, self.W), np.float32)
        t = np.empty((self.H, self.W), np.float32)
        n = np.empty((self.H, self.W), np.uint32)
        load().orc_get_image(self.h, _p(c), _p(t), _p(n))
        return c, t, n

    def geom(self):
        P = self.P
        out = dict(depth=np.empty(P, np.float32), radii=np.empty(P, np.int32), xy=np.empty((P, 2), np.float32),
                   conic_opacity=np.empty((P, 4), np.float32), rgb=np.empty((P, 3), np.float32),
                   tiles_touched=np.empty(P, np.uint32), clamped=np.empty((P, 3), np.uint8))
        load().orc_get_geom(self.h, *[_p(out[k]) for k in
                                      ("depth", "radii", "xy", "conic_opacity", "rgb", "tiles_touched", "clamped")])
        return out

    def binning(self):
        N = self.num_rendered
        keys = np.empty(max(N, 1), np.uint64)
        vals = np.empty(max(N, 1), np.uint32)
        ranges = np.empty((self.num_tiles, 2), np.uint32)
        load().orc_get_binning(self.h, _p(keys), _p(vals), _p(ranges))
        return keys[:N], vals[:N], ranges

    def backward(self, dL_dpix, f64: bool = False):
        """Gradients of this view. f64: the same backward evaluated in double (which entries
        blend still decided in float, as the forward did): the high-precision reference."""
        P, M = self.P, self.M
        d = np.ascontiguousarray(dL_dpix, dtype=np.float32).reshape(3, self.H, self.W)
        out = dict(dmean2D=np.empty((P, 3), np.float32), dconic=np.empty((P, 3), np.float32),
                   dopacity=np.empty(P, np.float32), dcolor=np.empty((P, 3), np.float32),
                   dmean3D=np.empty((P, 3), np.float32), dcov6=np.empty((P, 6), np.float32),
                   dsh=np.empty((P, max(M, 1), 3), np.float32) if self.shs is not None else None)
        fn = load().orc_backward_f64 if f64 else load().orc_backward
        fn(self.h, _p(d), _p(out["dmean2D"]), _p(out["dconic"]), _p(out["dopacity"]),
                            _p(out["dcolor"]), _p(out["dmean3D"]), _p(out["dcov6"]), _p(out["dsh"]))
        return out

    def close(self):
        if self.h:
            load().orc_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_settings(means, shs, colors, opacities, cov6, st: dict, i: int, bg, H, W, sh_degree):
    """Render view i of a camera_settings() dict (the tensors render_cuda hands to the
    rasterizer), with Gaussians already rescaled by st['scale'][i] like the reference."""
    s = float(st["scale"][i])
    m = np.asarray(means, np.float32) * np.float32(s)
    c = np.asarray(cov6, np.float32) * np.float32(np.float32(s) * np.float32(s))
    return View(m, shs, colors, opacities, c, st["viewmatrix"][i], st["projmatrix"][i], st["campos"][i],
                float(st["tanfovx"][i]), float(st["tanfovy"][i]), bg, H, W, sh_degree)


def conic_grad(a: float, b: float, c: float, dconic, form: int) -> np.ndarray:
    """dL/d(a, b, c) of cov2D from dL/dconic (render-backward convention), in double: form 0
    the kernels' -S G S, form 1 upstream's denom2inv formula (orc_conic_grad)."""
    d = np.ascontiguousarray(dconic, np.float64)
    out = np.empty(3, np.float64)
    load().orc_conic_grad(float(a), float(b), float(c), d.ctypes.data, int(form), out.ctypes.data)
    return out
