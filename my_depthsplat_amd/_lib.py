"""ctypes binding of libdsplat_hip.so (C ABI declared in include/dsplat_hip.h).

The product path has NO CPU fallback: if the HIP library is missing or no GPU is
visible, every op raises. torch is imported first so that the HIP runtime the
library links (libamdhip64.so.7) resolves to the one torch already loaded, and
the library shares torch's streams and device allocations.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_uint32, c_void_p
from pathlib import Path

import torch  # noqa: F401  (must be loaded before the HIP library)

# (DSPLAT_LIB: another build of the same ABI, e.g. a tools/ab_build.py A/B variant)
LIB_PATH = Path(os.environ.get("DSPLAT_LIB") or Path(__file__).resolve().parent / "lib" / "libdsplat_hip.so")

# name -> (restype, argtypes); mirrors include/dsplat_hip.h exactly.
_P = c_void_p
_I = c_int
SIGNATURES: dict[str, tuple] = {
    "dsr_build_cameras": (_I, [_I, _P, _P, _P, _P, _P, _P, _I, _P, _P, c_uint32, _P]),
    "dsr_preprocess_fwd": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "dsr_bin_scan": (_I, [_I, _I, _I, _P, _P, _P, _P, _P]),
    "dsr_bin_scatter": (_I, [_I, _I, _I, _I, _P, _P, _P, _I, _P]),
    "dsr_project_bin": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "dsr_cut_superblock": (_I, [_I, _I]),
    "dsr_preprocess_cut": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I,
                                _P]),
    "dsr_bin_cutoff": (_I, [_I, _I, _I, _P, c_uint32, _P, _P]),
    "dsr_bin_scatter_cut": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, ctypes.c_uint64, _P]),
    "dsr_survivor_layout": (_I, [_I, _I, _P, _P]),
    "dsr_project_survivors": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I,
                                   _P]),
    "dsr_bin_sort": (_I, [_I, _I, _I, _I, _P, _P, c_uint32, _P, _P, c_uint32, _P, c_uint32, _P, _P, _P]),
    "dsr_bin_sort_workspace_size": (ctypes.c_size_t, [_I, _I, _I, c_uint32]),
    "dsr_workspace_size": (_I, [_I, _I, _I, _I, ctypes.c_uint64, _P]),
    "dsr_sort_lds_capacity": (c_uint32, []),
    "dsr_render_fwd": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, c_uint32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "dsr_sort_render": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, c_uint32, _P, _P, _P, _I, _I, c_uint32, _I, _P, _P, _P,
                            _P, _P]),
    "dsr_project_bin_cameras": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P,
                                     _P, _P, _P, _P, _P, c_uint32, _I, _P]),
    "dsr_grad_scale": (_I, [_I, _I, _I, _P, _P, _P]),
    "dsr_render_bwd": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, c_uint32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "dsr_dgeom_to_float": (_I, [_I, _I, _P, _P, _P, _P, _P, _P]),
    "dsr_preprocess_bwd": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "dsr_head_bwd": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, c_float, c_float, _P, _I, _I, _P, _P, _P, _P, _P,
                          _P, _P, _P, _P, _P]),
    "dcv_cost_volume_workspace_size": (ctypes.c_size_t, [_I, _I, _I, _I, _I]),
    "dcv_cost_volume_bwd_workspace_size": (ctypes.c_size_t, [_I, _I, _I, _I, _I]),
    "dcv_cost_volume_path": (_I, [_I, _I, _I, _I, _I]),
    "dcv_cost_volume_bwd_shape": (_I, [_I, _I, _I, _I, _I, _I, _P, _P]),
    "dcv_cost_volume_fwd": (_I, [_I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, c_float, _P, _P, _P]),
    "dcv_cost_volume_bwd": (_I, [_I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, c_float, _P, _P,
                                 _P, _P, _P]),
    "dcv_cost_volume_views_workspace_size": (ctypes.c_size_t, [_I, _I, _I, _I, _I]),
    "dcv_cost_volume_views_bwd_workspace_size": (ctypes.c_size_t, [_I, _I, _I, _I, _I]),
    "dcv_cost_volume_views_fwd": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, c_float, _P, _P, _P]),
    "dcv_cost_volume_views_bwd": (_I, [_I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, c_float, _P, _P, _P,
                                       _P]),
    "dcv_warp_fwd": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, c_float, _P, _P]),
    "dcv_warp_bwd": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, c_float, _P, _P]),
    "dga_adapter_cameras": (_I, [_I, _P, _P, _I, _P, _P, _P]),
    "dga_head_rows": (_I, [_I, _I, _I, _I, _I, _P, _P, _P]),
    "dga_head_rows_bwd": (_I, [_I, _I, _I, _I, _I, _P, _P, _P]),
    "dga_adapter_fwd": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, c_float, c_float, _P, _P, _P, _P, _P, _P]),
    "dga_adapter_bwd": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, c_float, c_float, _P, _P, _P, _P, _P, _P, _P,
                             _P]),
    "dga_adapter_forward": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, c_float, c_float, _P, c_float, _P, _P, _P,
                                 _P, _P, _P]),
    "dga_adapter_backward": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, c_float, c_float, _P, c_float, _P, _P, _P,
                                  _P, _P, _P, _P, _P, _P]),
    "dls_loss_workspace_size": (ctypes.c_size_t, [_I, ctypes.c_int64]),
    "dls_l1_mse_psnr": (_I, [_I, ctypes.c_int64, _P, _P, c_float, c_float, _P, _P, _P, _P, _P]),
    "dsplat_last_error": (ctypes.c_char_p, []),
    "dsplat_abi_version": (_I, []),
}

class Workspace(ctypes.Structure):
    """dsr_workspace (include/dsplat_hip.h): bytes of every caller-owned buffer."""
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "cams_bytes", "geom_bytes", "radii_bytes", "seg_count_bytes", "seg_start_bytes", "keys_bytes",
        "scratch_bytes", "sort_ws_bytes", "color_bytes", "final_T_bytes", "n_contrib_bytes", "dgeom_bytes",
        "total_bytes")] + [("tiles", ctypes.c_int32), ("fixed_capacity", ctypes.c_int32)]


_lib = None


class DsplatError(RuntimeError):
    pass


def load(path: Path | str | None = None) -> ctypes.CDLL:
    """Load (once) and type the HIP library. Raises if it is missing or incomplete."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise DsplatError(
            f"HIP extension not built: {p} is missing. Run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(str(p), mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError here = ABI drift between header and .so
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = load().dsplat_last_error().decode(errors="replace")
        raise DsplatError(f"{what} failed (status {status}): {msg}")


def require_gpu(*tensors: torch.Tensor) -> None:
    """The product path runs only on the GPU; CPU tensors are an error, not a fallback."""
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise DsplatError("my_depthsplat_amd ops need device (HIP) tensors; got a CPU tensor. "
                              "There is no CPU fallback (the CPU restatement in oracle/ is test-only).")


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def stream_of(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream
