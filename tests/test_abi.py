"""The C-ABI library loads without a GPU and exports exactly what include/dsplat_hip.h
declares; the ctypes signature table matches the header's parameter counts."""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "dsplat_hip.h"


def header_functions():
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:const\s+)?\w+\s*\*?\s*(\w+)\s*\(([^;]*?)\)\s*;", txt, flags=re.M | re.S):
        name, args = m.group(1), m.group(2).strip()
        n = 0 if args in ("", "void") else len([a for a in args.split(",") if a.strip()])
        out[name] = n
    return out


def test_header_parses():
    fns = header_functions()
    assert {"dsr_preprocess_fwd", "dsr_render_fwd", "dsr_render_bwd", "dsr_preprocess_bwd",
            "dcv_cost_volume_fwd", "dcv_cost_volume_bwd", "dsplat_last_error"} <= set(fns)


def test_library_exports_every_header_symbol():
    from my_depthsplat_amd import _lib
    lib_path = _lib.LIB_PATH
    if not lib_path.exists():
        pytest.skip("extension not built (run __graft_entry__.build())")
    nm = subprocess.run(["nm", "-D", "--defined-only", str(lib_path)], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if " T " in ln}
    missing = set(header_functions()) - exported
    assert not missing, missing


def test_ctypes_table_matches_header():
    from my_depthsplat_amd import _lib
    fns = header_functions()
    assert set(_lib.SIGNATURES) == set(fns)
    for name, (_, args) in _lib.SIGNATURES.items():
        assert len(args) == fns[name], (name, len(args), fns[name])


def test_load_without_gpu_and_error_channel():
    from my_depthsplat_amd import _lib
    if not _lib.LIB_PATH.exists():
        pytest.skip("extension not built")
    lib = _lib.load()
    assert lib.dsplat_abi_version() == 20
    assert lib.dsr_sort_lds_capacity() >= 256
    # argument validation happens before any HIP call -> works on a GPU-less host
    rc = lib.dsr_render_fwd(0, 1, 8, 8, None, None, None, None, 0, None, None, None, None, None, None, None, None)
    assert rc == 1 and b"bad sizes" in lib.dsplat_last_error()
    with pytest.raises(_lib.DsplatError):
        _lib.check(rc, "dsr_render_fwd")


def test_cpu_tensors_fail_loudly():
    import torch

    from my_depthsplat_amd import _lib, raster
    if not _lib.LIB_PATH.exists():
        pytest.skip("extension not built")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    cams = torch.zeros(1, raster.CAM_FLOATS)
    with pytest.raises(_lib.DsplatError):
        raster.rasterize_views(torch.zeros(1, 4, 3), torch.zeros(1, 4, 1, 3), torch.zeros(1, 4),
                               torch.zeros(1, 4, 6), cams, [0], use_sh=True, sh_degree=0, image_height=8,
                               image_width=8)


def test_head_rows_validation_without_gpu():
    """dga_head_rows / _bwd reject bad sizes, null pointers and tiles above the LDS budget
    before any HIP call (GPU-less host)."""
    from my_depthsplat_amd import _lib
    if not _lib.LIB_PATH.exists():
        pytest.skip("extension not built")
    lib = _lib.load()
    assert lib.dga_head_rows(0, 37, 8, 7, 12, None, None, None) == 1
    assert b"bad sizes" in lib.dsplat_last_error()
    assert lib.dga_head_rows(1, 37, 8, 7, 12, None, None, None) == 1
    assert b"null pointer" in lib.dsplat_last_error()
    x = ctypes.create_string_buffer(16)
    assert lib.dga_head_rows_bwd(1, 1000, 8, 2, 2, x, x, None) == 1  # 16 * 8 * 1001 * 4 B > 64 KiB
    assert b"LDS tile" in lib.dsplat_last_error()


def test_head_rows_rejects_mismatched_shapes_without_gpu():
    """the head-rows autograd function checks x against (C, r) before any pointer
    reaches the kernel (wrong channel count, rank or dtype raise ValueError, on any device)."""
    import pytest
    import torch
    from my_depthsplat_amd.training import _HeadRows
    for x in (torch.zeros(2, 5, 3, 3), torch.zeros(8, 3, 3), torch.zeros(2, 8, 3, 3, dtype=torch.float64)):
        with pytest.raises(ValueError):
            _HeadRows.apply(x, 2, 2)
