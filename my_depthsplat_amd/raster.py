"""Batched differentiable rasterization through libdsplat_hip.so.

`rasterize_views` is the single entry the drop-in shims (rasterizer.py, cuda_splatting.py,
decoder.py) call: it renders V views of S Gaussian scenes in ONE launch sequence
(preprocess -> bucket scan -> scatter -> per-tile LDS sort -> composite), replacing the
per-view Python loop, the two `.item()` syncs per view and the Gaussian x views repeat
of the reference (cuda_splatting.py:90-125, decoder_splatting_cuda.py:53-56).
The only host sync is one 8-byte read of (num_rendered, max tile count) per batch,
needed to size the key buffer.
"""
from __future__ import annotations

import ctypes
import math
import os
import warnings
from dataclasses import dataclass

import torch

from . import _lib

TILE = 16
GEOM_STRIDE = 12
CAM_FLOATS = 44  # sizeof(dsr_camera) / 4


def tiles(h: int, w: int) -> tuple[int, int]:
    return (w + TILE - 1) // TILE, (h + TILE - 1) // TILE


def pack_cameras(viewmatrix: torch.Tensor, projmatrix: torch.Tensor, campos: torch.Tensor,
                 tanfovx: torch.Tensor, tanfovy: torch.Tensor, bg: torch.Tensor,
                 scene: torch.Tensor, scale: torch.Tensor | None = None) -> torch.Tensor:
    """Build the device array of `dsr_camera` structs ([V, 44] float32, 176 B each).

    viewmatrix / projmatrix: [V, 4, 4] exactly as handed to GaussianRasterizationSettings
    (transposed torch matrices, cuda_splatting.py:83-86); campos [V, 3]; tanfov [V];
    bg [V, 3]; scene [V] int (which Gaussian set); scale [V] (1/near when the reference's
    scale-invariant rescale applies, else 1).
    """
    V = viewmatrix.shape[0]
    dev = viewmatrix.device
    f32 = torch.float32
    if scale is None:
        scale = torch.ones(V, dtype=f32, device=dev)
    scene_bits = scene.to(device=dev, dtype=torch.int32).view(f32).reshape(V, 1)
    cam = torch.cat([
        viewmatrix.reshape(V, 16).to(f32), projmatrix.reshape(V, 16).to(f32),
        campos.reshape(V, 3).to(f32), tanfovx.reshape(V, 1).to(f32), tanfovy.reshape(V, 1).to(f32),
        bg.reshape(V, 3).to(f32), scene_bits, scale.reshape(V, 1).to(f32),
        torch.zeros(V, 2, dtype=f32, device=dev),
    ], dim=1).contiguous()
    assert cam.shape[1] == CAM_FLOATS
    return cam


class KernelTimer:
    """HIP-event timing of C-ABI launches on the stream they are enqueued on (bench.py).
    `only`: restrict to these launch names (events perturb the timeline least)."""

    def __init__(self, only=None):
        self.events: dict[str, list] = {}
        self.only = None if only is None else set(only)

    def start(self, name):
        if self.only is not None and name not in self.only:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return name, e

    def stop(self, tok):
        name, e0 = tok
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.events.setdefault(name, []).append((e0, e1))

    def summary(self) -> dict[str, tuple[int, float]]:
        torch.cuda.synchronize()
        return {k: (len(v), sum(a.elapsed_time(b) for a, b in v) / len(v)) for k, v in self.events.items()}


# bench / profiling instrumentation only (HIP events around named launches); never set on
# the product path
_timer: KernelTimer | None = None


def set_timer(t: KernelTimer | None) -> None:
    global _timer
    _timer = t


def last_stats(ctx: "RasterContext | None" = None) -> dict:
    """(num_rendered, max tile count) of the last forward through `ctx` (default: the current
    device's default context). Reads the device: syncs."""
    return (ctx or default_context(torch.cuda.current_device())).last_stats()


def _timed(name, fn, *args):
    tok = _timer.start(name) if _timer is not None and not torch.cuda.is_current_stream_capturing() else None
    r = fn(*args)
    if tok is not None:
        _timer.stop(tok)
    return r


def algorithmic_bytes(kernel: str, *, G: int, V: int, N: int, HW: int, T: int | None = None, S: int = 1) -> int:
    """Compulsory HBM bytes of one launch: every input read once, every output
    written once. G Gaussians per scene, S scenes, V views, N (view, tile, Gaussian) entries,
    HW pixels per view. Per-entry gathers that caches can serve are not counted."""
    if kernel == "k_project_emit":  # 148 B of parameters per scene Gaussian in; 52 B record +
        return S * G * 148 + V * G * 52 + 8 * N  # radius per (view, Gaussian) + one key per entry out
    if kernel == "k_preprocess":   # 148 B of Gaussian params in, 48 B record + 4 B radius out
        return V * G * (148 + 52)
    if kernel == "k_scan":
        return 8 * V * (T or 0)
    if kernel == "k_scatter":      # xy, depth, radius in; one 8-B key out per entry
        return V * G * 16 + 8 * N
    if kernel == "k_sort":         # keys in + out
        return 16 * N
    if kernel == "k_render_fwd":   # keys; each 36-B compositing record once; RGB + T + n_contrib out
        return 8 * N + 36 * V * G + 20 * V * HW
    if kernel == "k_sort_render":  # keys in (sorted copy stays in LDS: inference), records, RGB + T
        return 8 * N + 36 * V * G + 16 * V * HW  # (no n_contrib on the inference path)
    if kernel == "k_render_bwd":   # keys, records, T + n_contrib + dL/dpixel in; 9 int64 sums per
        return 8 * N + 36 * V * G + 20 * V * HW + 72 * V * G  # rendered (view, Gaussian) out
    if kernel == "k_preprocess_bwd":  # params + per-view records and sums in; param grads out
        return S * G * (148 + 148) + V * G * (48 + 72)
    if kernel == "k_head_bwd":  # head row (148) + depth + pixel colour in, dhead (148) out per Gaussian;
        return S * G * (148 + 4 + 12 + 148) + V * G * (36 + 72)  # per view the record's 36 B, the 72-B sums
    raise KeyError(kernel)


def algorithmic_bytes_cut(kernel: str, *, G: int, V: int, N_written: int, HW: int, survivors: int,
                          S: int = 1) -> int:
    """Compulsory HBM bytes of one launch of the depth-cut kernels (deferred
    geometry): the count pass reads 40 B of parameters per scene Gaussian (no SH: no colour)
    and writes a radius + an 8-B rect record per (view, Gaussian); the scatter reads the rect
    records and writes one key per written entry; the survivor projection reads the listed
    Gaussians' 148 B and writes their 52-B record + radius; the fused sort + composite reads
    the written keys, the survivors' 36-B compositing records, writes RGB + T."""
    if kernel == "k_preprocess_cut":
        return S * G * 40 + V * G * 12
    if kernel == "k_scatter_cut":
        return V * G * 8 + 8 * N_written + 4 * survivors
    if kernel == "k_project_survivors":
        return survivors * (4 + 148 + 52)
    if kernel == "k_sort_render":
        return 8 * N_written + 36 * survivors + 16 * V * HW
    if kernel == "k_bin_cutoff":
        return V * 4 * 128 * 4
    raise KeyError(kernel)


class EntryOverflow(_lib.DsplatError):
    """The batch has too many (view, tile, Gaussian) entries for 32-bit key offsets."""


@dataclass
class RasterState:
    """Everything the backward needs (all device tensors)."""
    geom: torch.Tensor        # [V, G, 12]
    radii: torch.Tensor       # [V, G] int32
    seg_start: torch.Tensor | None  # [V*T + 1] int32 (prefix layout) or None
    seg_count: torch.Tensor   # [V*T] int32 entries per (view, tile)
    seg_stride: int           # 0: prefix layout; > 0: segment s starts at s * seg_stride
    keys: torch.Tensor        # int64 (uint64 keys, sorted per segment)
    final_T: torch.Tensor     # [V, H, W]
    n_contrib: torch.Tensor | None  # [V, H, W] int32 (None on the inference fast path)
    seg_sorted: torch.Tensor | None = None    # [V*T] sorted entries per segment (prefix-sort mode)
    seg_overflow: torch.Tensor | None = None  # [V*T(+1)] tiles re-sorted in full and re-rendered
    tile_count: torch.Tensor | None = None    # [V*T] all entries per tile (depth-cut mode: seg_count = ends)
    cams: torch.Tensor | None = None          # [V, 44] dsr_camera array the forward used
    # inference fast path with exact binning: the lists hold only entries whose alpha >= 1/255
    # ellipse reaches the tile, and n_contrib counts positions in those shorter lists
    pruned_lists: bool = False
    # the backward's int64 gradient accumulator, its rendered rows zeroed by the forward
    dgeom: torch.Tensor | None = None
    dgeom_filled: bool = False   # dgeom zeroed in full by this forward (not only its rendered rows)
    # bounded segments with a backward: the rebuilt tiles' sorted lists ([V*T, G] slots; read by
    # dsr_render_bwd for segments with seg_count > seg_stride)
    spill: torch.Tensor | None = None
    # depth-cut binning: (cut thresholds [V * super-blocks], compact records or None, super-block size)
    cut_plan: tuple | None = None
    # deferred geometry with a backward: [V*G] uint8, 1 for the rows projected in full (whose
    # records and accumulator rows exist); the preprocess backward reads only those
    row_live: torch.Tensor | None = None
    # False when the depth cut deferred the geometry (no backward): only the records of the
    # Gaussians a scatter pass listed are written (every Gaussian some list entry refers to)
    geom_complete: bool = True

    @property
    def counts(self) -> torch.Tensor:
        """Entries per (view, tile), whether or not all of them were written."""
        return self.seg_count if self.tile_count is None else self.tile_count

    @property
    def num_rendered(self) -> int:  # host read: syncs
        return int(self.counts.sum())

    @property
    def max_count(self) -> int:
        return int(self.counts.max())

    def written(self) -> torch.Tensor:
        """Entries per segment present (sorted) in `keys`."""
        if self.seg_stride == SEG_ENDS:
            return self.seg_count.long() - self.seg_start[:-1].long()
        return self.seg_count


# Key-buffer sizing. N (the number of (view, tile, Gaussian) entries) is only known on the
# device after the scan. Instead of reading it back mid-pipeline (the reference's per-view
# D2H + .item() syncs), the key buffers are sized by the exact worst case V*G*tiles when
# that fits KEY_BUDGET_BYTES (1.6 GB at 2x256^2 x 3 views; 34 GB for config C's 64 training
# views: cheap on a 288 GB part, and untouched pages cost no bandwidth); the whole forward
# then runs with NO host sync and the projection emits keys directly (no scan / scatter).
# Larger problems fall back to one 8-byte read of (N, max tile count) after the scan.
# None = automatic per RasterContext: 48 GiB, at most 40 % of the device's memory and half of
# what is free when the context first asks (env DSPLAT_KEY_BUDGET_GB overrides; tests set 0 to
# force the two-phase layout).
#
# The upper-case settings below are the DEFAULTS of every RasterContext option of the same
# name (read at call time where a context leaves the option unset); the product path never
# assigns them: a decoder changes its own context (RasterContext.set).
_kb_env = os.environ.get("DSPLAT_KEY_BUDGET_GB")
KEY_BUDGET_BYTES = None if _kb_env is None else int(float(_kb_env) * (1 << 30))


# Segment capacity of the inference fast path (bounded key memory): None = automatic per
# RasterContext — twice the largest tile list of the context's earlier calls rounded up to a
# power of two, at least 4096 (16384 before any call), at most G. A tile that gets more
# entries than its capacity is rebuilt from the geometry records by dsr_sort_render (exact,
# slow), so the capacity affects memory and speed only. Keys + sort scratch then take
# 16 B x views x tiles x capacity (0.8 GB at 16 scenes of config B) instead of x G (26 GB).
SEG_CAPACITY = None if os.environ.get("DSPLAT_SEG_CAPACITY") is None else int(os.environ["DSPLAT_SEG_CAPACITY"])

# Segments larger than this many entries (only when some exceed the LDS sort) get only their
# nearest SORT_PREFIX entries put in order (dsr_bin_sort prefix mode): at 6x448x768 the
# compositor uses at most ~1.2K of 30-40K entries per tile. 0 sorts everything.
SORT_PREFIX = int(os.environ.get("DSPLAT_SORT_PREFIX", "4096"))
# Depth-cut binning for the two-phase path (include/dsplat_hip.h): only about CUT_PREFIX
# entries per tile, the nearest depth buckets, are written and sorted; tiles whose pixels do
# not all saturate within them get the rest appended, sorted and rendered again. 0 = off.
CUT_PREFIX = int(os.environ.get("DSPLAT_CUT_PREFIX", "2048"))
# LDS sort class for the written parts (larger ones sort through HBM). 3072 keys (4 workgroups
# per CU) beat 4096 (3) and 2048 (heads above it go through HBM): config D 1.095 / 1.075 /
# 1.34 ms, config E 31.8 / 31.0 / 34.6 ms per scene (round 5, profiles/r05w_ab_cut_sort_hint.log)
CUT_SORT_HINT = 3072
# Depth cut (need_state False or True): the count pass writes no geometry record and evaluates
# no colour; each scatter pass lists the Gaussians that may emit and dsr_project_survivors
# projects only those (~3 % of the (view, Gaussian) pairs at 12x512x960). Off only where the
# compact 8-byte pre-test records cannot address the grid (more than 255 tiles a side) and in
# the test that keeps the full-record kernel covered. Without a backward the written heads are
# sorted and composited by one dsr_sort_render launch (flags for the tail pass as
# dsr_render_fwd's).
DEFER_GEOM = True
LAYOUT_DEFER_GEOM = 32
# Fixed-capacity binning with tile lists up to FUSED_MAX entries (the hint from earlier calls)
# sorts and composites in one launch (dsr_sort_render); longer lists take dsr_bin_sort +
# dsr_render_fwd (MSD split, prefix sort). Either is exact for any list length.
FUSED_SORT_RENDER = True
FUSED_MAX = 4096
# dsr_sort_render's LDS class comes from the largest count of earlier calls (the context's
# hints); a nonzero override pins it (tests: every class on the same lists)
SORT_RENDER_HINT = 0
# inference fast path: cameras inside the binning kernel, self-zeroing counters (False: the
# separate camera launch of the stateful path)
INKERNEL_CAMERAS = True
# Binning of the inference fast path: exact (a (Gaussian, tile) pair is kept only when the
# alpha >= 1/255 ellipse reaches the tile; same images, shorter lists) or the reference's
# 3-sigma rects (DSR_LAYOUT_RECT_BINNING; bench.py reports both throughputs).
EXACT_BINNING = True
LAYOUT_RECT_BINNING = 8
# The same exact test on the stateful (training) path, in the fixed-capacity and plain
# two-phase layouts (DSR_LAYOUT_EXACT_BINNING; the depth-cut layout keeps 3-sigma rects): the
# lists are order-preserving subsequences of the reference's, the dropped pairs fail the
# per-pixel alpha test at every pixel of their tile, so images and gradients are unchanged
# (tests/test_raster_gpu.py) while the sort, the forward and the backward walk about half the
# entries. Off: the reference's lists exactly (the oracle list tests switch it off).
STATEFUL_EXACT_BINNING = True
LAYOUT_EXACT_BINNING = 16
# Forwards with a backward use bounded fixed-capacity segments too (forward_raw, round 5)
BOUNDED_TRAIN_SEGMENTS = True
# Test hook (tests/test_fullsize_parity.py): the fast path also snapshots its per-tile counts
# and writes its sorted keys back, so its lists can be compared with the oracle's. It adds a
# copy and the key stores; the product never sets it.
DEBUG_KEEP_FAST_LISTS = False
SEG_ENDS = 0xFFFFFFFF  # DSR_SEG_ENDS
# Depth cut: queue the scatter before the N read-back, into keys sized from the previous call
# (round 6; DSPLAT_EARLY_CUT_SCATTER=0 restores the synchronous order for A/B timing)
EARLY_CUT_SCATTER = os.environ.get("DSPLAT_EARLY_CUT_SCATTER", "1") != "0"
_HIST_LDS_MAX = 32768  # tiles per view binned in k_project_emit's LDS histogram (kHistLdsMax)


class RasterContext:
    """Per-(device, caller) rasterizer state: the options of one decoder and the adaptive
    hints its earlier calls produced. SURVEY §8(b): nothing that one caller's calls learn or
    set leaks into another's (two decoders of different workloads, on different streams or
    devices, each keep their own LDS sort class, depth-cut plan, zeroed-counter pool and
    binning options; a hipGraph captured through a context keeps the hint it had then).

    Options (None: the module default of the same upper-case name, read at call time):
      exact_binning (inference path), stateful_exact_binning (training path),
      fused_sort_render, sort_render_hint, inkernel_cameras, sort_prefix, cut_prefix,
      debug_keep_fast_lists, key_budget_bytes (None and no module override: automatic,
      min(48 GiB, 40 % of the device, half of its memory free when first asked)),
      seg_capacity (inference fast path: entries per (view, tile) segment; None = from the
      hints, see SEG_CAPACITY), defer_geom (depth cut: see DEFER_GEOM).
    hints: max_count (largest tile list seen: picks the fused sort's LDS class),
      two_phase_max (largest list of the last two-phase call: plans the depth cut).
    adapt_hints False freezes the hints (tests pin a class)."""

    _OPTS = {"exact_binning": "EXACT_BINNING", "stateful_exact_binning": "STATEFUL_EXACT_BINNING",
             "fused_sort_render": "FUSED_SORT_RENDER", "sort_render_hint": "SORT_RENDER_HINT",
             "inkernel_cameras": "INKERNEL_CAMERAS", "sort_prefix": "SORT_PREFIX", "cut_prefix": "CUT_PREFIX",
             "debug_keep_fast_lists": "DEBUG_KEEP_FAST_LISTS", "key_budget_bytes": "KEY_BUDGET_BYTES",
             "seg_capacity": "SEG_CAPACITY", "defer_geom": "DEFER_GEOM",
             "bounded_train_segments": "BOUNDED_TRAIN_SEGMENTS"}

    def __init__(self, **options):
        unknown = set(options) - set(self._OPTS)
        if unknown:
            raise TypeError(f"unknown rasterizer options {sorted(unknown)}")
        self.options = dict(options)
        self.hints = {"max_count": 0, "two_phase_max": None}
        self.adapt_hints = True
        self._inflight: list = []      # (pinned int32 counts, event) read-backs, consumed without blocking
        self._last: dict = {"counts": None, "host_counts": None}
        self._auto_budget: dict = {}   # device index -> bytes
        self._clean_counts: dict = {}  # (device, n) -> (zeroed counters, last stream, event)
        self._graph_owned: list = []
        self._warned_rebuild = False

    def opt(self, name: str):
        v = self.options.get(name)
        return globals()[self._OPTS[name]] if v is None else v

    def set(self, **options) -> "RasterContext":
        unknown = set(options) - set(self._OPTS)
        if unknown:
            raise TypeError(f"unknown rasterizer options {sorted(unknown)}")
        self.options.update(options)
        return self

    def seg_capacity(self, G: int) -> int:
        """Segment capacity of the inference fast path (SEG_CAPACITY)."""
        c = self.opt("seg_capacity")
        if c is None:
            m = self.hints["max_count"]
            c = 16384 if m == 0 else max(4096, 1 << max(0, 2 * m - 1).bit_length())
        return max(1, min(int(c), G))

    def key_budget(self, device) -> int:
        b = self.opt("key_budget_bytes")
        if b is not None:
            return int(b)
        idx = torch.device(device).index or 0
        b = self._auto_budget.get(idx)
        if b is None:
            total = torch.cuda.get_device_properties(idx).total_memory
            free, _ = torch.cuda.mem_get_info(idx)
            b = self._auto_budget[idx] = int(min(48 * (1 << 30), 0.4 * total, 0.5 * free))
        return b

    def note_counts(self, counts: torch.Tensor, capacity: int | None = None) -> None:
        """Queue a non-blocking copy of the per-segment counts to pinned memory; completed
        copies from earlier calls update the LDS-sort size hint (their max). Never waits on
        the device, never adds a kernel (a device-side max would need same-address atomics
        from every workgroup, which serialise). capacity: the bounded segment capacity of that
        call (inference fast path); tiles above it were rebuilt from the geometry records by
        dsr_sort_render (exact, but one pass over the view's records per radix digit): counted
        in last_stats()["rebuilt_tiles"], and warned about when the hints are frozen (the
        capacity cannot grow to absorb them)."""
        if torch.cuda.is_current_stream_capturing():
            return  # inside a hipGraph capture: no host-side bookkeeping (hint stays fixed)
        while self._inflight and self._inflight[0][1].query():
            host, _, cap = self._inflight.pop(0)
            m = int(host.max())
            if self.adapt_hints:
                self.hints["max_count"] = m
            elif cap is not None and m > cap and not self._warned_rebuild:
                self._warned_rebuild = True
                warnings.warn(f"{int((host > cap).sum())} tile list(s) of up to {m} entries exceeded the frozen "
                              f"segment capacity {cap}: rebuilt from the geometry records (exact, slow); unfreeze "
                              "the hints (adapt_hints) or set a larger seg_capacity", RuntimeWarning, stacklevel=3)
        if len(self._inflight) < 4:
            host = torch.empty(counts.shape, dtype=torch.int32, pin_memory=True)
            host.copy_(counts, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._inflight.append((host, ev, capacity))
            self._last["host_counts"] = (host, ev)
            self._last["capacity"] = capacity

    def last_stats(self) -> dict:
        """(num_rendered, max tile count) of this context's last forward (syncs); after a
        depth-cut forward also the entries written (sorted + composited) and the (view,
        Gaussian) records projected by the survivor passes."""
        c = self._last["counts"]
        if c is None:  # consumed on the device (inference fast path): the newest pinned copy
            hc = self._last.get("host_counts")
            if hc is None:
                return {"num_rendered": 0, "max_count": 0}
            hc[1].synchronize()
            c = hc[0]
        n, m = int(c.sum()), int(c.max())
        if self.adapt_hints:
            self.hints["max_count"] = m
        out = {"num_rendered": n, "max_count": m}
        cap = self._last.get("capacity")
        if c is not None and cap is not None and self._last["counts"] is None:
            out["rebuilt_tiles"] = int((c > cap).sum())  # bounded segments rebuilt by dsr_sort_render
        cut = self._last.get("cut")
        if cut is not None:
            start, ends, surv_n = cut
            out["written"] = int((ends.long() - start[:-1].long()).sum())
            if surv_n is not None:
                out["survivors"] = int(surv_n.long().sum())
        return out

    # Counter buffers that are zero once the work of their last user is done:
    # dsr_sort_render(clear_counts=1) zeroes each counter as it consumes it, so the next
    # inference forward needs no zeroing launch (dsr_project_bin_cameras takes them as
    # zeroed). A buffer is reused on the stream that last used it (stream order), or on another
    # stream once an event recorded after its last use has completed. A buffer taken while a
    # stream is captured into a graph belongs to that graph from then on (each replay leaves
    # it zeroed again).
    def take_clean_counts(self, n: int, dev, stream) -> torch.Tensor | None:
        key = (str(dev), n)
        ent = self._clean_counts.get(key)
        capturing = torch.cuda.is_current_stream_capturing()
        if ent is not None:
            t, last_stream, ev = ent
            # (events cannot be queried during capture: graphs.GraphedCall synchronizes the device
            # before capturing, so the buffer's last user has finished by then)
            if capturing or last_stream == int(stream) or ev.query():
                del self._clean_counts[key]
                return t
        if capturing:
            return None  # a zeroing node inside the graph would cost what the fast path saves
        return torch.zeros(n, dtype=torch.int32, device=dev)

    def give_back_clean_counts(self, t: torch.Tensor, dev, stream) -> None:
        if torch.cuda.is_current_stream_capturing():
            self._graph_owned.append(t)  # the captured graph keeps using (and re-zeroing) it
            return
        ev = torch.cuda.Event()
        ev.record()
        if len(self._clean_counts) > 64:
            self._clean_counts.clear()
        self._clean_counts[(str(dev), t.numel())] = (t, int(stream), ev)


_default_contexts: dict = {}


def default_context(device=None) -> RasterContext:
    """The context of callers that bring none (the functional API: render_cuda & co.), one
    per device."""
    idx = torch.device(device).index if device is not None else torch.cuda.current_device()
    idx = idx or 0
    ctx = _default_contexts.get(idx)
    if ctx is None:
        ctx = _default_contexts[idx] = RasterContext()
    return ctx


def key_budget(device, ctx: RasterContext | None = None) -> int:
    return (ctx or default_context(device)).key_budget(device)


_ws_cache: dict = {}


def workspace(G: int, H: int, W: int, V: int, device=None, ctx: RasterContext | None = None) -> _lib.Workspace:
    """dsr_workspace_size: the bytes of every buffer of one call sequence and whether the
    sync-free fixed-capacity layout fits the key budget (the C ABI's own sizing rule)."""
    budget = key_budget(device if device is not None else torch.cuda.current_device(), ctx)
    key = (G, H, W, V, budget)
    ws = _ws_cache.get(key)
    if ws is None:
        ws = _lib.Workspace()
        _lib.check(_lib.load().dsr_workspace_size(G, H, W, V, budget, _lib.ctypes.byref(ws)),
                   "dsr_workspace_size")
        if len(_ws_cache) > 256:
            _ws_cache.clear()
        _ws_cache[key] = ws
    return ws


_index_cache: dict = {}


def device_index(values, device) -> torch.Tensor:
    """Small int32 index arrays (view -> scene maps) cached on the device, so steady-state
    calls do no pageable H2D copy (which would serialise the host with the stream)."""
    key = (tuple(int(v) for v in values), str(device))
    t = _index_cache.get(key)
    if t is None:
        if len(_index_cache) > 256:
            _index_cache.clear()
        t = torch.tensor(key[0], dtype=torch.int32).to(device)
        _index_cache[key] = t
    return t


_bg_cache: dict = {}


def _dense_bg(bg: torch.Tensor) -> torch.Tensor:
    """Contiguous [V, 3] background. The decoder passes its background buffer expanded over
    the views (stride 0); materialising it each call costs a copy kernel per step, so the
    dense copy is cached per (storage, view count, version)."""
    if bg.is_contiguous() and bg.dtype == torch.float32:
        return bg.detach()
    base = bg._base if bg._base is not None else bg
    key = (id(base), bg.storage_offset(), tuple(bg.shape), tuple(bg.stride()))
    hit = _bg_cache.get(key)
    # the entry holds the base tensor itself (so its id / memory cannot be reused while
    # cached) and its version counter (so in-place edits of the background invalidate it)
    if hit is not None and hit[0] is base and hit[1] == base._version:
        return hit[2]
    if len(_bg_cache) > 64:
        _bg_cache.clear()
    t = bg.detach().contiguous().float()
    _bg_cache[key] = (base, base._version, t)
    return t


@dataclass
class CameraInputs:
    """render_cuda's camera inputs, turned into dsr_camera structs by the first kernel that
    needs them (dsr_build_cameras, or inside dsr_project_bin_cameras: no launch of its own).
    extrinsics [V,4,4] c2w, intrinsics [V,3,3] normalised, near/far [V], bg [V,3] dense,
    view_scene [V] int32 (device)."""
    extrinsics: torch.Tensor
    intrinsics: torch.Tensor
    near: torch.Tensor
    far: torch.Tensor
    bg: torch.Tensor
    view_scene: torch.Tensor
    scale_invariant: bool
    # views grouped by scene in order (view v renders scene v // views_per_scene), 0 otherwise:
    # lets the binning kernel place whole scenes on one XCD
    views_per_scene: int = 0

    @property
    def V(self) -> int:
        return self.extrinsics.shape[0]


def views_per_scene(view_scene) -> int:
    """k if view_scene == [0]*k + [1]*k + ... (the decoder's (b, v) flattening), else 0."""
    vs = [int(x) for x in view_scene]
    if not vs:
        return 0
    k = vs.count(0)
    if k == 0 or len(vs) % k or any(s != i // k for i, s in enumerate(vs)):
        return 0
    return k if k < 256 else 0


@dataclass
class CameraBlock:
    """A caller-built dsr_camera array [V, 44] float32 (pack_cameras of the reference wrapper's
    GaussianRasterizationSettings, or build_cameras) for the inference fast path: the benched
    kernels (dsr_project_bin_cameras in camera-block mode + dsr_sort_render) on exactly these
    cameras instead of the ones they would set up in float from the render_cuda inputs."""
    cams: torch.Tensor

    @property
    def V(self) -> int:
        return self.cams.shape[0]


def camera_inputs(extrinsics, intrinsics, near, far, bg, view_scene, scale_invariant=True) -> CameraInputs:
    dev = extrinsics.device
    _lib.require_gpu(extrinsics, intrinsics, near, far, bg)
    vps = 0 if isinstance(view_scene, torch.Tensor) else views_per_scene(view_scene)
    vs = view_scene.to(device=dev, dtype=torch.int32) if isinstance(view_scene, torch.Tensor) \
        else device_index(view_scene, dev)
    f = lambda t: t.detach().contiguous().float()  # noqa: E731
    return CameraInputs(f(extrinsics), f(intrinsics), f(near), f(far), _dense_bg(bg), vs, bool(scale_invariant),
                        vps)


def build_cameras(extrinsics, intrinsics, near, far, bg, view_scene, scale_invariant=True,
                  zero_counts: torch.Tensor | None = None) -> torch.Tensor:
    """Device-side camera set-up (dsr_build_cameras) -> [V, 44] float32 dsr_camera array.
    zero_counts (int32, optional) is zeroed by the same launch (see rasterize_views)."""
    lib = _lib.load()
    V = extrinsics.shape[0]
    dev = extrinsics.device
    _lib.require_gpu(extrinsics, intrinsics, near, far, bg)
    cams = torch.empty((V, CAM_FLOATS), dtype=torch.float32, device=dev)
    vs = view_scene.to(device=dev, dtype=torch.int32) if isinstance(view_scene, torch.Tensor) \
        else device_index(view_scene, dev)
    f = lambda t: t.detach().contiguous().float()  # noqa: E731
    ext, K, n, fa = f(extrinsics), f(intrinsics), f(near), f(far)
    b = _dense_bg(bg)
    _lib.check(lib.dsr_build_cameras(V, ext.data_ptr(), K.data_ptr(), n.data_ptr(), fa.data_ptr(), b.data_ptr(),
                                     vs.data_ptr(), int(bool(scale_invariant)), cams.data_ptr(),
                                     _ptr(zero_counts), 0 if zero_counts is None else zero_counts.numel(),
                                     _lib.stream_of(dev)), "dsr_build_cameras")
    return cams


LAYOUT_SH_CHANNEL_MAJOR = 1  # feats [S,G,3,M] (Gaussians.harmonics) instead of [S,G,M,3]
LAYOUT_COV_FULL = 2          # covariance [S,G,3,3] instead of cov6 [S,G,6]
LAYOUT_COUNTS_ZEROED = 4     # seg_count handed in already zeroed


def input_layout(feats, cov6, use_sh, channel_major_sh):
    lay = LAYOUT_COV_FULL if cov6.dim() >= 2 and tuple(cov6.shape[-2:]) == (3, 3) else 0
    if use_sh and channel_major_sh:
        lay |= LAYOUT_SH_CHANNEL_MAJOR
    return lay


def forward_raw(means, feats, use_sh, sh_degree, opacities, cov6, cams, V, H, W, layout=0, zeroed_counts=None,
                need_state=True, dgeom_zero: torch.Tensor | None = None, ctx: RasterContext | None = None):
    """Run the forward kernels. means [S,G,3]; feats [S,G,M,3] (use_sh; [S,G,3,M] with
    LAYOUT_SH_CHANNEL_MAJOR) or [S,G,3]; opacities [S,G]; cov6 [S,G,6] (or [S,G,3,3] with
    LAYOUT_COV_FULL); cams [V,44]. Returns (color [V,3,H,W], RasterState).

    Two binning layouts (include/dsplat_hip.h): when the fixed-capacity key buffer
    (V*T*G slots) fits KEY_BUDGET_BYTES, dsr_project_bin projects and emits keys in one
    kernel (no scan, no second pass over the geometry, no host sync); otherwise the
    two-phase path counts, scans (one 8-byte read-back of N), scatters.
    dgeom_zero: the backward's [V, G, DGEOM_WORDS] int64 accumulator, whose rendered rows
    the projection kernel zeroes as it writes their records (no separate fill pass).
    ctx: the caller's RasterContext (options + adaptive hints; default: the device's)."""
    lib = _lib.load()
    cam_in = cams if isinstance(cams, CameraInputs) else None
    cam_blk = cams if isinstance(cams, CameraBlock) else None
    if cam_blk is not None:
        cams = cam_blk.cams
    _lib.require_gpu(means, feats, opacities, cov6, None if cam_in is not None else cams)
    S, G = means.shape[0], means.shape[1]
    M = (feats.shape[3] if layout & LAYOUT_SH_CHANNEL_MAJOR else feats.shape[2]) if use_sh else 0
    dev = means.device
    ctx = ctx or default_context(dev)
    spec = ctx.hints
    gx, gy = tiles(H, W)
    T = gx * gy
    st = _lib.stream_of(dev)
    deg = sh_degree if use_sh else -1
    shs_p = feats.data_ptr() if use_sh else None
    col_p = None if use_sh else feats.data_ptr()
    geom = torch.empty((V, G, GEOM_STRIDE), dtype=torch.float32, device=dev)
    radii = torch.empty((V, G), dtype=torch.int32, device=dev)
    dgeom_filled = False
    lds_cap = lib.dsr_sort_lds_capacity()
    maxc_hint = spec["max_count"] or lds_cap
    # eager inference fast path: cameras set up inside the binning kernel, counters taken zeroed
    # from the previous call's sort + composite (two launches per forward), segments of bounded
    # capacity (keys + scratch: 16 B per (view, tile, capacity slot))
    debug_lists = ctx.opt("debug_keep_fast_lists")
    cut_fused = False  # depth cut without a backward: heads sorted + composited by dsr_sort_render
    cap = G if debug_lists else ctx.seg_capacity(G)
    fast = (ctx.opt("fused_sort_render") and maxc_hint <= FUSED_MAX
            and ((ctx.opt("inkernel_cameras") and cam_in is not None) or cam_blk is not None)
            and not need_state and zeroed_counts is None and T <= _HIST_LDS_MAX
            and V * T * cap < (1 << 32) and 16 * V * T * cap <= ctx.key_budget(dev))
    clean = ctx.take_clean_counts(V * T, dev, st) if fast else None
    fast = clean is not None
    fixed = fast or bool(workspace(G, H, W, V, dev, ctx).fixed_capacity)
    fused = fixed and ctx.opt("fused_sort_render") and maxc_hint <= FUSED_MAX
    # training with bounded segments (round 5): the fixed-capacity layout with the same adaptive
    # capacity as the inference fast path instead of G slots per (view, tile) — config C's keys
    # then span 1 GB instead of 17 GB (the scattered key stores and the sort's reads touched a
    # new page per segment). A tile above the capacity is rendered exactly (rebuilt by
    # dsr_sort_render), which stores its sorted list in the spill area ([V*T, G] slots, touched
    # only by such tiles) where dsr_render_bwd reads it: no host check between the passes.
    bounded = (not fast and fused and need_state and not debug_lists and ctx.opt("bounded_train_segments")
               and cap < G and T <= _HIST_LDS_MAX and V * T * cap < (1 << 32))
    stride = cap if (fast or bounded) else G
    if fast:
        seg_count = clean
        layout |= LAYOUT_COUNTS_ZEROED
        if not ctx.opt("exact_binning"):
            layout |= LAYOUT_RECT_BINNING
        if cam_blk is None:  # written by the binning kernel's camera set-up
            cams = torch.empty((V, CAM_FLOATS), dtype=torch.float32, device=dev)
    elif zeroed_counts is not None:  # zeroed by dsr_build_cameras (one launch fewer)
        assert zeroed_counts.numel() == V * T and zeroed_counts.dtype == torch.int32
        seg_count = zeroed_counts
        layout |= LAYOUT_COUNTS_ZEROED
    else:
        seg_count = torch.empty(V * T, dtype=torch.int32, device=dev)
    if cam_in is not None and not fast:  # one launch: cameras + zeroed counters
        cams = build_cameras(cam_in.extrinsics, cam_in.intrinsics, cam_in.near, cam_in.far, cam_in.bg,
                             cam_in.view_scene, cam_in.scale_invariant,
                             zero_counts=None if layout & LAYOUT_COUNTS_ZEROED else seg_count)
        layout |= LAYOUT_COUNTS_ZEROED
    surv = None      # depth cut, deferred geometry: the survivor lists of the scatter passes
    row_live = None  # ... with a backward: the (view, Gaussian) rows projected in full (survivors)
    if fixed:
        keys = torch.empty(V * T * stride, dtype=torch.int64, device=dev)
        # scratch for segments above the LDS sort (their size is unknown before the sort)
        scratch = torch.empty(V * T * stride, dtype=torch.int64, device=dev)
        spill = torch.empty(V * T * G, dtype=torch.int64, device=dev) if bounded else None
        if fast:
            ci = cam_in
            # camera-block mode: NULL render_cuda inputs, cams is the caller's (an input)
            cin = (None,) * 6 + (0,) if ci is None else (
                ci.extrinsics.data_ptr(), ci.intrinsics.data_ptr(), ci.near.data_ptr(), ci.far.data_ptr(),
                ci.bg.data_ptr(), ci.view_scene.data_ptr(), int(ci.scale_invariant))
            vps = ci.views_per_scene if ci is not None and S >= 8 else 0
            _lib.check(_timed("k_project_emit", lib.dsr_project_bin_cameras,
                S, G, V, H, W, deg, M, means.data_ptr(), shs_p, col_p, opacities.data_ptr(), cov6.data_ptr(),
                *cin, cams.data_ptr(),
                geom.data_ptr(), radii.data_ptr(), _ptr(dgeom_zero), seg_count.data_ptr(), keys.data_ptr(), stride,
                layout | (vps << 16), st),
                "dsr_project_bin_cameras")
        else:
            if ctx.opt("stateful_exact_binning"):
                layout |= LAYOUT_EXACT_BINNING
            # the backward's accumulator: here (every row of the view is projected) one streaming
            # fill beats zeroing the 72-B rows inside the projection kernel (config C step 3.16 ->
            # 3.06 ms, same-box A/B); the depth-cut path below keeps the in-kernel zeroing of the
            # few rows it projects in full
            dz = dgeom_zero
            if dz is not None:
                dz.zero_()
            dgeom_filled = dz is not None
            dz = None
            if bounded:  # camera-block mode: the same kernel with a segment capacity
                if not layout & LAYOUT_EXACT_BINNING:  # (dsr_sort_render rebuilds with the same test)
                    layout |= LAYOUT_RECT_BINNING
                _lib.check(_timed("k_project_emit", lib.dsr_project_bin_cameras,
                    S, G, V, H, W, deg, M, means.data_ptr(), shs_p, col_p, opacities.data_ptr(), cov6.data_ptr(),
                    *((None,) * 6 + (0,)), cams.data_ptr(), geom.data_ptr(), radii.data_ptr(), None,
                    seg_count.data_ptr(), keys.data_ptr(), stride, layout, st), "dsr_project_bin_cameras(bounded)")
            else:
                _lib.check(_timed("k_project_emit", lib.dsr_project_bin,
                    S, G, V, H, W, deg, M, means.data_ptr(), shs_p, col_p, opacities.data_ptr(), cov6.data_ptr(),
                    cams.data_ptr(), geom.data_ptr(), radii.data_ptr(), _ptr(dz), seg_count.data_ptr(),
                    keys.data_ptr(), layout, st), "dsr_project_bin")
        seg_start = None
        seg_sorted = None
        if not fused:
            ws = _sort_workspace(lib, V, H, W, maxc_hint, dev)
            seg_sorted = _prefix_sort(lib, G, V, H, W, None, seg_count, stride, keys, scratch, maxc_hint, ws, st,
                                      lds_cap, ctx.opt("sort_prefix"))
        ctx.note_counts(seg_count, stride if (fast or bounded) and stride < G else None)
    else:
        # the depth cut pays when tile lists are long; the previous two-phase call's largest
        # list (None on the first call) decides whether this one builds the depth histogram
        cut_prefix = ctx.opt("cut_prefix")
        defer, surv, surv_n = False, None, None  # deferred geometry (set below when the cut is planned)
        prev = spec.get("two_phase_max")
        want_cut = cut_prefix > 0 and (prev is None or prev > 4 * cut_prefix)
        sb = lib.dsr_cut_superblock(H, W) if want_cut else 0
        if sb > 0:
            nsb = -(-gx // sb) * -(-gy // sb)
            hist = torch.empty(V * nsb * 128, dtype=torch.int32, device=dev)
            # 8 bytes per (view, Gaussian) for the scatter's pre-test instead of the 48-byte record
            cut_rec = torch.empty(V * G * 2, dtype=torch.int32, device=dev) \
                if gx <= 255 and gy <= 255 else None
            # deferred geometry, with or without a backward: records (and, with a backward, the
            # accumulator rows) only for the Gaussians the scatter passes list; row_live marks
            # those rows for the preprocess backward (config D training: ~10 % of V x G)
            defer = bool(ctx.opt("defer_geom")) and cut_rec is not None
            if defer and need_state:
                row_live = torch.zeros(V * G, dtype=torch.uint8, device=dev)
            _lib.check(_timed("k_preprocess_cut", lib.dsr_preprocess_cut,
                S, G, V, H, W, deg, M, means.data_ptr(), shs_p, col_p, opacities.data_ptr(), cov6.data_ptr(),
                cams.data_ptr(), geom.data_ptr(), radii.data_ptr(), None if defer else _ptr(dgeom_zero),
                seg_count.data_ptr(),
                hist.data_ptr(), _ptr(cut_rec), layout | (LAYOUT_DEFER_GEOM if defer else 0), st),
                "dsr_preprocess_cut")
        else:
            if ctx.opt("stateful_exact_binning"):  # the scatter below repeats the same test
                layout |= LAYOUT_EXACT_BINNING
            _lib.check(_timed("k_preprocess", lib.dsr_preprocess_fwd,
                S, G, V, H, W, deg, M, means.data_ptr(), shs_p, col_p, opacities.data_ptr(), cov6.data_ptr(),
                cams.data_ptr(), geom.data_ptr(), radii.data_ptr(), _ptr(dgeom_zero), seg_count.data_ptr(), layout,
                st), "dsr_preprocess_fwd")
        seg_start = torch.empty(V * T + 1, dtype=torch.int32, device=dev)
        cursor = torch.empty(V * T, dtype=torch.int32, device=dev)
        totals = torch.empty(4, dtype=torch.int32, device=dev)
        _lib.check(_timed("k_scan", lib.dsr_bin_scan, V, H, W, seg_count.data_ptr(), seg_start.data_ptr(),
                          cursor.data_ptr(), totals.data_ptr(), st), "dsr_bin_scan")
        if torch.cuda.is_current_stream_capturing():
            raise _lib.DsplatError(f"V*G*tiles = {V * G * T} key slots exceed the key budget: this size needs a "
                                   "host read-back and cannot be captured into a graph")
        early = None  # capacity of the depth-cut scatter queued before the read-back
        if sb > 0:
            # what does not depend on N is queued before the read-back, so the device has work
            # while the host waits on it (the cut thresholds; the survivor counters)
            cut = torch.empty(V * nsb, dtype=torch.int32, device=dev)
            _lib.check(_timed("k_bin_cutoff", lib.dsr_bin_cutoff, V, H, W, hist.data_ptr(), cut_prefix,
                              cut.data_ptr(), st), "dsr_bin_cutoff")
            # deferred geometry: per view a list of the Gaussians each scatter pass may emit
            # (first pass: counts [0, V), tail: [V, 2V)), projected right after the pass
            if defer:
                slots, ncnt = ctypes.c_int64(), ctypes.c_int()
                _lib.check(lib.dsr_survivor_layout(G, V, ctypes.byref(slots), ctypes.byref(ncnt)),
                           "dsr_survivor_layout")
                surv = torch.empty(slots.value, dtype=torch.int32, device=dev)
                surv_n = torch.zeros(2 * ncnt.value, dtype=torch.int32, device=dev)
            proj = (S, G, V, H, W, deg, M, means.data_ptr(), shs_p, col_p, opacities.data_ptr(), cov6.data_ptr(),
                    cams.data_ptr())
            prev_n = spec.get("two_phase_n")
            if prev_n and EARLY_CUT_SCATTER:
                # round 6: the scatter (and its survivor projection) queued BEFORE the read-back,
                # into keys sized from the previous call's N: the device runs it while the host
                # waits, instead of idling from the cut thresholds to the host's next launch. The
                # launch checks N on the device and does nothing when the buffer is too small
                # (then it is re-run below with the exact size)
                early = int(prev_n * 1.25) + (1 << 16)
                keys = torch.empty(early, dtype=torch.int64, device=dev)
                scratch = torch.empty(early, dtype=torch.int64, device=dev)  # only big segments touch it
                _lib.check(_timed("k_scatter_cut", lib.dsr_bin_scatter_cut, G, V, H, W, geom.data_ptr(),
                                  cursor.data_ptr(), keys.data_ptr(), cut.data_ptr(), 0, None, _ptr(cut_rec),
                                  _ptr(surv), _ptr(surv_n), totals.data_ptr(), early, st), "dsr_bin_scatter_cut")
                if defer:
                    _lib.check(_timed("k_project_survivors", lib.dsr_project_survivors, *proj, surv.data_ptr(),
                                      surv_n.data_ptr(), geom.data_ptr(), radii.data_ptr(), _ptr(dgeom_zero),
                                      _ptr(row_live), layout, st), "dsr_project_survivors")
        tot = totals[:3].cpu()  # one small read-back: N sizes the key buffer
        N, maxc = int(tot[0]), int(tot[1])
        if ctx.adapt_hints:
            spec["two_phase_max"] = maxc
        if int(tot[2]):
            raise EntryOverflow(f"{V} views x {G} Gaussians produce >= 2^31 (view, tile, Gaussian) entries: "
                                "render fewer views per call")
        spec["two_phase_n"] = N
        if early is not None and (N > early or maxc <= 2 * cut_prefix):
            if N <= early:  # it ran, but the lists are short after all: cursors and counters back
                cursor.copy_(seg_start[:-1])
                if surv_n is not None:
                    surv_n.zero_()
            early = None
        if early is None:
            keys = torch.empty(max(N, 1), dtype=torch.int64, device=dev)
        if sb > 0 and maxc <= 2 * cut_prefix:  # short lists after all: write everything
            sb = 0
            surv = surv_n = None
            if defer:  # the full scatter reads every record: project them all now
                _project_all(lib, S, G, V, H, W, deg, M, means, shs_p, col_p, opacities, cov6, cams, geom, radii,
                             layout, dev, st, dgeom_zero, row_live)
        if sb > 0:
            # depth cut: write only each tile's nearest entries (cursor ends at their end)
            if early is None:
                scratch = torch.empty(max(N, 1), dtype=torch.int64, device=dev)  # only big segments touch it
                _lib.check(_timed("k_scatter_cut", lib.dsr_bin_scatter_cut, G, V, H, W, geom.data_ptr(),
                                  cursor.data_ptr(), keys.data_ptr(), cut.data_ptr(), 0, None, _ptr(cut_rec),
                                  _ptr(surv), _ptr(surv_n), None, 0, st), "dsr_bin_scatter_cut")
                if defer:
                    _lib.check(_timed("k_project_survivors", lib.dsr_project_survivors, *proj, surv.data_ptr(),
                                      surv_n.data_ptr(), geom.data_ptr(), radii.data_ptr(), _ptr(dgeom_zero),
                                      _ptr(row_live), layout, st), "dsr_project_survivors")
            tile_count, seg_count, stride = seg_count, cursor, SEG_ENDS
            # no backward: the written heads are sorted and composited in one launch below
            # (dsr_sort_render, flags as dsr_render_fwd); the keys stay unsorted in HBM unless a
            # test asks for the lists (debug_keep_fast_lists)
            cut_fused = not need_state
            if not cut_fused:
                _lib.check(_timed("k_sort", lib.dsr_bin_sort, G, V, H, W, seg_start.data_ptr(), seg_count.data_ptr(),
                                  stride, keys.data_ptr(), scratch.data_ptr(), CUT_SORT_HINT, None, 0, None, None,
                                  st), "dsr_bin_sort")
            seg_sorted = None
        else:
            scratch = torch.empty(max(N, 1), dtype=torch.int64, device=dev) if maxc > lds_cap else None
            # (counted by dsr_preprocess_cut when the cut was planned: 3-sigma rects, no exact bit)
            _lib.check(_timed("k_scatter", lib.dsr_bin_scatter, G, V, H, W, geom.data_ptr(), cursor.data_ptr(),
                              keys.data_ptr(), layout & LAYOUT_EXACT_BINNING, st), "dsr_bin_scatter")
            ws = _sort_workspace(lib, V, H, W, maxc, dev)
            stride = 0
            seg_sorted = _prefix_sort(lib, G, V, H, W, seg_start, seg_count, stride, keys, scratch, maxc, ws, st,
                                      lds_cap, ctx.opt("sort_prefix"))
    color = torch.empty((V, 3, H, W), dtype=torch.float32, device=dev)
    final_T = torch.empty((V, H, W), dtype=torch.float32, device=dev)
    # n_contrib (the last blended position, read only by the backward) is skipped on the
    # inference fast path: not tracking it takes ~4 VALU instructions off every (pixel, entry)
    keep_nc = not fast or need_state or debug_lists
    n_contrib = torch.empty((V, H, W), dtype=torch.int32, device=dev) if keep_nc else None
    outs = (color.data_ptr(), final_T.data_ptr(), _ptr(n_contrib), st)
    if fused:  # sort + composite in one launch; sorted keys kept only when a backward needs them
        snap = seg_count.clone() if (fast and debug_lists) else None
        _lib.check(_timed("k_sort_render", lib.dsr_sort_render, G, V, H, W, cams.data_ptr(), geom.data_ptr(), None,
                          seg_count.data_ptr(), stride, keys.data_ptr(), scratch.data_ptr(), _ptr(spill),
                          int(bool(need_state) or snap is not None), int(fast),
                          ctx.opt("sort_render_hint") or spec["max_count"], layout, *outs[:3], None, st),
                   "dsr_sort_render")
        state = RasterState(geom, radii, seg_start, seg_count, stride, keys, final_T, n_contrib, cams=cams,
                            dgeom_filled=dgeom_filled)
        state.spill = spill
        if fast:  # the counters are zero again once the launch above has run
            ctx.give_back_clean_counts(seg_count, dev, st)
            # consumed (no backward in this mode); with exact binning n_contrib counts positions
            # in the pruned lists (a subsequence of the reference's), not in the 3-sigma lists
            state.seg_count = snap
            state.pruned_lists = not (layout & LAYOUT_RECT_BINNING)
        else:
            state.pruned_lists = bool(layout & LAYOUT_EXACT_BINNING)
        ctx._last["counts"] = None if fast else state.counts
        ctx._last["cut"] = None
        return color, state
    overflow = None
    if seg_sorted is not None:
        overflow = torch.zeros(V * T + 1, dtype=torch.int32, device=dev)  # + the any-flag word
    elif stride == SEG_ENDS:  # + any-flag + flags per (view, super-block)
        overflow = torch.zeros(V * T + 1 + V * nsb, dtype=torch.int32, device=dev)
    if cut_fused:  # n_contrib only from the tail's re-render: not exposed (state.n_contrib None)
        _lib.check(_timed("k_sort_render", lib.dsr_sort_render, G, V, H, W, cams.data_ptr(), geom.data_ptr(),
                          seg_start.data_ptr(), seg_count.data_ptr(), stride, keys.data_ptr(), scratch.data_ptr(),
                          None, int(bool(debug_lists)), 0, CUT_SORT_HINT, layout, color.data_ptr(), final_T.data_ptr(),
                          None, overflow.data_ptr(), st), "dsr_sort_render(depth cut)")
    else:
        _lib.check(_timed("k_render_fwd", lib.dsr_render_fwd, G, V, H, W, cams.data_ptr(), geom.data_ptr(),
                          _ptr(seg_start), seg_count.data_ptr(), stride, keys.data_ptr(), _ptr(seg_sorted),
                          _ptr(overflow), None, *outs), "dsr_render_fwd")
    if overflow is not None:
        # tiles whose unsorted (or unwritten) tail would have blended: complete them, sort them
        # in full, render them again (every launch returns at once for unflagged tiles; no sync)
        if stride == SEG_ENDS:
            tail_n = None if surv is None else surv_n[surv_n.numel() // 2:]
            _lib.check(lib.dsr_bin_scatter_cut(G, V, H, W, geom.data_ptr(), seg_count.data_ptr(), keys.data_ptr(),
                                               cut.data_ptr(), 1, overflow.data_ptr(), _ptr(cut_rec), _ptr(surv),
                                               _ptr(tail_n), None, 0, st), "dsr_bin_scatter_cut(tail)")
            if surv is not None:
                _lib.check(lib.dsr_project_survivors(*proj, surv.data_ptr(), tail_n.data_ptr(), geom.data_ptr(),
                                                     radii.data_ptr(), _ptr(dgeom_zero), _ptr(row_live), layout, st),
                           "dsr_project_survivors(tail)")
        _lib.check(lib.dsr_bin_sort(G, V, H, W, _ptr(seg_start), seg_count.data_ptr(), stride, keys.data_ptr(),
                                    scratch.data_ptr(), 0, None, 0, _ptr(seg_sorted), overflow.data_ptr(), st),
                   "dsr_bin_sort(overflow)")
        _lib.check(lib.dsr_render_fwd(G, V, H, W, cams.data_ptr(), geom.data_ptr(), _ptr(seg_start),
                                      seg_count.data_ptr(), stride, keys.data_ptr(), None, None, overflow.data_ptr(),
                                      *outs), "dsr_render_fwd(overflow)")
    state = RasterState(geom, radii, seg_start, seg_count, stride, keys, final_T, None if cut_fused else n_contrib,
                        seg_sorted, overflow, tile_count if stride == SEG_ENDS else None, cams=cams)
    state.row_live = row_live
    state.dgeom_filled = dgeom_filled
    state.pruned_lists = bool(layout & LAYOUT_EXACT_BINNING) and stride != SEG_ENDS
    if stride == SEG_ENDS:  # the depth-cut plan (tools/cut_case.py statistics)
        state.cut_plan = (cut, cut_rec, lib.dsr_cut_superblock(H, W))
        state.geom_complete = surv is None
    ctx._last["counts"] = state.counts
    # depth cut: per-segment ends and the survivor counters (small; bench.py's roofline of the
    # cut kernels reads the entries written and the records projected from them)
    ctx._last["cut"] = (seg_start, seg_count, surv_n) if stride == SEG_ENDS else None
    return color, state


def _project_all(lib, S, G, V, H, W, deg, M, means, shs_p, col_p, opacities, cov6, cams, geom, radii, layout, dev, st,
                 dgeom_zero=None, row_live=None):
    """Deferred geometry abandoned (the lists turned out short): every record, through the
    survivor projection with lists that hold every Gaussian (slice p of a view: the blocks p,
    p + per_view, ... that the scatter's workgroup p walks)."""
    slots, ncnt = ctypes.c_int64(), ctypes.c_int()
    _lib.check(lib.dsr_survivor_layout(G, V, ctypes.byref(slots), ctypes.byref(ncnt)), "dsr_survivor_layout")
    pv, nt = ncnt.value // V, 256
    cap = slots.value // ncnt.value
    blk = torch.arange(cap // nt, device=dev)[None, :] * pv + torch.arange(pv, device=dev)[:, None]  # [pv, cap/nt]
    g = (blk[:, :, None] * nt + torch.arange(nt, device=dev)).reshape(pv, cap)
    n = (g < G).sum(1).to(torch.int32)  # the valid ids come first in every slice
    ids = g.clamp(max=G - 1).to(torch.int32).repeat(V, 1).reshape(-1)
    n = n.repeat(V)
    _lib.check(lib.dsr_project_survivors(S, G, V, H, W, deg, M, means.data_ptr(), shs_p, col_p, opacities.data_ptr(),
                                         cov6.data_ptr(), cams.data_ptr(), ids.data_ptr(), n.data_ptr(),
                                         geom.data_ptr(), radii.data_ptr(), _ptr(dgeom_zero), _ptr(row_live), layout,
                                         st), "dsr_project_survivors(all)")


def _prefix_sort(lib, G, V, H, W, seg_start, seg_count, stride, keys, scratch, max_count, ws, st, lds_cap,
                 sort_prefix):
    """dsr_bin_sort; prefix mode (returns seg_sorted) when segments exceed the LDS sort."""
    prefix = sort_prefix if (scratch is not None and max_count > lds_cap and sort_prefix > 0) else 0
    seg_sorted = torch.empty(seg_count.numel(), dtype=torch.int32, device=keys.device) if prefix else None
    _lib.check(_timed("k_sort", lib.dsr_bin_sort, G, V, H, W, _ptr(seg_start), seg_count.data_ptr(), stride,
                      keys.data_ptr(), _ptr(scratch), max_count, _ptr(ws), prefix, _ptr(seg_sorted), None, st),
               "dsr_bin_sort")
    return seg_sorted


def _ptr(t):
    return None if t is None else t.data_ptr()


def _sort_workspace(lib, V, H, W, max_count, dev):
    n = lib.dsr_bin_sort_workspace_size(V, H, W, max_count)
    return torch.empty(n, dtype=torch.uint8, device=dev) if n else None


DGEOM_WORDS = 9           # DSR_DGEOM_WORDS: int64 fixed-point gradient words per (view, Gaussian)
GRAD_SCALE_BLOCKS = 512   # DSR_GRAD_SCALE_BLOCKS




def render_bwd_raw(state: RasterState, cams, dcolor: torch.Tensor, G: int):
    """K7 of a forward's state: dsr_grad_scale + dsr_render_bwd into the 64-bit fixed-point rows
    (the forward's zeroed accumulator when it made one). Returns (dgeom_fx [V,G,DGEOM_WORDS],
    grad_scale)."""
    lib = _lib.load()
    V, _, H, W = dcolor.shape
    dev = dcolor.device
    st = _lib.stream_of(dev)
    dcolor = dcolor.contiguous().float()
    if state.dgeom is not None:  # rendered rows zeroed by the forward's projection kernel
        dgeom_fx, state.dgeom = state.dgeom, None
    else:
        dgeom_fx = torch.zeros((V, G, DGEOM_WORDS), dtype=torch.int64, device=dev)
    gscale = torch.empty(GRAD_SCALE_BLOCKS, dtype=torch.float32, device=dev)
    _lib.check(lib.dsr_grad_scale(V, H, W, dcolor.data_ptr(), gscale.data_ptr(), st), "dsr_grad_scale")
    _lib.check(_timed("k_render_bwd", lib.dsr_render_bwd, G, V, H, W, cams.data_ptr(), state.geom.data_ptr(),
                      _ptr(state.seg_start), state.seg_count.data_ptr(), state.seg_stride, state.keys.data_ptr(),
                      _ptr(state.spill), state.final_T.data_ptr(), state.n_contrib.data_ptr(), dcolor.data_ptr(),
                      gscale.data_ptr(), dgeom_fx.data_ptr(), st), "dsr_render_bwd")
    return dgeom_fx, gscale


def scene_view_index(view_scene, S: int, dev) -> torch.Tensor:
    """[scene_view_start (S + 1), scene_views (V)] int32 on the device: the views of each scene in
    view order (the fixed summation order of the preprocess backward)."""
    V = len(view_scene)
    order = sorted(range(V), key=lambda v: (view_scene[v], v))
    starts = [0] * (S + 1)
    for v in range(V):
        starts[view_scene[v] + 1] += 1
    for s in range(S):
        starts[s + 1] += starts[s]
    return device_index(starts + order, dev)


def backward_raw(means, feats, use_sh, sh_degree, opacities, cov6, cams, view_scene, state: RasterState,
                 dcolor, want_mean2d: bool, layout=0, want_dgeom: bool = False):
    """Rasterizer backward (K7 -> K8 + K9). Deterministic: the per-Gaussian sums are 64-bit
    fixed-point atomics (dsr_grad_scale + dsr_render_bwd), bit-identical run to run.
    Returns dmeans, dfeat, dopac, dcov6, dmean2d (or None), dgeom [V,G,12] float (only with
    want_dgeom; the values K8 + K9 consumed, else None)."""
    lib = _lib.load()
    S, G = means.shape[0], means.shape[1]
    V, _, H, W = dcolor.shape
    M = (feats.shape[3] if layout & LAYOUT_SH_CHANNEL_MAJOR else feats.shape[2]) if use_sh else 0
    dev = means.device
    st = _lib.stream_of(dev)
    dgeom_fx, gscale = render_bwd_raw(state, cams, dcolor, G)
    dgeom = None
    if want_dgeom:
        dgeom = torch.empty((V, G, GEOM_STRIDE), dtype=torch.float32, device=dev)
        _lib.check(lib.dsr_dgeom_to_float(G, V, state.geom.data_ptr(), dgeom_fx.data_ptr(), gscale.data_ptr(),
                                          _ptr(state.row_live), dgeom.data_ptr(), st), "dsr_dgeom_to_float")
    idx = scene_view_index(view_scene, S, dev)
    dmeans = torch.empty((S, G, 3), dtype=torch.float32, device=dev)
    dfeat = torch.empty_like(feats, dtype=torch.float32)
    dopac = torch.empty((S, G), dtype=torch.float32, device=dev)
    dcov6 = torch.empty_like(cov6, dtype=torch.float32)
    dmean2d = torch.empty((V, G, 3), dtype=torch.float32, device=dev) if want_mean2d else None
    _lib.check(_timed("k_preprocess_bwd", lib.dsr_preprocess_bwd,
        S, G, V, H, W, sh_degree if use_sh else -1, M, means.data_ptr(), feats.data_ptr() if use_sh else None,
        cov6.data_ptr(), cams.data_ptr(), state.geom.data_ptr(), dgeom_fx.data_ptr(), gscale.data_ptr(),
        idx.data_ptr(),
        idx[S + 1:].data_ptr(), _ptr(state.row_live), dmeans.data_ptr(), dfeat.data_ptr() if use_sh else None,
        None if use_sh else dfeat.data_ptr(), dopac.data_ptr(), dcov6.data_ptr(),
        None if dmean2d is None else dmean2d.data_ptr(), layout, st),
        "dsr_preprocess_bwd")
    return dmeans, dfeat, dopac, dcov6, dmean2d, dgeom


class _RasterizeViews(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means, feats, opacities, cov6, means2d, cams, view_scene, use_sh, sh_degree, H, W, layout,
                zeroed_counts, rctx):
        V = len(view_scene)
        need = any(ctx.needs_input_grad[:5])
        # the backward's accumulator: its rendered rows are zeroed by the projection kernel
        rc = rctx or default_context(means.device)
        dgeom = torch.empty((V, means.shape[1], DGEOM_WORDS), dtype=torch.int64, device=means.device) \
            if need else None
        color, state = forward_raw(means, feats, use_sh, sh_degree, opacities, cov6, cams, V, H, W, layout,
                                   zeroed_counts, need_state=need, dgeom_zero=dgeom, ctx=rc)
        state.dgeom = dgeom
        ctx.save_for_backward(means, feats, opacities, cov6, state.cams)
        ctx.state = state
        ctx.meta = (view_scene, use_sh, sh_degree, None if means2d is None else means2d.shape, layout)
        ctx.mark_non_differentiable(state.radii)
        return color, state.radii

    @staticmethod
    def backward(ctx, dcolor, _dradii):
        means, feats, opacities, cov6, cams = ctx.saved_tensors
        view_scene, use_sh, sh_degree, m2d_shape, layout = ctx.meta
        want_m2d = m2d_shape is not None and ctx.needs_input_grad[4]
        dmeans, dfeat, dopac, dcov6, dmean2d, _ = backward_raw(
            means, feats, use_sh, sh_degree, opacities, cov6, cams, view_scene, ctx.state, dcolor,
            want_mean2d=want_m2d, layout=layout)
        if dmean2d is not None:
            dmean2d = dmean2d.view(m2d_shape)
        return dmeans, dfeat, dopac, dcov6, dmean2d, None, None, None, None, None, None, None, None, None


def rasterize_views(means: torch.Tensor, feats: torch.Tensor, opacities: torch.Tensor, cov6: torch.Tensor,
                    cams: torch.Tensor, view_scene: list[int], *, use_sh: bool, sh_degree: int,
                    image_height: int, image_width: int, means2d: torch.Tensor | None = None,
                    channel_major_sh: bool = False, zeroed_counts: torch.Tensor | None = None,
                    ctx: RasterContext | None = None):
    """Differentiable render of V views. means [S,G,3]; feats [S,G,M,3] (SH, coefficient-major
    like the rasterizer's `shs`; [S,G,3,M] = Gaussians.harmonics with channel_major_sh) or
    [S,G,3] (colors_precomp); opacities [S,G]; cov6 [S,G,6] or the full [S,G,3,3] matrices
    (read through the reference's triu gather); cams [V,44] (pack_cameras / build_cameras);
    view_scene[v] = scene index of view v. zeroed_counts: optional [V*tiles] int32 buffer already
    zeroed (build_cameras(zero_counts=...)). ctx: the caller's RasterContext (a decoder's own;
    default: the device's). Returns color [V,3,H,W] and radii [V,G] (int32)."""
    S = means.shape[0]
    n_cams = cams.V if isinstance(cams, (CameraInputs, CameraBlock)) else cams.shape[0]
    if len(view_scene) != n_cams:
        raise ValueError(f"view_scene has {len(view_scene)} entries for {n_cams} cameras")
    if any(not (0 <= s < S) for s in view_scene):
        raise ValueError(f"view_scene entries must be in [0, {S})")
    n_coef = (feats.shape[3] if channel_major_sh else feats.shape[2]) if use_sh else 0
    if use_sh and not (0 <= sh_degree <= 3 and n_coef >= (sh_degree + 1) ** 2):
        raise ValueError(f"unsupported sh_degree={sh_degree} for {n_coef} coefficients")
    if image_height <= 0 or image_width <= 0:
        raise ValueError("image size must be positive")
    f = lambda t: t.contiguous().float()  # noqa: E731
    layout = input_layout(feats, cov6, use_sh, channel_major_sh)
    return _RasterizeViews.apply(f(means), f(feats), f(opacities), f(cov6), means2d,
                                 cams if isinstance(cams, CameraInputs) else
                                 CameraBlock(cams.cams.contiguous()) if isinstance(cams, CameraBlock) else cams.contiguous(),
                                 list(view_scene), use_sh, int(sh_degree), int(image_height), int(image_width),
                                 layout, zeroed_counts, ctx)


def sh_degree_of(n_coeffs: int) -> int:
    return math.isqrt(n_coeffs) - 1
