"""Host logic of the decoder layer (CPU, no kernels): the chunked multi-view driver
(model_wrapper.py:455-484) over a stub decoder that records the views it was asked for."""
from __future__ import annotations

import pytest
import torch

from my_depthsplat_amd.decoder import DecoderOutput, render_chunked


class _StubDecoder:
    def __init__(self):
        self.calls = []

    def __call__(self, gaussians, extrinsics, intrinsics, near, far, image_shape, depth_mode=None):
        b, v = extrinsics.shape[:2]
        h, w = image_shape
        self.calls.append((v, depth_mode))
        # colour = the view's translation x (identifies the view); depth only when asked
        color = extrinsics[:, :, 0, 3][..., None, None, None].expand(b, v, 3, h, w).clone()
        depth = None if depth_mode is None else torch.full((b, v, h, w), float(len(self.calls)))
        return DecoderOutput(color, depth)


@pytest.mark.parametrize("chunk", [None, 1, 3, 10, 25])
def test_render_chunked_matches_one_call(chunk):
    b, v, h, w = 2, 10, 4, 5
    ext = torch.eye(4).repeat(b, v, 1, 1)
    ext[:, :, 0, 3] = torch.arange(b * v, dtype=torch.float32).view(b, v)
    K = torch.eye(3).repeat(b, v, 1, 1)
    near, far = torch.full((b, v), 0.5), torch.full((b, v), 100.0)
    dec = _StubDecoder()
    out = render_chunked(dec, None, ext, K, near, far, (h, w), chunk, depth_mode="depth")
    assert out.color.shape == (b, v, 3, h, w)
    assert torch.equal(out.color[:, :, 0, 0, 0], ext[:, :, 0, 3])
    n = 1 if chunk is None else -(-v // chunk)
    assert [c[0] for c in dec.calls] == ([v] if chunk is None else [min(chunk, v - i * chunk) for i in range(n)])
    # depth: the first chunk's only, as the reference ignores the rest
    assert [c[1] for c in dec.calls] == ["depth"] + [None] * (n - 1)
    assert out.depth.shape[1] == (v if chunk is None else min(chunk, v))


def test_render_chunked_rejects_bad_chunk():
    ext = torch.eye(4).repeat(1, 2, 1, 1)
    with pytest.raises(ValueError):
        render_chunked(_StubDecoder(), None, ext, ext[..., :3, :3], torch.ones(1, 2), torch.ones(1, 2), (2, 2), 0)
