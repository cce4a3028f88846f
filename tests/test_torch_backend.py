"""The torch C++ extension binding `_pvcnn_backend` (csrc/torch_backend.cpp):
the reference's 12 binding names (third_party/pvcnn/modules/functional/src/
bindings.cpp:10-44) over the same C ABI as the default ctypes binding.
CPU: the module loads and exports the 12 names, CPU tensors and the PointNet++
operators outside the hot path raise.  GPU: every in-scope function returns
exactly what the ctypes binding (pcfm.ops.backend) returns."""
import os
import sys

import pytest
import torch

REF_NAMES = sorted([
    "gather_features_forward", "gather_features_backward", "furthest_point_sampling",
    "ball_query", "grouping_forward", "grouping_backward",
    "three_nearest_neighbors_interpolate_forward", "three_nearest_neighbors_interpolate_backward",
    "trilinear_devoxelize_forward", "trilinear_devoxelize_backward",
    "avg_voxelize_forward", "avg_voxelize_backward"])


def _ext():
    from modules.functional import backend
    if backend._torch_backend is None:
        pytest.skip("_pvcnn_backend not built (csrc/build_torch_backend.py)")
    return backend._torch_backend


def test_extension_exports_the_reference_names():
    ext = _ext()
    assert sorted(n for n in dir(ext) if not n.startswith("_")) == REF_NAMES


def test_extension_rejects_host_tensors_and_out_of_scope_ops():
    ext = _ext()
    with pytest.raises(RuntimeError, match="HIP tensor"):
        ext.avg_voxelize_forward(torch.zeros(1, 2, 3), torch.zeros(1, 3, 3, dtype=torch.int32), 4)
    with pytest.raises(RuntimeError, match="outside this build's hot path"):
        ext.furthest_point_sampling(torch.zeros(1, 3, 8), 2)


@pytest.mark.gpu
def test_extension_matches_ctypes_binding():
    from pcfm import _lib
    from pcfm.ops import backend as ct
    _lib.load()
    ext = _ext()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    b, c, n, r = 2, 16, 3000, 8
    feat = torch.randn(b, c, n, device=dev, generator=g)
    vc = torch.randint(0, r, (b, 3, n), device=dev, generator=g, dtype=torch.int32)
    for x, y in zip(ext.avg_voxelize_forward(feat, vc, r), ct.avg_voxelize_forward(feat, vc, r)):
        assert torch.equal(x, y)
    out, ind, cnt = ct.avg_voxelize_forward(feat, vc, r)
    gy = torch.randn(b, c, r ** 3, device=dev, generator=g)
    assert torch.equal(ext.avg_voxelize_backward(gy, ind, cnt), ct.avg_voxelize_backward(gy, ind, cnt))
    coords = torch.rand(b, 3, n, device=dev, generator=g) * (r - 1)
    grid = torch.randn(b, c, r ** 3, device=dev, generator=g)
    for training in (True, False):
        e = ext.trilinear_devoxelize_forward(r, training, coords, grid)
        t = ct.trilinear_devoxelize_forward(r, training, coords, grid)
        for x, y in zip(e, t):
            assert torch.equal(x, y)
    _, inds, wgts = ct.trilinear_devoxelize_forward(r, True, coords, grid)
    gd = torch.randn(b, c, n, device=dev, generator=g)
    assert torch.equal(ext.trilinear_devoxelize_backward(gd, inds, wgts, r),
                       ct.trilinear_devoxelize_backward(gd, inds, wgts, r))
    centers = torch.rand(b, 3, 64, device=dev, generator=g)
    pts = torch.rand(b, 3, n, device=dev, generator=g)
    idx = ext.ball_query(centers, pts, 0.1, 16)
    assert torch.equal(idx, ct.ball_query(centers, pts, 0.1, 16))
    assert torch.equal(ext.grouping_forward(feat, idx), ct.grouping_forward(feat, idx))
    gg = torch.randn(b, c, 64, 16, device=dev, generator=g)
    assert torch.equal(ext.grouping_backward(gg, idx, n), ct.grouping_backward(gg, idx, n))
    # launched on torch's current stream
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        o2 = ext.grouping_forward(feat, idx)
    s.synchronize()
    assert torch.equal(o2, ct.grouping_forward(feat, idx))
