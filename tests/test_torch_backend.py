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


def _loss_exts():
    import importlib
    try:
        return (importlib.import_module("chamfer3D.chamfer_3D"),
                importlib.import_module("PyTorchEMD.emd_cuda"))
    except ImportError:
        pytest.skip("chamfer_3D / emd_cuda extensions not built (csrc/build_torch_backend.py)")


def test_loss_extensions_export_the_reference_names():
    ch, emd = _loss_exts()
    # chamfer_cuda.cpp:29-32 and PyTorchEMD/cuda/emd.cpp:23-27
    assert sorted(n for n in dir(ch) if not n.startswith("_")) == ["backward", "forward"]
    assert sorted(n for n in dir(emd) if not n.startswith("_")) == [
        "approxmatch_forward", "matchcost_backward", "matchcost_forward"]
    # the reference's chamfer returns 0 (after printing) on bad input
    z = torch.zeros(1, 4, 3)
    assert ch.forward(z, z, torch.zeros(1, 4), torch.zeros(1, 4), torch.zeros(1, 4, dtype=torch.int32),
                      torch.zeros(1, 4, dtype=torch.int32)) == 0
    # the reference's own extension name (PyTorchEMD/setup.py:26-29, backend.py:11-12),
    # as a module and through the drop-in backend.py's `emd_cuda_dynamic`
    import importlib
    ext = importlib.import_module("PyTorchEMD.emd_ext")
    assert sorted(n for n in dir(ext) if not n.startswith("_")) == [
        "approxmatch_forward", "matchcost_backward", "matchcost_forward"]
    from PyTorchEMD.backend import emd_cuda_dynamic
    assert emd_cuda_dynamic is ext


def test_extensions_check_shapes_before_any_launch():
    """A caller's shape or device mistake is a TORCH_CHECK error (chamfer: status
    0 after the message, as chamfer_cuda.cpp does), never a kernel launch.  The
    checks run before the HIP-tensor check can matter only on a GPU box, so the
    messages are matched where the order allows it on the CPU too."""
    ch, emd = _loss_exts()
    be = _ext()
    z = torch.zeros(1, 4, 3)
    # wrong idx2 shape: 0 on the CPU (host tensor) and on the GPU (shape)
    assert ch.forward(z, z, torch.zeros(1, 4), torch.zeros(1, 4),
                      torch.zeros(1, 4, dtype=torch.int32), torch.zeros(1, 5, dtype=torch.int32)) == 0
    with pytest.raises(RuntimeError):
        emd.matchcost_forward(z.double(), z.double(), torch.zeros(1, 3, 4, dtype=torch.float64))
    with pytest.raises(RuntimeError):
        be.trilinear_devoxelize_backward(torch.zeros(1, 2, 5), torch.zeros(1, 8, 4, dtype=torch.int32),
                                         torch.zeros(1, 8, 5), 2)


def test_torch_backend_flag_keeps_the_cpu_path(monkeypatch):
    """PCFM_TORCH_BACKEND=1: HIP tensors go to the extensions, CPU tensors still
    run the pure-PyTorch backend (pcfm.ops.host_routed)."""
    import importlib
    _ext()
    _loss_exts()
    monkeypatch.setenv("PCFM_TORCH_BACKEND", "1")
    import modules.functional.backend as be
    import chamfer3D.dist_chamfer_3D as dc
    import PyTorchEMD.emd as pe
    try:
        for m in (be, dc, pe):
            importlib.reload(m)
        assert be._backend.extension is be._torch_backend
        feat = torch.randn(2, 3, 50)
        coords = torch.randint(0, 4, (2, 3, 50), dtype=torch.int32)
        out, ind, cnt = be._backend.avg_voxelize_forward(feat, coords, 4)
        from pcfm import cpu_ops
        e_out, e_ind, e_cnt = cpu_ops.avg_voxelize_forward(feat, coords, 4)
        assert torch.equal(ind, e_ind) and torch.equal(cnt, e_cnt) and torch.allclose(out, e_out)
        a, b = torch.randn(2, 30, 3), torch.randn(2, 20, 3)
        d1, d2, i1, i2 = dc.chamfer_3DDist()(a, b)
        assert d1.shape == (2, 30) and i2.dtype == torch.int32
        cost = pe.earth_mover_distance(a, b, transpose=False)
        assert cost.shape == (2,) and torch.isfinite(cost).all()
    finally:
        monkeypatch.delenv("PCFM_TORCH_BACKEND")
        for m in (be, dc, pe):
            importlib.reload(m)


@pytest.mark.gpu
def test_loss_extensions_match_ctypes_bindings():
    from pcfm import _lib
    from pcfm import ops
    _lib.load()
    ch, emd = _loss_exts()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    b, n, m = 2, 700, 500
    x1 = torch.rand(b, n, 3, device=dev, generator=g)
    x2 = torch.rand(b, m, 3, device=dev, generator=g)

    def outs():
        return (torch.empty(b, n, device=dev), torch.empty(b, m, device=dev),
                torch.empty(b, n, device=dev, dtype=torch.int32),
                torch.empty(b, m, device=dev, dtype=torch.int32))
    a, c = outs(), outs()
    assert ch.forward(x1, x2, *a) == 1 and ops.chamfer_3D.forward(x1, x2, *c) == 1
    for p, q in zip(a, c):
        assert torch.equal(p, q)
    gd1, gd2 = torch.randn(b, n, device=dev, generator=g), torch.randn(b, m, device=dev, generator=g)
    ga = (torch.zeros_like(x1), torch.zeros_like(x2))  # the backward accumulates
    gc = (torch.zeros_like(x1), torch.zeros_like(x2))
    assert ch.backward(x1, x2, *ga, gd1, gd2, a[2], a[3]) == 1
    assert ops.chamfer_3D.backward(x1, x2, *gc, gd1, gd2, c[2], c[3]) == 1
    # the backward scatters with float atomics, as the reference's NmDistanceGradKernel
    # (chamfer3D.cu:155-195): the summation order, so the last bits, vary run to run
    for p, q in zip(ga, gc):
        assert torch.allclose(p, q, rtol=1e-5, atol=1e-6)
    for dt in (torch.float32, torch.float64):
        y1, y2 = x1.to(dt), x2.to(dt)
        mt = emd.approxmatch_forward(y1, y2)
        assert torch.equal(mt, ops.emd_cuda.approxmatch_forward(y1, y2))
        assert torch.equal(emd.matchcost_forward(y1, y2, mt), ops.emd_cuda.matchcost_forward(y1, y2, mt))
        gcost = torch.rand(b, device=dev, dtype=dt, generator=g) if dt == torch.float32 else \
            torch.rand(b, device=dev, generator=g).to(dt)
        for p, q in zip(emd.matchcost_backward(gcost, y1, y2, mt),
                        ops.emd_cuda.matchcost_backward(gcost, y1, y2, mt)):
            assert torch.equal(p, q)


@pytest.mark.gpu
def test_extensions_reject_wrong_shapes_on_the_gpu():
    """HIP tensors of the wrong shape or on mixed devices: a TORCH_CHECK error (or
    chamfer's 0), matching the ctypes binding's checks -- no kernel runs."""
    ch, emd = _loss_exts()
    be = _ext()
    d = "cuda"
    z = torch.zeros(1, 4, 3, device=d)
    i4 = torch.zeros(1, 4, dtype=torch.int32, device=d)
    assert ch.forward(z, z, torch.zeros(1, 4, device=d), torch.zeros(1, 4, device=d), i4,
                      torch.zeros(1, 5, dtype=torch.int32, device=d)) == 0
    assert ch.forward(z, z, torch.zeros(1, 4, device=d), torch.zeros(1, 4), i4, i4) == 0
    with pytest.raises(RuntimeError, match="match"):
        emd.matchcost_forward(z, z, torch.zeros(1, 3, 4, device=d))
    with pytest.raises(RuntimeError, match="grad_cost"):
        emd.matchcost_backward(torch.zeros(2, device=d), z, z, torch.zeros(1, 4, 4, device=d))
    with pytest.raises(RuntimeError, match="features"):
        be.trilinear_devoxelize_forward(4, True, torch.zeros(1, 3, 9, device=d),
                                        torch.zeros(1, 2, 63, device=d))
    with pytest.raises(RuntimeError, match="indices"):
        be.trilinear_devoxelize_backward(torch.zeros(1, 2, 5, device=d),
                                         torch.zeros(1, 8, 4, dtype=torch.int32, device=d),
                                         torch.zeros(1, 8, 5, device=d), 2)
    with pytest.raises(RuntimeError, match="coords"):
        be.avg_voxelize_forward(torch.zeros(1, 2, 5, device=d),
                                torch.zeros(1, 3, 4, dtype=torch.int32, device=d), 2)
    with pytest.raises(RuntimeError, match="indices"):
        be.grouping_backward(torch.zeros(1, 2, 3, 4, device=d),
                             torch.zeros(1, 3, 5, dtype=torch.int32, device=d), 10)
