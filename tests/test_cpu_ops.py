"""The product's pure-PyTorch CPU backend (pcfm.cpu_ops, BASELINE configs[0])
against the C oracle (oracle/pcfm_oracle.c) and the reference's fixtures.

Two independent restatements of the reference kernels -- sequential C with
explicit fmaf, and vectorised torch (scatter_add_ / gather / blocked argmin) --
are held to each other: integer outputs bit-exact, gathers bit-exact (same
per-element expression), scatter sums to 1e-6 relative (summation order only,
as the reference's own float atomics).  Everything goes through the reference
entry-point names on pcfm.ops with CPU tensors.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from pcfm import ops

RNG = np.random.default_rng(20261016)


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def _close(got, exp, rtol=1e-6, atol=1e-6):
    np.testing.assert_allclose(got.numpy() if isinstance(got, torch.Tensor) else got, exp,
                               rtol=rtol, atol=atol)


VOX_CASES = [(2, 5, 300, 8), (1, 3, 1, 4), (3, 16, 1000, 1), (2, 4, 2000, 32), (1, 2, 0, 4),
             (2, 7, 513, 100)]


@pytest.mark.parametrize("b,c,n,r", VOX_CASES)
def test_avg_voxelize_fwd_bwd(b, c, n, r):
    feat = RNG.standard_normal((b, c, n)).astype(np.float32)
    vc = RNG.integers(0, r, (b, 3, n)).astype(np.int32)
    out, ind, cnt = ops.avg_voxelize_forward(_t(feat), _t(vc), r)
    e_out, e_ind, e_cnt = O.avg_voxelize_fwd(feat, vc, r)
    assert np.array_equal(ind.numpy(), e_ind) and np.array_equal(cnt.numpy(), e_cnt)
    _close(out, e_out)
    gy = RNG.standard_normal((b, c, r ** 3)).astype(np.float32)
    gx = ops.avg_voxelize_backward(_t(gy), ind, cnt)
    assert np.array_equal(gx.numpy(), O.avg_voxelize_bwd(gy, e_ind, e_cnt))  # pure gather


@pytest.mark.parametrize("b,c,n,r", VOX_CASES)
@pytest.mark.parametrize("training", [True, False])
def test_trilinear_devoxelize_fwd_bwd(b, c, n, r, training):
    pts = (RNG.random((b, 3, n)) * (r - 1)).astype(np.float32)
    if n > 4:  # integer coordinates hit the x_hi = x_lo sentinel (trilinear_devox.cu:64-75)
        pts[:, :, :4] = np.round(pts[:, :, :4])
    grid = RNG.standard_normal((b, c, r ** 3)).astype(np.float32)
    o, i, w = ops.trilinear_devoxelize_forward(r, training, _t(pts), _t(grid))
    e_o, e_i, e_w = O.trilinear_devoxelize_fwd(pts, grid, r, training)
    _close(o, e_o, rtol=2e-7, atol=1e-7)
    if not training:
        assert i.shape == (1,) and w.shape == (1,)
        return
    assert np.array_equal(i.numpy(), e_i) and np.array_equal(w.numpy(), e_w)
    gy = RNG.standard_normal((b, c, n)).astype(np.float32)
    gx = ops.trilinear_devoxelize_backward(_t(gy), i, w, r)
    _close(gx, O.trilinear_devoxelize_bwd(gy, e_i, e_w, r), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("b,m,n,radius,u", [(2, 64, 500, 0.3, 16), (1, 5, 40, 10.0, 8),
                                             (2, 33, 100, 1e-3, 4), (1, 7, 0, 0.5, 3),
                                             (3, 100, 257, 0.5, 64), (1, 10, 20, 0.8, 32)])
def test_ball_query_bit_exact(b, m, n, radius, u):
    pts = RNG.random((b, 3, n)).astype(np.float32)
    centers = RNG.random((b, 3, m)).astype(np.float32)
    if n >= m:  # centers on points: d^2 = 0 is a hit
        centers[:, :, : m // 2] = pts[:, :, : m // 2]
    idx = ops.ball_query(_t(centers), _t(pts), radius, u)
    assert np.array_equal(idx.numpy(), O.ball_query(centers, pts, radius, u))


@pytest.mark.parametrize("b,c,n,m,u", [(2, 5, 100, 30, 8), (1, 1, 7, 3, 2), (2, 3, 50, 0, 4)])
def test_grouping_fwd_bwd(b, c, n, m, u):
    feat = RNG.standard_normal((b, c, n)).astype(np.float32)
    idx = RNG.integers(0, n, (b, m, u)).astype(np.int32)
    out = ops.grouping_forward(_t(feat), _t(idx))
    assert np.array_equal(out.numpy(), O.grouping_fwd(feat, idx))
    gy = RNG.standard_normal((b, c, m, u)).astype(np.float32)
    gx = ops.grouping_backward(_t(gy), _t(idx), n)
    _close(gx, O.grouping_bwd(gy, idx, n), rtol=1e-5, atol=1e-6)


def _chamfer_cpu(a, c):
    from chamfer3D.dist_chamfer_3D import chamfer_3DDist
    x1 = _t(a).requires_grad_(True)
    x2 = _t(c).requires_grad_(True)
    d1, d2, i1, i2 = chamfer_3DDist()(x1, x2)
    return x1, x2, d1, d2, i1, i2


@pytest.mark.parametrize("case", ["unit", "wide", "small", "ties", "timing_shape"])
def test_chamfer_against_reference_fixture(golden, case):
    """chamfer_python.distChamfer outputs (the reference's own CUDA-test oracle)."""
    g = golden("chamfer_python.npz")
    a, c = g[f"{case}_xyz1"], g[f"{case}_xyz2"]
    _, _, d1, d2, i1, i2 = _chamfer_cpu(a, c)
    assert np.array_equal(i1.numpy(), g[f"{case}_idx1"])
    assert np.array_equal(i2.numpy(), g[f"{case}_idx2"])
    # unit_test.py:23-34 asserts mean squared difference < 1e-8
    assert np.mean((d1.detach().numpy() - g[f"{case}_dist1"]) ** 2) < 1e-8
    assert np.mean((d2.detach().numpy() - g[f"{case}_dist2"]) ** 2) < 1e-8


@pytest.mark.parametrize("b,n,m", [(2, 300, 200), (1, 1, 5), (3, 64, 64)])
def test_chamfer_fwd_bwd_against_oracle(b, n, m):
    a = RNG.standard_normal((b, n, 3)).astype(np.float32)
    c = RNG.standard_normal((b, m, 3)).astype(np.float32)
    c[:, :2] = a[:, :2]  # exact hits: distance 0
    x1, x2, d1, d2, i1, i2 = _chamfer_cpu(a, c)
    e = O.chamfer_fwd(a, c)
    for got, exp in zip((d1, d2, i1, i2), e):
        assert np.array_equal(got.detach().numpy(), exp)  # same fma contract: bit-exact
    gd1 = RNG.standard_normal((b, n)).astype(np.float32)
    gd2 = RNG.standard_normal((b, m)).astype(np.float32)
    torch.autograd.backward([d1, d2], [_t(gd1), _t(gd2)])
    e1, e2 = O.chamfer_bwd(a, c, gd1, gd2, e[2], e[3])
    _close(x1.grad, e1, rtol=1e-5, atol=1e-6)
    _close(x2.grad, e2, rtol=1e-5, atol=1e-6)


def test_chamfer_self_distance_is_zero():
    """README.md:116-133: CD(x, x) = 0 with idx = identity for distinct points."""
    a = RNG.standard_normal((2, 2048, 3)).astype(np.float32)
    _, _, d1, d2, i1, i2 = _chamfer_cpu(a, a)
    assert float(d1.detach().abs().max()) == 0.0 and float(d2.detach().abs().max()) == 0.0
    ar = np.arange(2048)
    assert np.array_equal(i1.numpy()[0], ar) and np.array_equal(i2.numpy()[1], ar)


def test_emd_known_answer(golden):
    """PyTorchEMD/test_emd_loss.py: EMD = exact assignment (0.355 per element)."""
    from PyTorchEMD.emd import earth_mover_distance
    g = golden("emd_known.npz")
    p1 = _t(g["p1"]).requires_grad_(True)
    p2 = _t(g["p2"]).requires_grad_(True)
    d = earth_mover_distance(p1, p2, transpose=False)
    _close(d.detach(), g["gt_per_element"], rtol=1e-4, atol=1e-6)
    (d * _t(g["weights"])).sum().backward()
    # the script's ground truth weights the unnormalised pair cost: d(loss) = gt / N
    _close(p1.grad, g["gt_grad1"] / 2, rtol=1e-3, atol=1e-5)
    _close(p2.grad, g["gt_grad2"] / 2, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("b,n,m", [(2, 40, 40), (1, 30, 70), (2, 64, 16)])
def test_emd_against_oracle(dtype, b, n, m):
    a = RNG.random((b, n, 3)).astype(dtype)
    c = RNG.random((b, m, 3)).astype(dtype)
    match = ops.approxmatch_forward(_t(a), _t(c))
    e_match = O.emd_approxmatch(a, c)
    # the oracle evaluates exp in float (the reference's __expf); relative 1e-4
    _close(match, e_match, rtol=1e-3, atol=5e-5)
    cost = ops.matchcost_forward(_t(a), _t(c), match)
    _close(cost, O.emd_matchcost(a, c, e_match), rtol=1e-4, atol=1e-6)
    gc = RNG.random((b,)).astype(dtype)
    g1, g2 = ops.matchcost_backward(_t(gc), _t(a), _t(c), match)
    e1, e2 = O.emd_matchcost_bwd(gc, a, c, e_match)
    _close(g1, e1, rtol=1e-3, atol=1e-4)
    _close(g2, e2, rtol=1e-3, atol=1e-4)
