"""The CPU oracle against the reference's own fixtures and known answers.

This is what pins the oracle before it is trusted as the GPU checker
(DESIGN.md "Oracle").  Runs on the CPU (no GPU marker).
"""
import numpy as np
import pytest

from oracle import oracle as O

CHAMFER_CASES = ["unit", "wide", "small", "timing_shape", "ties"]


@pytest.mark.parametrize("case", CHAMFER_CASES)
def test_chamfer_oracle_matches_reference_python(golden, case):
    """unit_test.py:23-34: mean squared dist error < 1e-8 and identical indices."""
    g = golden("chamfer_python.npz")
    a, c = g[f"{case}_xyz1"], g[f"{case}_xyz2"]
    if case == "timing_shape":  # keep the CPU suite fast: first batch element only
        a, c = a[:1], c[:1]
        sl = np.s_[:1]
    else:
        sl = np.s_[:]
    d1, d2, i1, i2 = O.chamfer_fwd(a, c)
    assert np.mean((d1 - g[f"{case}_dist1"][sl]) ** 2) + np.mean((d2 - g[f"{case}_dist2"][sl]) ** 2) < 1e-8
    np.testing.assert_array_equal(i1, g[f"{case}_idx1"][sl])
    np.testing.assert_array_equal(i2, g[f"{case}_idx2"][sl])


def test_chamfer_self_is_zero_identity():
    """README.md:116-133: CD(x, x) = 0; for distinct points idx = identity."""
    x = np.random.default_rng(0).standard_normal((2, 2048, 3)).astype(np.float32)
    d1, d2, i1, i2 = O.chamfer_fwd(x, x)
    assert np.all(d1 == 0) and np.all(d2 == 0)
    np.testing.assert_array_equal(i1, np.broadcast_to(np.arange(2048), (2, 2048)))
    np.testing.assert_array_equal(i2, i1)


def test_chamfer_bwd_matches_autograd_formula():
    rng = np.random.default_rng(1)
    a = rng.random((2, 50, 3), dtype=np.float32)
    c = rng.random((2, 40, 3), dtype=np.float32)
    d1, d2, i1, i2 = O.chamfer_fwd(a, c)
    gd1 = rng.random(d1.shape, dtype=np.float32)
    gd2 = rng.random(d2.shape, dtype=np.float32)
    g1, g2 = O.chamfer_bwd(a, c, gd1, gd2, i1, i2)
    e1 = np.zeros_like(a)
    e2 = np.zeros_like(c)
    for b in range(2):
        for j in range(50):
            t = 2 * gd1[b, j] * (a[b, j] - c[b, i1[b, j]])
            e1[b, j] += t
            e2[b, i1[b, j]] -= t
        for j in range(40):
            t = 2 * gd2[b, j] * (c[b, j] - a[b, i2[b, j]])
            e2[b, j] += t
            e1[b, i2[b, j]] -= t
    np.testing.assert_allclose(g1, e1, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(g2, e2, rtol=1e-5, atol=1e-6)


def test_emd_oracle_known_answer(golden):
    """test_emd_loss.py: approx EMD ~= exact assignment cost on well-separated pairs."""
    g = golden("emd_known.npz")
    for dt in (np.float32, np.float64):
        p1, p2 = g["p1"].astype(dt), g["p2"].astype(dt)
        match = O.emd_approxmatch(p1, p2)
        cost = O.emd_matchcost(p1, p2, match)
        emd = cost / p1.shape[1]
        np.testing.assert_allclose(emd, g["gt_per_element"], rtol=1e-4)
        # match is (numerically) the permutation [[0,1],[1,0]]
        np.testing.assert_allclose(match[0], [[0, 1], [1, 0]], atol=1e-6)
        # the script's loss is sum_b w_b * emd_b with emd = cost / N (N = 2); its
        # ground truth weights the UNnormalised pair cost, so d(loss) = gt_grad / N
        w = g["weights"].astype(dt)
        g1, g2 = O.emd_matchcost_bwd(w / p1.shape[1], p1, p2, match)
        np.testing.assert_allclose(g1, g["gt_grad1"] / 2, rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(g2, g["gt_grad2"] / 2, rtol=1e-4, atol=1e-5)


def test_emd_match_marginals():
    """Approxmatch transports at most multiL/multiR mass per point (emd_kernel.cu:27-33)."""
    rng = np.random.default_rng(3)
    a = rng.random((2, 64, 3), dtype=np.float32)
    c = rng.random((2, 32, 3), dtype=np.float32)
    match = O.emd_approxmatch(a, c)  # (b, m, n), n=64 >= m=32 -> multiR = 2
    assert match.shape == (2, 32, 64)
    assert np.all(match >= 0)
    assert np.all(match.sum(axis=1) <= 1 + 1e-4)      # each xyz1 point: <= multiL = 1
    assert np.all(match.sum(axis=2) <= 2 + 1e-4)      # each xyz2 point: <= multiR = 2
    assert match.sum() > 0.9 * 2 * 64


def test_avg_voxelize_known_answer():
    # 4 points; points 0,1,3 share voxel (1,0,1) at r=2, point 2 alone in (0,1,0)
    feat = np.array([[[1, 2, 3, 4], [10, 20, 30, 40]]], np.float32)
    coords = np.array([[[1, 1, 0, 1], [0, 0, 1, 0], [1, 1, 0, 1]]], np.int32)
    out, ind, cnt = O.avg_voxelize_fwd(feat, coords, 2)
    v_a, v_b = 1 * 4 + 0 * 2 + 1, 0 * 4 + 1 * 2 + 0
    np.testing.assert_array_equal(ind[0], [v_a, v_a, v_b, v_a])
    assert cnt[0, v_a] == 3 and cnt[0, v_b] == 1 and cnt.sum() == 4
    np.testing.assert_allclose(out[0, :, v_a], [(1 + 2 + 4) / 3, (10 + 20 + 40) / 3], rtol=1e-6)
    np.testing.assert_allclose(out[0, :, v_b], [3, 30])
    assert np.count_nonzero(out) == 4
    gy = np.arange(2 * 8, dtype=np.float32).reshape(1, 2, 8)
    gx = O.avg_voxelize_bwd(gy, ind, cnt)
    np.testing.assert_allclose(gx[0, 0], [gy[0, 0, v_a] / 3] * 2 + [gy[0, 0, v_b]] + [gy[0, 0, v_a] / 3])


def test_devoxelize_known_answer():
    r = 4
    grid = np.random.default_rng(5).random((1, 3, r ** 3), dtype=np.float32)
    # integer coords reproduce the grid exactly; fraction 0 -> hi == lo (trilinear_devox.cu:64-75)
    pts = np.array([[[0, 3, 1.0], [2, 0, 3.0], [1, 3, 0.0]]], np.float32)
    out, inds, wgts = O.trilinear_devoxelize_fwd(pts, grid, r)
    for i in range(3):
        v = int(pts[0, 0, i]) * 16 + int(pts[0, 1, i]) * 4 + int(pts[0, 2, i])
        np.testing.assert_array_equal(out[0, :, i], grid[0, :, v])
        assert np.all(inds[0, :, i] == v)
        assert wgts[0, 0, i] == 1.0 and np.all(wgts[0, 1:, i] == 0)
    # midpoints average the 8 corners; weights always sum to 1
    pts = np.random.default_rng(6).random((1, 3, 100), dtype=np.float32) * (r - 1)
    out, inds, wgts = O.trilinear_devoxelize_fwd(pts, grid, r)
    np.testing.assert_allclose(wgts.sum(axis=1), 1.0, rtol=1e-6)
    ref = np.einsum("kn,ckn->cn", wgts[0], grid[0][:, inds[0]])
    np.testing.assert_allclose(out[0], ref, rtol=1e-5, atol=1e-6)
    # backward is the adjoint of forward: <devox(G), Y> == <G, devox^T(Y)>
    gy = np.random.default_rng(7).random(out.shape, dtype=np.float32)
    gx = O.trilinear_devoxelize_bwd(gy, inds, wgts, r)
    np.testing.assert_allclose((out * gy).sum(), (grid * gx).sum(), rtol=1e-5)


def test_ball_query_known_answer():
    pts = np.array([[[0, 1, 0.1, 5, 0.2], [0, 0, 0, 0, 0], [0, 0, 0, 0, 0]]], np.float32)
    ctr = np.array([[[0, 4.8], [0, 0], [0, 0]]], np.float32)
    idx = O.ball_query(ctr, pts, 0.5, 4)
    np.testing.assert_array_equal(idx[0, 0], [0, 2, 4, 0])   # 3 hits in index order, pad first
    np.testing.assert_array_equal(idx[0, 1], [3, 3, 3, 3])   # 1 hit
    idx = O.ball_query(ctr, pts, 0.01, 3)
    np.testing.assert_array_equal(idx[0, 1], [0, 0, 0])      # no hit -> zeros
    idx = O.ball_query(ctr, pts, 10.0, 2)                    # more hits than u
    np.testing.assert_array_equal(idx[0, 0], [0, 1])


def test_grouping_roundtrip():
    rng = np.random.default_rng(8)
    feat = rng.random((2, 5, 30), dtype=np.float32)
    idx = rng.integers(0, 30, (2, 7, 4)).astype(np.int32)
    out = O.grouping_fwd(feat, idx)
    np.testing.assert_array_equal(out, np.take_along_axis(feat[:, :, None, :].repeat(7, 2),
                                                          idx[:, None].repeat(5, 1), 3))
    gy = rng.random(out.shape, dtype=np.float32)
    gx = O.grouping_bwd(gy, idx, 30)
    np.testing.assert_allclose((out * gy).sum(), (feat * gx).sum(), rtol=1e-5)


# --- outside pins: third-party implementations of the same arithmetic --------
# The reference holds no fixtures for the PVCNN kernels and its CUDA cannot run
# here, so these pin the oracle against PyTorch's own algorithms instead.

def test_devoxelize_fwd_bwd_match_grid_sample():
    import torch
    from golden_util import grid_sample_devox as _grid_sample_devox
    rng = np.random.default_rng(11)
    for r, n in ((8, 3000), (5, 500)):
        grid = rng.standard_normal((2, 6, r ** 3)).astype(np.float32)
        pts = (rng.random((2, 3, n)) * (r - 1)).astype(np.float32)
        pts[:, :, :8] = np.round(pts[:, :, :8])       # on-lattice points, incl. the r-1 face
        pts[:, 0, 8] = r - 1
        out, inds, wgts = O.trilinear_devoxelize_fwd(pts, grid, r)
        tg = torch.from_numpy(grid).double().requires_grad_(True)
        ref = _grid_sample_devox(tg, torch.from_numpy(pts).double(), r)
        np.testing.assert_allclose(out, ref.detach().numpy(), rtol=1e-5, atol=1e-5)
        gy = rng.standard_normal(out.shape).astype(np.float32)
        (gref,) = torch.autograd.grad(ref, tg, torch.from_numpy(gy).double())
        gx = O.trilinear_devoxelize_bwd(gy, inds, wgts, r)
        np.testing.assert_allclose(gx, gref.numpy(), rtol=1e-5, atol=1e-4)


def test_avg_voxelize_matches_scatter_reduce_mean():
    import torch
    rng = np.random.default_rng(12)
    r, b, c, n = 6, 2, 5, 2000
    coords = rng.integers(0, r, (b, 3, n)).astype(np.int32)
    feat = rng.standard_normal((b, c, n)).astype(np.float32)
    out, ind, cnt = O.avg_voxelize_fwd(feat, coords, r)
    lin = torch.from_numpy(coords).long()
    lin = lin[:, 0] * r * r + lin[:, 1] * r + lin[:, 2]                  # vox.cu:24-30
    np.testing.assert_array_equal(ind, lin.int().numpy())
    np.testing.assert_array_equal(cnt, torch.stack([torch.bincount(l, minlength=r ** 3)
                                                    for l in lin]).int().numpy())
    ref = torch.zeros(b, c, r ** 3, dtype=torch.float64).scatter_reduce(
        2, lin[:, None].expand(b, c, n), torch.from_numpy(feat).double(), "mean",
        include_self=False)
    np.testing.assert_allclose(out, ref.numpy(), rtol=1e-5, atol=1e-6)
    gy = rng.standard_normal(out.shape).astype(np.float32)
    gx = O.avg_voxelize_bwd(gy, ind, cnt)
    c64 = torch.from_numpy(cnt).double().clamp_min(1)
    gref = torch.gather(torch.from_numpy(gy).double() / c64[:, None], 2, lin[:, None].expand(b, c, n))
    np.testing.assert_allclose(gx, gref.numpy(), rtol=1e-6, atol=1e-7)
