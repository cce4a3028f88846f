"""GPU parity: every hot-path op through the C ABI against the CPU oracle and the
reference's fixtures.

Bar (DESIGN.md "Parity"):
  * integer / index outputs (ind, cnt, inds, ball-query and nearest-neighbour
    indices): bit-exact;
  * deterministic float outputs (devox forward, voxelize backward, grouping
    forward, Chamfer distances): bit-exact -- same fp contract as the oracle;
  * float sums whose order the reference leaves to atomics (voxelize forward,
    devox / grouping backward, Chamfer backward): rtol 1e-5 (atol 1e-6 ... scaled
    to the summand magnitude);
  * EMD (reference built with --use_fast_math, hardware exp): rtol 1e-4.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _native():
    from pcfm import _lib
    _lib.load()
    assert torch.cuda.is_available()


def rng(seed):
    return np.random.default_rng(seed)


def cu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def np_(t):
    return t.detach().cpu().numpy()


# ------------------------------------------------------------------ voxelize
VOX_CASES = [
    # b, c, n, r, layout
    (2, 4, 100, 2, "uniform"),
    (3, 16, 1000, 8, "uniform"),
    (2, 64, 5000, 16, "clustered"),
    (2, 128, 20000, 32, "clustered"),
    (1, 3, 4000, 64, "uniform"),     # r^3 > LDS row: chunked path
    (2, 2, 3000, 100, "uniform"),    # sort blocks each span > LDS: multi-pass per block
    (2, 5, 300, 4, "one_voxel"),     # every point in one voxel
    (1, 7, 0, 4, "uniform"),         # empty cloud
    (2, 3, 17, 1, "uniform"),        # r = 1
]


def vox_coords(g, b, n, r, layout):
    if layout == "uniform":
        return g.integers(0, r, (b, 3, n)).astype(np.int32)
    if layout == "one_voxel":
        return np.full((b, 3, n), r // 2, np.int32)
    c = np.clip(np.round(g.normal(r / 2, r / 8, (b, 3, n))), 0, r - 1)
    return c.astype(np.int32)


@pytest.mark.parametrize("b,c,n,r,layout", VOX_CASES)
def test_avg_voxelize(b, c, n, r, layout):
    from pcfm import ops
    g = rng(b * 1000 + c + n + r)
    feat = g.standard_normal((b, c, n)).astype(np.float32)
    coords = vox_coords(g, b, n, r, layout)
    out, ind, cnt = ops.avg_voxelize_forward(cu(feat), cu(coords), r)
    e_out, e_ind, e_cnt = O.avg_voxelize_fwd(feat, coords, r)
    np.testing.assert_array_equal(np_(ind), e_ind)
    np.testing.assert_array_equal(np_(cnt), e_cnt)
    # the sort is stable: a voxel's items are summed in index order, as the
    # oracle's sequential loop does -- bit-exact unless a 16-voxel tile holds more
    # than one work unit (256 items), whose partial sums are added at the end
    v = r ** 3
    per_tile = np.add.reduceat(e_cnt, np.arange(0, v, 16), axis=1) if v else e_cnt
    if per_tile.size == 0 or per_tile.max() <= 256:
        np.testing.assert_array_equal(np_(out), e_out)
    else:
        np.testing.assert_allclose(np_(out), e_out, rtol=1e-5, atol=1e-6)
    gy = g.standard_normal((b, c, r ** 3)).astype(np.float32)
    gx = ops.avg_voxelize_backward(cu(gy), ind, cnt)
    np.testing.assert_array_equal(np_(gx), O.avg_voxelize_bwd(gy, e_ind, e_cnt))


# ---------------------------------------------------------------- devoxelize
DEVOX_CASES = [
    (2, 4, 100, 2), (3, 16, 1000, 8), (2, 256, 20000, 8), (2, 256, 20000, 16),
    (2, 128, 20000, 32), (1, 3, 3000, 64), (1, 5, 0, 4), (2, 3, 50, 1), (1, 2, 2000, 100),
]


def devox_coords(g, b, n, r):
    pts = (g.random((b, 3, n)) * (r - 1)).astype(np.float32)
    if n >= 8:  # integer coordinates and the upper boundary r-1 (hi == lo)
        pts[:, :, : n // 8] = np.round(pts[:, :, : n // 8])
        pts[:, :, -1] = r - 1
    return pts


@pytest.mark.parametrize("b,c,n,r", DEVOX_CASES)
@pytest.mark.parametrize("training", [True, False])
def test_trilinear_devoxelize(b, c, n, r, training):
    from pcfm import ops
    g = rng(b * 7 + c + n + r)
    pts = devox_coords(g, b, n, r)
    grid = g.standard_normal((b, c, r ** 3)).astype(np.float32)
    out, inds, wgts = ops.trilinear_devoxelize_forward(r, training, cu(pts), cu(grid))
    e_out, e_inds, e_wgts = O.trilinear_devoxelize_fwd(pts, grid, r, training)
    np.testing.assert_array_equal(np_(out), e_out)          # bit-exact (same fma order)
    if not training:
        assert inds.shape == (1,) and wgts.shape == (1,)
        return
    np.testing.assert_array_equal(np_(inds), e_inds)
    np.testing.assert_array_equal(np_(wgts), e_wgts)
    gy = g.standard_normal((b, c, n)).astype(np.float32)
    gx = ops.trilinear_devoxelize_backward(cu(gy), inds, wgts, r)
    e_gx = O.trilinear_devoxelize_bwd(gy, e_inds, e_wgts, r)
    scale = max(1.0, float(np.abs(e_gx).max()))
    np.testing.assert_allclose(np_(gx), e_gx, rtol=1e-5, atol=1e-6 * scale)


@pytest.mark.parametrize("r,c", [(8, 256), (16, 64), (32, 8)])
def test_devox_coords_outside_the_volume(r, c):
    """Coordinates outside [0, r-1]: a corner whose linear index leaves [0, r^3)
    contributes 0 (the oracle; the backward's stored-pair check), the stored
    pairs stay the reference's unclamped ones, and forward and backward agree
    (the backward is the forward's adjoint on every point).  One shape per
    gather form: 4-channel (r 8, 16), 1-channel (r 32)."""
    from pcfm import ops
    g = rng(900 + r)
    b, n = 2, 3000
    pts = (g.random((b, 3, n)) * (r + 3) - 1.5).astype(np.float32)  # ~30 % outside
    grid = g.standard_normal((b, c, r ** 3)).astype(np.float32)
    out, inds, wgts = ops.trilinear_devoxelize_forward(r, True, cu(pts), cu(grid))
    e_out, e_inds, e_wgts = O.trilinear_devoxelize_fwd(pts, grid, r, True)
    np.testing.assert_array_equal(np_(inds), e_inds)
    np.testing.assert_array_equal(np_(wgts), e_wgts)
    np.testing.assert_array_equal(np_(out), e_out)
    eval_out, _, _ = ops.trilinear_devoxelize_forward(r, False, cu(pts), cu(grid))
    np.testing.assert_array_equal(np_(eval_out), e_out)
    scale = torch.rand(b, c, device=DEV)
    add = torch.randn(b, c, n, device=DEV)
    o2, _, _ = ops.trilinear_devoxelize_scale_add(r, True, cu(pts), cu(grid), scale, add)
    ref2 = torch.from_numpy(e_out).to(DEV) * scale[:, :, None] + add
    torch.testing.assert_close(o2, ref2, rtol=0, atol=0)
    gy = g.standard_normal((b, c, n)).astype(np.float32)
    gx = ops.trilinear_devoxelize_backward(cu(gy), inds, wgts, r)
    lhs = float((np_(out).astype(np.float64) * gy).sum())
    rhs = float((grid.astype(np.float64) * np_(gx)).sum())
    assert abs(lhs - rhs) <= 1e-5 * max(1.0, abs(lhs)), (lhs, rhs)


def test_devox_full_size_properties():
    """C2 stage-1 size: forward linear in the grid, backward its adjoint."""
    from pcfm import ops
    b, c, n, r = 8, 128, 20000, 32
    g = torch.Generator(device=DEV).manual_seed(3)
    pts = torch.rand(b, 3, n, device=DEV, generator=g) * (r - 1)
    grid = torch.randn(b, c, r ** 3, device=DEV, generator=g)
    out, inds, wgts = ops.trilinear_devoxelize_forward(r, True, pts, grid)
    out2, _, _ = ops.trilinear_devoxelize_forward(r, True, pts, 2.0 * grid)
    assert torch.equal(out2, 2.0 * out)                       # exact: scaling by 2
    gy = torch.randn(b, c, n, device=DEV, generator=g)
    gx = ops.trilinear_devoxelize_backward(gy, inds, wgts, r)
    lhs = (out.double() * gy.double()).sum()
    rhs = (grid.double() * gx.double()).sum()
    assert abs(lhs - rhs) <= 1e-4 * abs(lhs)
    assert torch.allclose(wgts.sum(1), torch.ones_like(wgts[:, 0]), atol=1e-6)


@pytest.mark.parametrize("c,r", [(128, 32), (256, 16), (256, 8)])
def test_devox_c2_matches_grid_sample(c, r):
    """Outside pin at the C2 stage shapes: the devox kernels against PyTorch's
    own trilinear interpolation (grid_sample, align_corners=True, fp64) and its
    autograd adjoint; plus the product's SE-scale + point-branch gather
    (out = s * devox(grid) + pf)."""
    from pcfm import ops
    from golden_util import grid_sample_devox as _grid_sample_devox
    b, n = 8, 20000
    g = torch.Generator(device=DEV).manual_seed(r)
    pts = torch.rand(b, 3, n, device=DEV, generator=g) * (r - 1)
    pts[:, :, :64] = pts[:, :, :64].round()
    grid = torch.randn(b, c, r ** 3, device=DEV, generator=g)
    out, inds, wgts = ops.trilinear_devoxelize_forward(r, True, pts, grid)
    tg = grid.double().requires_grad_(True)
    ref = _grid_sample_devox(tg, pts.double(), r)
    torch.testing.assert_close(out.double(), ref.detach(), rtol=1e-5, atol=1e-5)
    gy = torch.randn(b, c, n, device=DEV, generator=g)
    (gref,) = torch.autograd.grad(ref, tg, gy.double())
    gx = ops.trilinear_devoxelize_backward(gy, inds, wgts, r)
    torch.testing.assert_close(gx.double(), gref, rtol=1e-5, atol=1e-4)
    s = torch.rand(b, c, device=DEV, generator=g)
    pf = torch.randn(b, c, n, device=DEV, generator=g)
    fused, _, _ = ops.trilinear_devoxelize_scale_add(r, False, pts, grid, s, pf)
    torch.testing.assert_close(fused.double(), ref.detach() * s.double()[..., None] + pf.double(),
                               rtol=1e-5, atol=1e-5)


def test_voxelize_full_size_properties():
    from pcfm import ops
    b, c, n, r = 8, 128, 20000, 32
    g = torch.Generator(device=DEV).manual_seed(4)
    coords = torch.randint(0, r, (b, 3, n), device=DEV, generator=g, dtype=torch.int32)
    feat = torch.randn(b, c, n, device=DEV, generator=g)
    out, ind, cnt = ops.avg_voxelize_forward(feat, coords, r)
    assert int(cnt.sum()) == b * n
    # sum_v out[c,v]*cnt[v] == sum_i feat[c,i]
    lhs = (out.double() * cnt[:, None, :].double()).sum(-1)
    rhs = feat.double().sum(-1)
    assert torch.allclose(lhs, rhs, rtol=1e-5, atol=1e-3)
    # determinism of the integer outputs across calls
    out2, ind2, cnt2 = ops.avg_voxelize_forward(feat, coords, r)
    assert torch.equal(ind, ind2) and torch.equal(cnt, cnt2)


@pytest.mark.parametrize("c,r", [(128, 32), (256, 16), (256, 8)])
def test_scatters_deterministic_c2(c, r):
    """The stable sort + fixed-order sums: two calls at a C2 stage shape return
    identical bits (voxelize forward, devoxelize backward, grouping backward)."""
    from pcfm import ops
    b, n = 8, 20000
    g = torch.Generator(device=DEV).manual_seed(c + r)
    x = torch.randn(b, 3, n, device=DEV, generator=g)
    x = x - x.mean(2, keepdim=True)
    x = x / (x.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values * 2.0 + 1e-6) + 0.5
    nc = torch.clamp(x * r, 0, r - 1)
    vc = torch.round(nc).to(torch.int32)
    feat = torch.randn(b, c, n, device=DEV, generator=g)
    o1, _, _ = ops.avg_voxelize_forward(feat, vc, r)
    o2, _, _ = ops.avg_voxelize_forward(feat, vc, r)
    assert torch.equal(o1, o2)
    grid = torch.randn(b, c, r ** 3, device=DEV, generator=g)
    _, inds, wgts = ops.trilinear_devoxelize_forward(r, True, nc, grid)
    g1 = ops.trilinear_devoxelize_backward(feat, inds, wgts, r)
    g2 = ops.trilinear_devoxelize_backward(feat, inds, wgts, r)
    assert torch.equal(g1, g2)
    idx = torch.randint(0, n, (b, 512, 32), device=DEV, generator=g, dtype=torch.int32)
    gy = torch.randn(b, 16, 512, 32, device=DEV, generator=g)
    assert torch.equal(ops.grouping_backward(gy, idx, n), ops.grouping_backward(gy, idx, n))


# -------------------------------------------------------- ball query, grouping
@pytest.mark.parametrize("b,m,n,radius,u", [(2, 64, 1000, 0.2, 16), (1, 500, 4096, 0.1, 32),
                                            (3, 7, 50, 10.0, 8), (2, 33, 100, 1e-4, 4),
                                            (1, 300, 0, 0.5, 3), (2, 17, 5000, 0.3, 100),
                                            (1, 40, 2049, 2.0, 70), (1, 3, 9000, 0.05, 1)])
def test_ball_query(b, m, n, radius, u):
    from pcfm import ops
    g = rng(m + n + u)
    pts = g.random((b, 3, n)).astype(np.float32)
    ctr = g.random((b, 3, m)).astype(np.float32)
    if n > 0:
        ctr[:, :, : m // 4] = pts[:, :, : m // 4]  # centers on points: d2 == 0 hits
    idx = ops.ball_query(cu(ctr), cu(pts), radius, u)
    np.testing.assert_array_equal(np_(idx), O.ball_query(ctr, pts, radius, u))


@pytest.mark.parametrize("b,c,n,m,u", [(2, 16, 1000, 64, 16), (1, 128, 20000, 512, 32),
                                       (2, 3, 10, 5, 4), (1, 4, 40000, 100, 8)])
def test_grouping(b, c, n, m, u):
    from pcfm import ops
    g = rng(c + n + m + u)
    feat = g.standard_normal((b, c, n)).astype(np.float32)
    idx = g.integers(0, n, (b, m, u)).astype(np.int32)
    out = ops.grouping_forward(cu(feat), cu(idx))
    np.testing.assert_array_equal(np_(out), O.grouping_fwd(feat, idx))
    gy = g.standard_normal((b, c, m, u)).astype(np.float32)
    gx = ops.grouping_backward(cu(gy), cu(idx), n)
    np.testing.assert_allclose(np_(gx), O.grouping_bwd(gy, idx, n), rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------- chamfer
@pytest.mark.parametrize("case", ["unit", "wide", "small", "timing_shape", "ties"])
def test_chamfer_reference_fixtures(golden, case):
    """The reference's own unit-test bar (unit_test.py:23-34) against
    chamfer_python.distChamfer outputs, plus bit-equality with the oracle."""
    from chamfer3D.dist_chamfer_3D import chamfer_3DDist
    g = golden("chamfer_python.npz")
    a, c = g[f"{case}_xyz1"], g[f"{case}_xyz2"]
    d1, d2, i1, i2 = chamfer_3DDist()(cu(a), cu(c))
    assert (np.mean((np_(d1) - g[f"{case}_dist1"]) ** 2)
            + np.mean((np_(d2) - g[f"{case}_dist2"]) ** 2)) < 1e-8
    np.testing.assert_array_equal(np_(i1), g[f"{case}_idx1"])
    np.testing.assert_array_equal(np_(i2), g[f"{case}_idx2"])
    e = O.chamfer_fwd(a, c)
    np.testing.assert_array_equal(np_(d1), e[0])
    np.testing.assert_array_equal(np_(d2), e[1])


@pytest.mark.parametrize("b,n,m", [(1, 1, 1), (2, 5000, 3000), (8, 2048, 2048), (1, 100, 0),
                                   (3, 777, 1025), (32, 2000, 1000)])
def test_chamfer_vs_oracle(b, n, m):
    from pcfm import ops
    g = rng(b + n + m)
    a = g.standard_normal((b, n, 3)).astype(np.float32)
    c = g.standard_normal((b, m, 3)).astype(np.float32)
    if n and m:
        c[:, : min(n, m) // 3] = a[:, : min(n, m) // 3]  # exact hits
    d1 = torch.empty(b, n, device=DEV)
    d2 = torch.empty(b, m, device=DEV)
    i1 = torch.empty(b, n, dtype=torch.int32, device=DEV)
    i2 = torch.empty(b, m, dtype=torch.int32, device=DEV)
    assert ops.chamfer_3D.forward(cu(a), cu(c), d1, d2, i1, i2) == 1
    e = O.chamfer_fwd(a, c)
    for got, exp in zip((d1, d2, i1, i2), e):
        np.testing.assert_array_equal(np_(got), exp)
    if n and m:
        gd1 = g.random((b, n)).astype(np.float32)
        gd2 = g.random((b, m)).astype(np.float32)
        g1 = torch.zeros(b, n, 3, device=DEV)
        g2 = torch.zeros(b, m, 3, device=DEV)
        assert ops.chamfer_3D.backward(cu(a), cu(c), g1, g2, cu(gd1), cu(gd2), i1, i2) == 1
        e1, e2 = O.chamfer_bwd(a, c, gd1, gd2, e[2], e[3])
        np.testing.assert_allclose(np_(g1), e1, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(np_(g2), e2, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case", ["randn", "ties", "clusters", "degenerate", "uneven"])
def test_chamfer_culled_bit_exact(case):
    """The Morton-sorted tile-culled search (forced on with
    PCFM_CHAMFER_CULL_PAIRS, set for the whole GPU test session in conftest)
    must return the brute-force answer -- every distance and index equal to
    the oracle's full scan, lowest index on ties."""
    import os
    assert os.environ.get("PCFM_CHAMFER_CULL_PAIRS") == str(16 << 20)
    from pcfm import ops
    g = rng(hash(case) % 1000)
    b, n, m = 2, 4500, 4000
    if case == "uneven":
        n, m = 300, 60000
    a = g.standard_normal((b, n, 3)).astype(np.float32)
    c = g.standard_normal((b, m, 3)).astype(np.float32)
    if case == "ties":  # exact duplicates at several indices, queries on points
        c[:, 1000:1500] = c[:, :500]
        c[:, 3000:3100] = c[:, :100]
        a[:, :700] = c[:, 800:1500]
    elif case == "clusters":
        a = (g.integers(0, 4, (b, n, 1)) * 10.0 + 0.01 * g.standard_normal((b, n, 3))).astype(
            np.float32)
        c = (g.integers(0, 4, (b, m, 1)) * 10.0 + 0.01 * g.standard_normal((b, m, 3))).astype(
            np.float32)
    elif case == "degenerate":  # one point repeated: zero extent, every distance tied
        a[:] = 0.5
        c[:] = 0.5
    d1 = torch.empty(b, n, device=DEV)
    d2 = torch.empty(b, m, device=DEV)
    i1 = torch.empty(b, n, dtype=torch.int32, device=DEV)
    i2 = torch.empty(b, m, dtype=torch.int32, device=DEV)
    assert ops.chamfer_3D.forward(cu(a), cu(c), d1, d2, i1, i2) == 1
    e = O.chamfer_fwd(a, c)
    for got, exp in zip((d1, d2, i1, i2), e):
        np.testing.assert_array_equal(np_(got), exp)


def test_chamfer_full_size_sampled():
    """C2 size (B=8, N=M=20000): a sample of queries checked bit-exactly against
    the oracle run on the full candidate cloud."""
    from pcfm import ops
    b, n = 8, 20000
    g = rng(11)
    a = g.standard_normal((b, n, 3)).astype(np.float32)
    c = g.standard_normal((b, n, 3)).astype(np.float32)
    d1 = torch.empty(b, n, device=DEV)
    d2 = torch.empty(b, n, device=DEV)
    i1 = torch.empty(b, n, dtype=torch.int32, device=DEV)
    i2 = torch.empty(b, n, dtype=torch.int32, device=DEV)
    assert ops.chamfer_3D.forward(cu(a), cu(c), d1, d2, i1, i2) == 1
    q = g.choice(n, 64, replace=False)
    for bb in (0, 5):
        e = O.chamfer_fwd(a[bb:bb + 1, q], c[bb:bb + 1])
        np.testing.assert_array_equal(np_(d1)[bb, q], e[0][0])
        np.testing.assert_array_equal(np_(i1)[bb, q], e[2][0])
        e = O.chamfer_fwd(c[bb:bb + 1, q], a[bb:bb + 1])
        np.testing.assert_array_equal(np_(d2)[bb, q], e[0][0])
        np.testing.assert_array_equal(np_(i2)[bb, q], e[2][0])


def test_chamfer_self_zero():
    from chamfer3D.dist_chamfer_3D import chamfer_3DDist
    x = torch.randn(2, 2048, 3, device=DEV)
    d1, d2, i1, i2 = chamfer_3DDist()(x, x)
    assert float(d1.abs().max()) == 0 and float(d2.abs().max()) == 0
    assert torch.equal(i1.long(), torch.arange(2048, device=DEV).expand(2, -1))


# ----------------------------------------------------------------------- EMD
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("b,n,m", [(2, 64, 64), (3, 100, 37), (2, 37, 100), (1, 513, 300)])
def test_emd_vs_oracle(dtype, b, n, m):
    from pcfm import ops
    g = rng(n * m)
    a = g.random((b, n, 3)).astype(dtype)
    c = g.random((b, m, 3)).astype(dtype)
    match = ops.approxmatch_forward(cu(a), cu(c))
    e_match = O.emd_approxmatch(a, c)
    # 10 levels x 3 passes of approximate exp (the reference's __expf; the oracle
    # uses libm expf) with min/max clamps in between: individual match entries
    # move by up to ~1e-4 absolute (entries are <= 1), the cost by < 1e-4 relative
    np.testing.assert_allclose(np_(match), e_match, rtol=1e-3, atol=5e-4)
    assert abs(np_(match).sum() - e_match.sum()) <= 1e-4 * e_match.sum()
    cost = ops.matchcost_forward(cu(a), cu(c), match)
    np.testing.assert_allclose(np_(cost), O.emd_matchcost(a, c, e_match), rtol=1e-4)
    # matchcost itself on identical inputs: summation order only
    np.testing.assert_allclose(np_(ops.matchcost_forward(cu(a), cu(c), cu(e_match))),
                               O.emd_matchcost(a, c, e_match), rtol=1e-5)
    gc = g.random(b).astype(dtype)
    g1, g2 = ops.matchcost_backward(cu(gc), cu(a), cu(c), cu(e_match))
    e1, e2 = O.emd_matchcost_bwd(gc, a, c, e_match)
    np.testing.assert_allclose(np_(g1), e1, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(np_(g2), e2, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("b,n,m", [(2, 64, 64), (3, 100, 37), (2, 37, 700), (8, 2048, 2048)])
def test_emd_fused_cost_matches_two_calls(dtype, b, n, m):
    """pcfm_emd_approxmatch_cost (the product forward of emd.py): the match
    it writes is bit-identical to approxmatch_forward's, its cost equals
    matchcost_forward on that match to summation order, and the cost-only form
    (no match written) returns the same bits (emd_kernel.cu:169-277)."""
    from pcfm import ops
    g = torch.Generator(device=DEV).manual_seed(n + m)
    a = torch.rand(b, n, 3, device=DEV, generator=g, dtype=dtype)
    c = torch.rand(b, m, 3, device=DEV, generator=g, dtype=dtype)
    match, cost = ops.approxmatch_cost_forward(a, c)
    assert torch.equal(match, ops.approxmatch_forward(a, c))
    ref = ops.matchcost_forward(a, c, match)
    torch.testing.assert_close(cost, ref, rtol=1e-5 if dtype == torch.float32 else 1e-12, atol=0)
    none, cost2 = ops.approxmatch_cost_forward(a, c, want_match=False)
    assert none is None and torch.equal(cost, cost2)


def test_emd_known_answer(golden):
    from PyTorchEMD.emd import earth_mover_distance
    g = golden("emd_known.npz")
    p1 = cu(g["p1"]).requires_grad_(True)
    p2 = cu(g["p2"]).requires_grad_(True)
    d = earth_mover_distance(p1, p2, transpose=False)
    np.testing.assert_allclose(np_(d), g["gt_per_element"], rtol=1e-4)
    loss = (d * cu(g["weights"])).sum()
    loss.backward()
    np.testing.assert_allclose(np_(p1.grad), g["gt_grad1"] / 2, rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(np_(p2.grad), g["gt_grad2"] / 2, rtol=1e-3, atol=1e-5)


def test_chamfer_c2_product_path(tmp_path, report):
    """The brute-force split-candidate Chamfer kernel the product runs at C2
    (B=8, N=M=20000), with the session's culling override removed: sampled
    queries bit-exact against the oracle's full scan (exact hits and duplicate
    candidates: lowest index on ties), backward within 1e-5
    (tests/helpers/chamfer_c2_product.py; chamfer3D.cu:12-174)."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k != "PCFM_CHAMFER_CULL_PAIRS"}
    out = tmp_path / "c2.json"
    subprocess.run([sys.executable, os.path.join(repo, "tests", "helpers",
                                                 "chamfer_c2_product.py"), str(out)],
                   check=True, timeout=240, env=env, cwd=repo)
    d = json.load(open(out))
    report("chamfer_c2_product_path", d)
    assert d["mismatches"] == {"d1": 0, "i1": 0, "d2": 0, "i2": 0}, d
    assert d["queries_checked"] == 8 * 2 * 400 and d["exact_hits"] >= 8 * 3000
    assert d["bwd_close"], d


def test_emd_rowpass_form_matches_split_form(tmp_path, report):
    """approxmatch's row-pass form (one launch per pass of each level, the
    finalize in the same block, the 16 column slices of a row summed in a fixed
    order; a level's third pass and the next level's first share one launch:
    21 launches; bit-identical to the unfused 31) against the split form (every pass and finalize its own
    launch, S-way partial sums: 62): the same matches to fp32 round-off over
    f32/f64, n >< m and ragged sizes (tests/helpers/emd_forms.py;
    emd_kernel.cu:24-156) -- the two differ only in the order of the column
    sums -- and the launch time of each at B=8, N=2048."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for form in ("split", "rowpass", "unfused"):
        env = dict(os.environ, PCFM_EMD_FORM=form)
        subprocess.run([sys.executable, os.path.join(repo, "tests", "helpers", "emd_forms.py"),
                        str(tmp_path / f"m{form}.npz"), str(tmp_path / f"t{form}.json")],
                       check=True, timeout=120, env=env, cwd=repo)
        res[form] = json.load(open(tmp_path / f"t{form}.json"))
    a, b = np.load(tmp_path / "msplit.npz"), np.load(tmp_path / "mrowpass.npz")
    u = np.load(tmp_path / "munfused.npz")
    for k in b.files:  # level j's third pass fused with level j+1's first: same sums, same order
        np.testing.assert_array_equal(b[k], u[k], err_msg=k)
    worst = 0.0
    for k in a.files:
        x, y = a[k], b[k]
        assert x.shape == y.shape and np.isfinite(y).all(), k
        tol = 1e-9 if x.dtype == np.float64 else 2e-5
        err = float(np.abs(x - y).max()) / max(float(np.abs(x).max()), 1e-30)
        worst = max(worst, err) if x.dtype != np.float64 else worst
        assert err <= tol, (k, err)
        np.testing.assert_allclose(x.sum(axis=(1, 2)), y.sum(axis=(1, 2)), rtol=tol * 10, err_msg=k)
    report("emd_forms", {"split_ms": res["split"]["approxmatch_ms_b8_n2048"],
                         "rowpass_ms": res["rowpass"]["approxmatch_ms_b8_n2048"],
                         "rowpass_unfused_ms": res["unfused"]["approxmatch_ms_b8_n2048"],
                         "max_rel_diff_f32": worst})
