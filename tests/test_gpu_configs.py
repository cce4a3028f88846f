"""GPU: the BASELINE.json workloads beyond the headline C2 train step.

* C5 -- configs[4]: B=4, N=100000 xyz+rgb.  The voxel ops at full size through
  size-independent properties (mass conservation, linearity, adjointness,
  determinism); Chamfer and ball query on sampled queries, bit-exact against the
  oracle scanning the FULL 100000-point candidate cloud; one train step.
* C4 -- configs[3]: generation at B=32, N=20000 with the reference's Heun
  (50 steps = 100 NFE) and adaptive dopri5; the eval-mode devoxelization (no
  inds / wgts, trilinear_devox.cpp:45-53) equals the training-mode output.
"""
import math
import time

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
B5, N5 = 4, 100000


def _surface(g, b, n):
    """Points near the unit sphere (dense voxels: the hard case for the scatter)."""
    p = torch.randn(b, n, 3, device=DEV, generator=g)
    return p / p.norm(dim=-1, keepdim=True) + 0.01 * torch.randn(b, n, 3, device=DEV, generator=g)


@pytest.mark.parametrize("c,r", [(128, 32), (256, 16), (256, 8)])
def test_c5_voxelize_properties(c, r):
    from modules.functional import avg_voxelize
    from modules.voxelization import Voxelization
    from pcfm import ops
    g = torch.Generator(device=DEV).manual_seed(r)
    xyz = _surface(g, B5, N5).permute(0, 2, 1).contiguous()
    feat = torch.randn(B5, c, N5, device=DEV, generator=g)
    grid, norm = Voxelization(r, normalize=True, eps=1e-6)(feat, xyz)
    assert grid.shape == (B5, c, r, r, r)
    vox = torch.round(norm).int().contiguous()
    out, ind, cnt = ops.avg_voxelize_forward(feat, vox, r)
    assert int(cnt.sum()) == B5 * N5 and int(cnt.min()) >= 0
    assert torch.equal(ind.long(), (vox[:, 0] * r * r + vox[:, 1] * r + vox[:, 2]).long())
    # sum_v out[c, v] * cnt[v] == sum_i feat[c, i]
    lhs = (out.double() * cnt[:, None, :].double()).sum(-1)
    rhs = feat.double().sum(-1)
    assert torch.allclose(lhs, rhs, rtol=1e-5, atol=1e-2)
    # deterministic: a second call returns the same bits
    out2, ind2, cnt2 = ops.avg_voxelize_forward(feat, vox, r)
    assert torch.equal(ind, ind2) and torch.equal(cnt, cnt2)
    assert torch.equal(out2, out)
    # backward = gather of grad / cnt: adjoint of the forward
    gy = torch.randn(B5, c, r ** 3, device=DEV, generator=g)
    gx = avg_voxelize(feat.requires_grad_(True), vox, r)
    gx.backward(gy.view_as(gx))
    a = (out.double() * gy.double()).sum()
    bb = (feat.double() * feat.grad.double()).sum()
    assert abs(a - bb) <= 1e-5 * abs(a)


@pytest.mark.parametrize("c,r", [(128, 32), (256, 8)])
def test_c5_devoxelize_properties(c, r):
    from pcfm import ops
    g = torch.Generator(device=DEV).manual_seed(100 + r)
    pts = torch.rand(B5, 3, N5, device=DEV, generator=g) * (r - 1)
    grid = torch.randn(B5, c, r ** 3, device=DEV, generator=g)
    out, inds, wgts = ops.trilinear_devoxelize_forward(r, True, pts, grid)
    out2, _, _ = ops.trilinear_devoxelize_forward(r, True, pts, 2.0 * grid)
    assert torch.equal(out2, 2.0 * out)
    ev, i1, w1 = ops.trilinear_devoxelize_forward(r, False, pts, grid)
    assert torch.equal(ev, out) and i1.numel() == 1 and w1.numel() == 1
    gy = torch.randn(B5, c, N5, device=DEV, generator=g)
    gx = ops.trilinear_devoxelize_backward(gy, inds, wgts, r)
    lhs = (out.double() * gy.double()).sum()
    rhs = (grid.double() * gx.double()).sum()
    assert abs(lhs - rhs) <= 1e-4 * abs(lhs)
    # oracle on a slice of points (same grid): bit-exact gather
    q = slice(0, 2000)
    e_o, e_i, _ = O.trilinear_devoxelize_fwd(pts[:1, :, q].cpu().numpy(), grid[:1].cpu().numpy(),
                                             r)
    np.testing.assert_array_equal(out[:1, :, q].cpu().numpy(), e_o)
    np.testing.assert_array_equal(inds[:1, :, q].cpu().numpy(), e_i)


def test_c5_chamfer_sampled_bit_exact(report):
    from pcfm import ops
    g = np.random.default_rng(5)
    a = g.standard_normal((B5, N5, 3)).astype(np.float32)
    c = g.standard_normal((B5, N5, 3)).astype(np.float32)
    c[:, :100] = a[:, :100]  # exact hits
    ca, cc = torch.from_numpy(a).to(DEV), torch.from_numpy(c).to(DEV)
    d1 = torch.empty(B5, N5, device=DEV)
    d2 = torch.empty(B5, N5, device=DEV)
    i1 = torch.empty(B5, N5, dtype=torch.int32, device=DEV)
    i2 = torch.empty(B5, N5, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    assert ops.chamfer_3D.forward(ca, cc, d1, d2, i1, i2) == 1
    torch.cuda.synchronize()
    report("c5_chamfer_fwd_ms", 1e3 * (time.perf_counter() - t0))
    q = np.concatenate([np.arange(8), g.choice(N5, 56, replace=False)])
    for bb in range(B5):
        e = O.chamfer_fwd(a[bb:bb + 1, q], c[bb:bb + 1])
        np.testing.assert_array_equal(d1[bb, q].cpu().numpy(), e[0][0])
        np.testing.assert_array_equal(i1[bb, q].cpu().numpy(), e[2][0])
        e = O.chamfer_fwd(c[bb:bb + 1, q], a[bb:bb + 1])
        np.testing.assert_array_equal(d2[bb, q].cpu().numpy(), e[0][0])
        np.testing.assert_array_equal(i2[bb, q].cpu().numpy(), e[2][0])


def test_c5_ball_query_sampled_bit_exact(report):
    from pcfm import ops
    g = np.random.default_rng(6)
    m, u = 4096, 32
    pts = g.random((B5, 3, N5)).astype(np.float32)
    ctr = g.random((B5, 3, m)).astype(np.float32)
    ctr[:, :, :64] = pts[:, :, :64]
    cp, cc = torch.from_numpy(pts).to(DEV), torch.from_numpy(ctr).to(DEV)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx = ops.ball_query(cc, cp, 0.05, u)
    torch.cuda.synchronize()
    report("c5_ball_query_ms_m4096_u32", 1e3 * (time.perf_counter() - t0))
    sel = np.concatenate([np.arange(64, 72), g.choice(m, 56, replace=False)])
    for bb in range(B5):
        e = O.ball_query(ctr[bb:bb + 1, :, sel], pts[bb:bb + 1], 0.05, u)
        np.testing.assert_array_equal(idx[bb, sel].cpu().numpy(), e[0])


def test_c5_train_step(report):
    from pcfm.train import TrainConfig, Trainer, synthetic_batch
    cfg = TrainConfig(batch_size=B5, num_points=N5, steps_per_epoch=10, epochs=2)
    tr = Trainer(cfg, DEV)
    tr.train_mode()
    batch = synthetic_batch(cfg, DEV, surface=True)
    out = tr.step(batch, epoch=201)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = tr.step(batch, epoch=201)
    torch.cuda.synchronize()
    report("c5_train_step_ms", 1e3 * (time.perf_counter() - t0))
    assert math.isfinite(out["loss_point"].item()) and math.isfinite(out["loss_latent"].item())


@pytest.fixture(scope="module")
def c4_models():
    from pcfm.train import TrainConfig, build_models
    torch.manual_seed(0)
    cfg = TrainConfig(batch_size=32, num_points=20000)
    _, pf, lf = build_models(cfg, DEV)
    return cfg, pf.eval(), lf.eval()


@pytest.mark.parametrize("method", ["heun", "dopri5"])
def test_c4_generate(c4_models, report, method):
    from pcfm.sample import generate
    cfg, pf, lf = c4_models
    torch.manual_seed(1)
    cond = torch.rand(32, cfg.cond_dim, device=DEV)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x, nfe = generate(pf, lf, 32, 20000, point_dim=6, latent_dim=cfg.latent_dim, cond=cond,
                      cond_dim=cfg.cond_dim, steps=50, method=method, rtol=1e-3, atol=1e-3)
    torch.cuda.synchronize()
    report(f"c4_generate_{method}", {"s": time.perf_counter() - t0, "nfe": nfe})
    assert x.shape == (32, 20000, 6) and torch.isfinite(x).all()
    if method == "heun":
        assert nfe == 100
    else:
        assert 7 <= nfe < 1000


def test_c4_eval_devox_equals_training(c4_models):
    """Eval mode skips inds / wgts (trilinear_devox.cpp:45-53) and returns (1,)
    dummies, with the same output values as training mode."""
    from pcfm import ops
    g = torch.Generator(device=DEV).manual_seed(9)
    for c, r in ((128, 32), (256, 16), (256, 8)):
        pts = torch.rand(32, 3, 20000, device=DEV, generator=g) * (r - 1)
        grid = torch.randn(32, c, r ** 3, device=DEV, generator=g)
        tr_out, _, _ = ops.trilinear_devoxelize_forward(r, True, pts, grid)
        ev, i, w = ops.trilinear_devoxelize_forward(r, False, pts, grid)
        assert torch.equal(ev, tr_out) and i.shape == (1,) and w.shape == (1,)
