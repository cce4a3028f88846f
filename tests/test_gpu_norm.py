"""Fused BatchNorm + ReLU / LeakyReLU (csrc/norm.hip) against torch's
nn.BatchNorm + activation in training mode: output, input / gamma / beta
gradients and the running-stat update.  fp32 with a different summation
order than MIOpen: rtol 1e-4 (outputs and grads are O(1))."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from pcfm import _lib, ops
    _lib.load()
    return ops


@pytest.mark.parametrize("shape,slope,eps", [((8, 256, 20000), 0.0, 1e-5),
                                             ((2, 128, 16, 16, 16), 0.1, 1e-4),
                                             ((3, 64, 100), 0.0, 1e-5),
                                             ((1, 32, 8, 8, 8), 0.1, 1e-4)])
def test_bn_act_matches_torch(ops, shape, slope, eps):
    from modules.norm_act import bn_act, _fusable
    torch.manual_seed(0)
    c = shape[1]
    kind = torch.nn.BatchNorm1d if len(shape) == 3 else torch.nn.BatchNorm3d
    ref = kind(c, eps=eps).cuda().train()
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.5, 0.5)
        ref.running_mean.uniform_(-1, 1)
    mod = copy.deepcopy(ref)
    x = (torch.randn(*shape, device="cuda") * 2.0 + 3.0)  # offset mean: cancellation check
    assert _fusable(x, mod)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    act = torch.nn.ReLU() if slope == 0 else torch.nn.LeakyReLU(slope)
    ya = act(ref(xa))
    yb = bn_act(xb, mod, slope)
    torch.testing.assert_close(yb, ya, rtol=1e-4, atol=1e-4)
    gy = torch.randn_like(ya)
    ya.backward(gy)
    yb.backward(gy)
    # elements whose BN output lies within rounding of the activation's kink can
    # take the other branch (either side is a valid subgradient): only those may
    # differ, and each moves the gamma / beta sums by at most |dy| * O(1)
    bad = ~torch.isclose(xb.grad, xa.grad, rtol=1e-4, atol=1e-4)
    pre = torch.nn.functional.batch_norm(x, None, None, ref.weight.detach(), ref.bias.detach(),
                                         training=True, eps=eps)
    assert int(bad.sum()) <= max(2, x.numel() // 1000000)
    assert bool((pre[bad].abs() < 1e-4).all())
    kink = 1e-3 + 4.0 * float(bad.sum()) * float(gy.abs().max())
    torch.testing.assert_close(mod.weight.grad, ref.weight.grad, rtol=1e-4, atol=kink)
    torch.testing.assert_close(mod.bias.grad, ref.bias.grad, rtol=1e-4, atol=kink)
    torch.testing.assert_close(mod.running_mean, ref.running_mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(mod.running_var, ref.running_var, rtol=1e-5, atol=1e-5)
    assert int(mod.num_batches_tracked) == int(ref.num_batches_tracked) == 1


def test_bn_act_falls_back_in_eval(ops):
    from modules.norm_act import bn_act, _fusable
    bn = torch.nn.BatchNorm1d(16).cuda().eval()
    x = torch.randn(2, 16, 40, device="cuda")
    assert not _fusable(x, bn)
    torch.testing.assert_close(bn_act(x, bn, 0.0), torch.relu(bn(x)))


@pytest.mark.parametrize("b,c,n,groups", [(8, 256, 20000, 32), (2, 128, 1000, 32), (3, 64, 36, 8)])
def test_gn_film_residual_matches_torch(ops, b, c, n, groups):
    """x + GroupNorm(x) * (1 + gamma) + beta (models.py _PVBlock / _FiLM1d) fused vs torch."""
    from modules.norm_act import gn_film_residual
    torch.manual_seed(1)
    norm = torch.nn.GroupNorm(groups, c).cuda()
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.5, 0.5)
    x = torch.randn(b, c, n, device="cuda") * 1.5 + 2.0
    gamma = (torch.randn(b, c, device="cuda") * 0.3).requires_grad_(True)
    beta = (torch.randn(b, c, device="cuda") * 0.3).requires_grad_(True)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ga, gb_ = gamma.detach().clone().requires_grad_(True), gamma.detach().clone().requires_grad_(True)
    ba, bb = beta.detach().clone().requires_grad_(True), beta.detach().clone().requires_grad_(True)
    ref = xa + (norm(xa) * (1.0 + ga[:, :, None]) + ba[:, :, None])
    grads_ref = None
    gy = torch.randn_like(ref)
    ref.backward(gy)
    grads_ref = [xa.grad, norm.weight.grad.clone(), norm.bias.grad.clone(), ga.grad, ba.grad]
    norm.zero_grad()
    out = gn_film_residual(xb, norm, gb_, bb)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    out.backward(gy)
    got = [xb.grad, norm.weight.grad, norm.bias.grad, gb_.grad, bb.grad]
    for a, r in zip(got, grads_ref):
        scale = r.abs().max().item()
        torch.testing.assert_close(a, r, rtol=1e-4, atol=1e-4 * max(1.0, scale))


@pytest.mark.parametrize("kind", ["pointwise", "voxel"])
def test_conv_bn_act_fused_matches_modules(ops, kind):
    """conv_bn_act (one fused autograd node, conv bias grad from the BN backward)
    vs the conv module + torch BatchNorm + activation."""
    from modules.norm_act import conv_bn_act
    from modules.shared_mlp import PointwiseConv1d
    from modules.voxel_conv import VoxelConv3d
    torch.manual_seed(2)
    if kind == "pointwise":
        conv = PointwiseConv1d(128, 256, 1).cuda()
        bn = torch.nn.BatchNorm1d(256).cuda()
        x = torch.randn(4, 128, 3000, device="cuda")
        slope = 0.0
    else:
        conv = VoxelConv3d(128, 128, 3, padding=1).cuda()
        bn = torch.nn.BatchNorm3d(128, eps=1e-4).cuda()
        x = torch.randn(2, 128, 16, 16, 16, device="cuda")
        slope = 0.1
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    act = torch.nn.ReLU() if slope == 0 else torch.nn.LeakyReLU(slope)
    za = act(bn(conv(xa)))
    zb = conv_bn_act(conv2, bn2, xb, slope)
    assert zb.grad_fn is not None and "BnAct" in type(zb.grad_fn).__name__
    torch.testing.assert_close(zb, za, rtol=1e-3, atol=1e-3)
    gz = torch.randn_like(za)
    za.backward(gz)
    zb.backward(gz)

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
    assert rel(xb.grad, xa.grad) < 1e-3
    assert rel(conv2.weight.grad, conv.weight.grad) < 1e-3
    # the conv bias feeds a BatchNorm: its exact gradient is 0 (sum of a centred
    # quantity); both sides are fp32 round-off of that zero
    assert conv2.bias.grad.abs().max() < 1e-2 and conv.bias.grad.abs().max() < 1e-2
    assert rel(bn2.weight.grad, bn.weight.grad) < 1e-3
    assert rel(bn2.bias.grad, bn.bias.grad) < 1e-3
    torch.testing.assert_close(bn2.running_mean, bn.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn2.running_var, bn.running_var, rtol=1e-4, atol=1e-5)
    # the fused kernel increments the counter itself (no separate add_ launch)
    assert int(bn2.num_batches_tracked) == int(bn.num_batches_tracked) == 1


@pytest.mark.parametrize("b,cin,n", [(8, 256, 20000), (8, 128, 8200)])
def test_pointwise_bn_stats_from_gemm(ops, monkeypatch, b, cin, n):
    """SharedMLP layer (shared_mlp.py:21-25) on the 256-row pointwise GEMM whose
    epilogue hands the BatchNorm its statistics (64-point groups, Chan-combined
    in a fixed order) vs the separate statistics pass: same output, batch
    statistics, running statistics and gradients to fp32 round-off (the two
    differ only in summation order), vs torch's BatchNorm within 1e-4, and
    deterministic (two calls bit-identical).  n = 8200: a ragged last group.
    Gradients are compared at slope 1 (no kink): at a ReLU kink a pre-activation
    within round-off of 0 may take either side in the two forms, which flips one
    entry of dy and so a whole column of dx (seen once in 40M on the GPU)."""
    import modules.norm_act as na
    from modules.shared_mlp import PointwiseConv1d
    torch.manual_seed(3)
    conv = PointwiseConv1d(cin, 256, 1).cuda()
    bn = torch.nn.BatchNorm1d(256).cuda()
    x = torch.randn(b, cin, n, device="cuda") * 2.0 + 0.5
    assert ops.pointwise_forward_bnstats(x, conv.weight, conv.bias) is not None
    for slope in (0.0, 1.0):
        res = {}
        for flag in (True, False, True):
            monkeypatch.setattr(na, "_BN_FROM_GEMM", flag)
            c2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
            xb = x.clone().requires_grad_(True)
            z = na.conv_bn_act(c2, bn2, xb, slope)
            z.backward(torch.linspace(-1, 1, z.numel(), device="cuda").view_as(z))
            res.setdefault(flag, []).append((z.detach(), bn2.running_mean.clone(),
                                             bn2.running_var.clone(), xb.grad, c2.weight.grad,
                                             bn2.weight.grad))
        fused, sep = res[True][0], res[False][0]
        for a, c_ in zip(res[True][0], res[True][1]):
            assert torch.equal(a, c_)  # deterministic
        for a, r in zip(fused if slope == 1.0 else fused[:3], sep):
            torch.testing.assert_close(a, r, rtol=2e-5, atol=2e-5 * max(1.0, r.abs().max().item()))
        if slope == 0.0:
            bn_ref = copy.deepcopy(bn)
            act = torch.relu(bn_ref(conv(x)))
            torch.testing.assert_close(fused[0], act, rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(fused[1], bn_ref.running_mean, rtol=1e-4, atol=1e-5)
            torch.testing.assert_close(fused[2], bn_ref.running_var, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("b,c,n,groups", [(8, 256, 20000, 32), (2, 128, 1000, 32), (3, 64, 36, 8)])
def test_gn_silu_matches_torch(ops, b, c, n, groups):
    """SiLU(GroupNorm(x)) (ContextNet head_norm + head_act) fused vs torch."""
    from modules.norm_act import gn_silu
    torch.manual_seed(2)
    norm = torch.nn.GroupNorm(groups, c).cuda()
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.5, 0.5)
    x = torch.randn(b, c, n, device="cuda") * 1.5 + 2.0
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ref = torch.nn.functional.silu(norm(xa))
    gy = torch.randn_like(ref)
    ref.backward(gy)
    grads_ref = [xa.grad, norm.weight.grad.clone(), norm.bias.grad.clone()]
    norm.zero_grad()
    out = gn_silu(xb, norm)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    out.backward(gy)
    got = [xb.grad, norm.weight.grad, norm.bias.grad]
    for a, r in zip(got, grads_ref):
        scale = r.abs().max().item()
        torch.testing.assert_close(a, r, rtol=1e-4, atol=1e-4 * max(1.0, scale))


@pytest.mark.parametrize("b,c,r,slope", [(2, 128, 16, 0.1), (8, 256, 8, 0.1), (1, 64, 4, 0.0)])
def test_bn_act_backward_split_matches_unfused(ops, b, c, r, slope):
    """pcfm_bn_act_bwd_split == pcfm_bn_act_bwd followed by pcfm_conv3d_split:
    the split images bit for bit (same per-element formula), dgamma / dbeta bit
    for bit (same stats pass), the conv bias gradient to fp32 summation order."""
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(b, c, r, r, r, device="cuda", generator=g) * 2.0 + 1.0
    dz = torch.randn(b, c, r, r, r, device="cuda", generator=g)
    gamma = torch.rand(c, device="cuda", generator=g) + 0.5
    beta = torch.rand(c, device="cuda", generator=g) - 0.5
    mean = x.mean(dim=(0, 2, 3, 4))
    invstd = torch.rsqrt(x.var(dim=(0, 2, 3, 4), unbiased=False) + 1e-5)
    dx, dg, dbt, db = ops.bn_act_backward(dz, x, gamma, beta, mean, invstd, slope,
                                          want_dbias_in=True)
    ref = ops.conv3d_split(dx)
    got, dg2, dbt2, db2 = ops.bn_act_backward_split(dz, x, gamma, beta, mean, invstd, slope,
                                                    want_dbias_in=True)
    assert torch.equal(got, ref)
    assert torch.equal(dg2, dg) and torch.equal(dbt2, dbt)
    # sum_{b,s} dx is analytically ~0 (sum xhat = 0): compare at the rounding
    # scale of the summed terms, not relative to the near-zero result
    scale = float(dx.abs().sum(dim=(0, 2, 3, 4)).max())
    torch.testing.assert_close(db2, db, rtol=0, atol=1e-5 * scale)
    _, _, _, none = ops.bn_act_backward_split(dz, x, gamma, beta, mean, invstd, slope)
    assert none is None


@pytest.mark.parametrize("b,c,r", [(2, 128, 16), (2, 256, 8), (1, 128, 32)])
def test_conv_bn_act_pair_matches_two_nodes(ops, b, c, r):
    """PVConv's fused pair node (inner activation only as Conv2's split input)
    equals two single-layer nodes bit for bit: the split of act(bn(y1)) is the
    same bf16 pair either way, so every output, gradient and running stat must
    agree exactly."""
    from modules.norm_act import _Conv3dBnActPair, conv_bn_act, conv_bn_act_pair
    from modules.voxel_conv import VoxelConv3d
    torch.manual_seed(5)
    mods = [VoxelConv3d(c, c, 3, padding=1).cuda(), torch.nn.BatchNorm3d(c, eps=1e-4).cuda(),
            VoxelConv3d(c, c, 3, padding=1).cuda(), torch.nn.BatchNorm3d(c, eps=1e-4).cuda()]
    ref = copy.deepcopy(mods)
    x = torch.randn(b, c, r, r, r, device="cuda")
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    za = conv_bn_act(ref[2], ref[3], conv_bn_act(ref[0], ref[1], xa, 0.1), 0.1)
    zb = conv_bn_act_pair(mods[0], mods[1], 0.1, mods[2], mods[3], 0.1, xb)
    assert isinstance(zb.grad_fn, _Conv3dBnActPair._backward_cls)
    assert torch.equal(za, zb)
    gz = torch.randn_like(za)
    za.backward(gz)
    zb.backward(gz)
    assert torch.equal(xa.grad, xb.grad)
    for m_ref, m in zip(ref, mods):
        for (name, p_ref), p in zip(m_ref.named_parameters(), m.parameters()):
            assert torch.equal(p_ref.grad, p.grad), name
        for (name, b_ref), bb in zip(m_ref.named_buffers(), m.buffers()):
            assert torch.equal(b_ref, bb), name
    assert int(mods[1].num_batches_tracked) == int(mods[3].num_batches_tracked) == 1


def _unsplit(buf, b, c, s):
    """Decode a conv split operand (pcfm_common.hpp split_off: channels-last rows,
    [hi 32 | lo 32] per 32-channel group) back to fp32 (B, C, S) = hi + lo."""
    t = buf.view(torch.bfloat16).view(b * s, c // 32, 2, 32).float()
    return (t[:, :, 0] + t[:, :, 1]).reshape(b, s, c).permute(0, 2, 1).contiguous()


@pytest.mark.parametrize("b,c,r,slope", [(2, 128, 16, 0.1), (8, 256, 8, 0.1), (2, 128, 32, 0.1),
                                         (1, 64, 4, 0.0)])
def test_bn_act_rowmean_and_bn_devox_match_unfused(ops, b, c, r, slope):
    """PVConv's BN2 fused with SE and the devoxelization, forward: the statistics,
    running stats and counter bit-equal to pcfm_bn_act_fwd (same passes); rowmean
    = the per-(b, c) mean of act(bn(x)) to fp32 summation order; the gather that
    applies bn + act while staging bit-equal to the plain gather of act(bn(x))."""
    g = torch.Generator(device="cuda").manual_seed(r)
    s = r ** 3
    x = torch.randn(b, c, r, r, r, device="cuda", generator=g) * 2.0 + 1.0
    gamma = torch.rand(c, device="cuda", generator=g) + 0.5
    beta = torch.rand(c, device="cuda", generator=g) - 0.5
    rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    rm2, rv2 = rm.clone(), rv.clone()
    nbt = torch.zeros((), dtype=torch.int64, device="cuda")
    nbt2 = nbt.clone()
    z, m, iv = ops.bn_act_forward(x, gamma, beta, 1e-4, slope, 0.1, rm, rv, nbt)
    rowmean, m2, iv2 = ops.bn_act_forward_rowmean(x, gamma, beta, 1e-4, slope, 0.1, rm2, rv2, nbt2)
    assert torch.equal(m, m2) and torch.equal(iv, iv2)
    assert torch.equal(rm, rm2) and torch.equal(rv, rv2) and int(nbt2) == 1
    ref = z.double().reshape(b, c, s).mean(-1)
    torch.testing.assert_close(rowmean.double(), ref, rtol=0, atol=2e-6 * float(z.abs().max()))
    n = 3000
    coords = torch.rand(b, 3, n, device="cuda", generator=g) * (r - 1)
    sc = torch.rand(b, c, device="cuda", generator=g)
    pf = torch.randn(b, c, n, device="cuda", generator=g)
    o_ref, i_ref, w_ref = ops.trilinear_devoxelize_scale_add(r, True, coords, z, sc, pf)
    o, i, w = ops.trilinear_devoxelize_bn_scale_add(r, True, coords, x, m2, iv2, gamma, beta,
                                                    slope, sc, pf)
    assert torch.equal(o, o_ref) and torch.equal(i, i_ref) and torch.equal(w, w_ref)


@pytest.mark.parametrize("b,c,r,slope", [(2, 128, 16, 0.1), (8, 256, 8, 0.1), (2, 128, 32, 0.1),
                                         (1, 64, 4, 0.0)])
def test_bn_se_backward_matches_composition(ops, b, c, r, slope):
    """PVConv's BN2 + SE backward from g = devox_bwd(dout): pcfm_bn_se_bwd_stats'
    ds = sum z g against fp64, and pcfm_bn_se_bwd_apply_split against the round-4
    composition (dz = rows_affine(g, s, dmv) -> pcfm_bn_act_bwd): dx (split operand,
    decoded), dgamma, dbeta within fp32 summation-order bounds."""
    gen = torch.Generator(device="cuda").manual_seed(7 + r)
    s = r ** 3
    x = torch.randn(b, c, r, r, r, device="cuda", generator=gen) * 2.0 + 1.0
    gr = torch.randn(b, c, r, r, r, device="cuda", generator=gen)
    gamma = torch.rand(c, device="cuda", generator=gen) + 0.5
    beta = torch.rand(c, device="cuda", generator=gen) - 0.5
    se_s = torch.rand(b, c, device="cuda", generator=gen)
    dmv = torch.randn(b, c, device="cuda", generator=gen) * 1e-3
    mean = x.mean(dim=(0, 2, 3, 4))
    invstd = torch.rsqrt(x.var(dim=(0, 2, 3, 4), unbiased=False) + 1e-4)
    # reference composition
    xh = (x.double() - mean.double()[None, :, None, None, None]) * invstd.double()[None, :, None,
                                                                                      None, None]
    t = xh * gamma.double()[None, :, None, None, None] + beta.double()[None, :, None, None, None]
    z = torch.where(t > 0, t, t * slope)
    ds_ref = (z * gr.double()).reshape(b, c, s).sum(-1)
    dz = gr.clone().reshape(b * c, s)
    ops.rows_affine_(dz, se_s.reshape(-1), dmv.reshape(-1))
    dx, dg, dbt, db = ops.bn_act_backward(dz.view_as(x), x, gamma, beta, mean, invstd, slope,
                                          want_dbias_in=True)
    # fused
    rowstats = ops.bn_se_backward_stats(gr, x, mean, invstd, gamma, beta, slope)
    assert rowstats.shape == (5, b, c)
    scale = float((z.abs() * gr.double().abs()).reshape(b, c, s).sum(-1).max())
    torch.testing.assert_close(rowstats[0].double(), ds_ref, rtol=0, atol=1e-5 * scale)
    dxs, dg2, dbt2, db2 = ops.bn_se_backward_apply_split(gr, x, mean, invstd, gamma, beta, se_s,
                                                         dmv, rowstats, slope, want_dbias_in=True)
    got = _unsplit(dxs, b, c, s)
    ref = dx.reshape(b, c, s)
    torch.testing.assert_close(got, ref, rtol=0, atol=2e-5 * float(ref.abs().max()))
    for a, e in ((dg2, dg), (dbt2, dbt)):
        torch.testing.assert_close(a, e, rtol=0, atol=2e-5 * float(e.abs().max()) + 1e-6)
    sc = float(dx.abs().sum(dim=(0, 2, 3, 4)).max())
    torch.testing.assert_close(db2, db, rtol=0, atol=1e-5 * sc)
    # deterministic
    rs2 = ops.bn_se_backward_stats(gr, x, mean, invstd, gamma, beta, slope)
    assert torch.equal(rowstats, rs2)


def _relerr(a, ref):
    a, ref = a.detach().double(), ref.detach().double()
    return ((a - ref).abs().max() / ref.pow(2).mean().sqrt().clamp_min(1e-30)).item()


@pytest.mark.parametrize("b,c,n,groups", [(8, 256, 20000, 32), (2, 128, 3000, 32), (3, 64, 36, 8)])
def test_post_gn_film_fused_matches_two_nodes(ops, monkeypatch, b, c, n, groups):
    """The PV block's tail as one node (_PostGNFiLMRes: the post SharedMLP's
    ReLU(BN(.)) read by the GroupNorm kernels from the conv output, never
    written) against the two-node form (SharedMLP node, then the GroupNorm-FiLM
    residual node).  The forward computes the same z bit for bit, so the output
    and running statistics are equal.  The BatchNorm backward sums come from the
    GroupNorm backward's blocks instead of the statistics pass (another summation
    order): every gradient within 1e-5 of the two-node form's in norm
    (||d|| / ||ref||) and 1e-4 in max |d| / rms; the conv bias, 0 up to rounding
    behind a training-mode BatchNorm, on the weight gradient's scale.  (An fp64
    evaluation is no reference here: at 4e7 elements some ReLU inputs round to the
    other side of 0 in fp32, moving single gradient entries by O(1) in both
    forms alike.)"""
    import modules.norm_act as na
    from modules.shared_mlp import SharedMLP
    torch.manual_seed(7)
    post = SharedMLP(c, [c]).cuda()
    norm = torch.nn.GroupNorm(groups, c, eps=1e-6).cuda()
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.5, 0.5)
        post.layers[1].weight.uniform_(0.5, 1.5)
        post.layers[1].bias.uniform_(-0.5, 0.5)
    mods = [post, norm]
    ref = copy.deepcopy(mods)
    x = torch.randn(b, c, n, device="cuda")
    gam = (0.2 * torch.randn(b, c, device="cuda")).requires_grad_(True)
    bet = (0.2 * torch.randn(b, c, device="cuda")).requires_grad_(True)
    gam2, bet2 = gam.detach().clone().requires_grad_(True), bet.detach().clone().requires_grad_(True)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    monkeypatch.setattr(na, "_POST_GN_FUSED", False)
    oa = na.post_gn_film_residual(ref[0], ref[1], xa, gam2, bet2)
    monkeypatch.setattr(na, "_POST_GN_FUSED", True)
    ob = na.post_gn_film_residual(mods[0], mods[1], xb, gam, bet)
    assert isinstance(ob.grad_fn, na._PostGNFiLMRes._backward_cls)
    assert not isinstance(oa.grad_fn, na._PostGNFiLMRes._backward_cls)
    assert torch.equal(oa, ob)
    for m_ref, m in zip(ref, mods):
        for (name, b_ref), bb in zip(m_ref.named_buffers(), m.buffers()):
            assert torch.equal(b_ref, bb), name
    go = torch.randn_like(oa)
    oa.backward(go)
    ob.backward(go)
    conv, bn = post.layers[0], post.layers[1]
    names = ["x", "conv.weight", "conv.bias", "bn.weight", "bn.bias", "gn.weight", "gn.bias",
             "gamma", "beta"]
    got_u = [xa.grad, ref[0].layers[0].weight.grad, ref[0].layers[0].bias.grad,
             ref[0].layers[1].weight.grad, ref[0].layers[1].bias.grad, ref[1].weight.grad,
             ref[1].bias.grad, gam2.grad, bet2.grad]
    got_f = [xb.grad, conv.weight.grad, conv.bias.grad, bn.weight.grad, bn.bias.grad,
             norm.weight.grad, norm.bias.grad, gam.grad, bet.grad]
    report = {}
    for nm, gu, gf in zip(names, got_u, got_f):
        d = (gf.double() - gu.double())
        scale = got_u[1].double() if nm == "conv.bias" else gu.double()
        rel_norm = (d.norm() / scale.norm().clamp_min(1e-30)).item()
        rel_max = (d.abs().max() / scale.pow(2).mean().sqrt().clamp_min(1e-30)).item()
        report[nm] = (rel_norm, rel_max)
        assert rel_norm < 1e-5 and rel_max < 1e-4, (nm, report)
