"""PVConv with SE3d + point-branch sum folded into the devoxelization
(modules/pvconv.py _SEDevoxAdd) against the unfused module chain (SE3d module,
trilinear_devoxelize, torch add), forward and backward, fp32 tolerance."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, ref):
    return ((a.double() - ref.double()).abs().max() / ref.double().pow(2).mean().sqrt()).item()


@pytest.fixture(scope="module")
def ops():
    from pcfm import _lib, ops
    _lib.load()
    return ops


def test_rows_dot_and_affine(ops):
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(37, 1000, device="cuda", generator=g)
    b = torch.randn(37, 1000, device="cuda", generator=g)
    ref = (a.double() * b.double()).sum(1)
    assert (ops.rows_dot(a, b, 1.0).double() - ref).abs().max() < 1e-4
    assert (ops.rows_dot(a, None, 0.5).double() - 0.5 * a.double().sum(1)).abs().max() < 1e-4
    odd = torch.randn(5, 7, device="cuda", generator=g)
    assert (ops.rows_dot(odd, odd, 1.0).double() - odd.double().pow(2).sum(1)).abs().max() < 1e-5
    s = torch.randn(37, device="cuda", generator=g)
    t = torch.randn(37, device="cuda", generator=g)
    x = a.clone()
    ops.rows_affine_(x, s, t)
    assert torch.allclose(x, s[:, None] * a + t[:, None], atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("b,c,h", [(8, 256, 32), (8, 128, 16), (3, 64, 8), (1, 7, 3)])
def test_se_mlp_kernels_match_torch(ops, b, c, h):
    """pcfm_se_mlp_fwd / _bwd (SE3d's MLP, se.py:9-19, one launch each way)
    against torch autograd over sigmoid(W2 relu(W1 m)) in fp32: outputs and all
    three gradients (dm with the pooling's 1/V folded in) to fp32 round-off."""
    g = torch.Generator(device="cuda").manual_seed(c)
    m = torch.randn(b, c, device="cuda", generator=g)
    w1 = torch.randn(h, c, device="cuda", generator=g) * c ** -0.5
    w2 = torch.randn(c, h, device="cuda", generator=g) * h ** -0.5
    ds = torch.randn(b, c, device="cuda", generator=g)
    assert ops.se_mlp_ok(m, w1)
    s, hid = ops.se_mlp_forward(m, w1, w2)
    dm, dw1, dw2 = ops.se_mlp_backward(m, hid, s, ds, w1, w2, 0.25)
    mr, w1r, w2r = (t.clone().requires_grad_(True) for t in (m, w1, w2))
    sr = torch.sigmoid(torch.relu(mr @ w1r.t()) @ w2r.t())
    sr.backward(ds)
    torch.testing.assert_close(s, sr.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(hid, torch.relu(m @ w1.t()), rtol=1e-5, atol=1e-6)
    for a, r_ in ((dm, 0.25 * mr.grad), (dw1, w1r.grad), (dw2, w2r.grad)):
        torch.testing.assert_close(a, r_, rtol=1e-5, atol=1e-6 * max(1.0, r_.abs().max().item()))
    s2, _ = ops.se_mlp_forward(m, w1, w2)
    assert torch.equal(s, s2)  # deterministic


@pytest.mark.parametrize("cin,cout,r,n", [(64, 128, 8, 3000), (128, 128, 16, 5000)])
def test_pvconv_se_devox_fused_matches_modules(ops, monkeypatch, cin, cout, r, n):
    import modules.pvconv as pv
    torch.manual_seed(r)
    mod = pv.PVConv(cin, cout, 3, r, with_se=True, normalize=True).cuda().train()
    feats = torch.randn(2, cin, n, device="cuda")
    coords = torch.rand(2, 3, n, device="cuda") * 2 - 1
    state = {k: v.clone() for k, v in mod.state_dict().items()}

    def run():
        mod.load_state_dict(state)
        f = feats.clone().requires_grad_(True)
        out, _ = mod((f, coords))
        gy = torch.randn(out.shape, device="cuda", generator=torch.Generator(
            device="cuda").manual_seed(1))
        out.backward(gy)
        grads = [("input", f.grad)] + [(k, p.grad.clone()) for k, p in mod.named_parameters()]
        mod.zero_grad(set_to_none=True)
        return out.detach(), grads

    fused_out, fused_grads = run()
    monkeypatch.setattr(pv, "_se_devox_ok", lambda *a: False)
    ref_out, ref_grads = run()
    assert _rel(fused_out, ref_out) < 1e-5
    # biases of the convolutions feeding a training-mode BatchNorm have an
    # analytically zero gradient: both sides are rounding noise, compared absolutely
    zero_grad = {"voxel_layers.0.bias", "voxel_layers.3.bias", "point_features.layers.0.bias"}
    for (name, a), (_, b) in zip(fused_grads, ref_grads):
        if name in zero_grad:
            assert (a - b).abs().max().item() < 1e-3, name
        else:
            assert _rel(a, b) < 1e-4, name


def test_pvconv_voxelize_tee_matches_separate_grads(ops, monkeypatch):
    """The tee'd voxelization (point-branch gradient added inside the voxelization's
    backward gather) against the module path where autograd adds the two."""
    import modules.pvconv as pv
    from modules.voxelization import Voxelization
    torch.manual_seed(2)
    mod = pv.PVConv(128, 128, 3, 16, with_se=True, normalize=True).cuda().train()
    feats = torch.randn(2, 128, 4000, device="cuda")
    coords = torch.rand(2, 3, 4000, device="cuda")
    state = {k: v.clone() for k, v in mod.state_dict().items()}
    gy = torch.randn(2, 128, 4000, device="cuda")

    def run():
        mod.load_state_dict(state)
        f = feats.clone().requires_grad_(True)
        out, _ = mod((f, coords))
        out.backward(gy)
        return out.detach(), f.grad

    o1, g1 = run()

    def plain(self, features, coords):
        grid, nc = self.forward(features, coords)
        return grid, nc, features

    monkeypatch.setattr(Voxelization, "forward_tee", plain)
    o0, g0 = run()
    # same sums, the point-branch add done in another kernel: fp32 rounding
    assert _rel(o1, o0) < 1e-4
    assert _rel(g1, g0) < 1e-4


@pytest.mark.parametrize("c,r,n", [(64, 8, 3000), (128, 32, 20000), (256, 16, 777)])
def test_planned_scatters_match_one_shot(ops, c, r, n):
    """Plan + apply (include/pcfm.h segment plans) == the one-shot scatters, bit
    for bit (same sort, same units, same fixed-order sums)."""
    g = torch.Generator(device="cuda").manual_seed(c + r)
    b = 3
    pts = torch.randn(b, 3, n, device="cuda", generator=g) * 0.3 + 0.5
    nc = torch.clamp(pts * r, 0, r - 1)
    vc = torch.round(nc).to(torch.int32)
    feat = torch.randn(b, c, n, device="cuda", generator=g)
    out0, ind0, cnt0 = ops.avg_voxelize_forward(feat, vc, r)
    plan = ops.avg_voxelize_plan(vc, r)
    assert torch.equal(plan.ind, ind0) and torch.equal(plan.cnt, cnt0)
    assert torch.equal(ops.avg_voxelize_forward_planned(feat, plan), out0)
    feat2 = torch.randn(b, c // 2, n, device="cuda", generator=g)  # the plan is C-free
    assert torch.equal(ops.avg_voxelize_forward_planned(feat2, plan),
                       ops.avg_voxelize_forward(feat2, vc, r)[0])
    grid = torch.randn(b, c, r ** 3, device="cuda", generator=g)
    _, inds, wgts = ops.trilinear_devoxelize_forward(r, True, nc, grid)
    gy = torch.randn(b, c, n, device="cuda", generator=g)
    ref = ops.trilinear_devoxelize_backward(gy, inds, wgts, r)
    dplan = ops.trilinear_devoxelize_backward_plan(inds, wgts, r)
    assert torch.equal(ops.trilinear_devoxelize_backward_planned(gy, dplan), ref)
    assert torch.equal(ops.trilinear_devoxelize_backward_planned(gy * 2.0, dplan), ref * 2.0)


def test_stage_blocks_share_plans(ops, monkeypatch):
    """A hybrid stage (1x1 lift + two PV blocks on the same points): the second
    block reuses the first one's grid coordinates, voxelization plan, corner
    indices and devoxelization-backward plan -- one plan build per kind per
    stage -- with outputs and gradients identical to building them per block."""
    from pcfm import plans
    from pcfm.models import _PVStage
    torch.manual_seed(4)
    st = _PVStage(64, 128, 2, 16, emb_dim=32, with_se=True).cuda().train()
    state = {k: v.clone() for k, v in st.state_dict().items()}
    feat = torch.randn(2, 64, 6000, device="cuda")
    coords = torch.randn(2, 3, 6000, device="cuda")
    emb = torch.randn(2, 32, device="cuda")
    gy = torch.randn(2, 128, 6000, device="cuda")
    builds = {"vox": 0, "devox": 0}
    vplan, dplan = ops.avg_voxelize_plan, ops.trilinear_devoxelize_backward_plan

    def count(kind, fn):
        def wrapped(*a, **k):
            builds[kind] += 1
            return fn(*a, **k)
        return wrapped
    monkeypatch.setattr(ops, "avg_voxelize_plan", count("vox", vplan))
    monkeypatch.setattr(ops, "trilinear_devoxelize_backward_plan", count("devox", dplan))

    def run(enabled):
        monkeypatch.setattr(plans, "ENABLED", enabled)
        st.load_state_dict(state)
        f = feat.clone().requires_grad_(True)
        out, _ = st(f, coords, emb)
        out.backward(gy)
        grads = [f.grad] + [p.grad.clone() for p in st.parameters()]
        st.zero_grad(set_to_none=True)
        return out.detach(), grads

    o1, g1 = run(True)
    assert builds == {"vox": 1, "devox": 1}
    o0, g0 = run(False)
    assert torch.equal(o1, o0)
    for a, b in zip(g1, g0):
        assert torch.equal(a, b)


def _voxelized(ops, b, c, r, n, seed, surface=False):
    """A voxelized grid of random features over a randn (or spherical-shell)
    cloud, its counts, and the occupancy masks."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    pts = torch.randn(b, 3, n, device="cuda", generator=g)
    if surface:
        pts = pts / pts.norm(dim=1, keepdim=True)
    c0 = pts - pts.mean(2, keepdim=True)
    unit = c0 / (2 * c0.norm(dim=1, keepdim=True).max(2, keepdim=True).values + 1e-6) + 0.5
    vox = torch.round(torch.clamp(unit * r, 0, r - 1)).int().contiguous()
    feats = torch.randn(b, c, n, device="cuda", generator=g)
    grid, _, cnt = ops.avg_voxelize_forward(feats, vox, r)
    occ = ops.conv3d_occupancy(cnt, r)
    return grid.view(b, c, r, r, r), cnt, occ


@pytest.mark.parametrize("cin,cout,r,surface", [(128, 128, 32, False), (128, 256, 16, False),
                                                (128, 128, 32, True)])
def test_conv_occupancy_skipping_is_exact(ops, cin, cout, r, surface, report):
    """PVConv's first conv over a voxelized grid with the occupancy masks:
    forward and weight gradient bit-identical to the unmasked kernels; the
    backward-data equal at every occupied voxel (0 in tiles without one where
    the masked kernel runs: unsplit launches of the 128 x 256-tile kernel)."""
    b = 4
    grid, cnt, occ = _voxelized(ops, b, cin, r, 6000, r + cin, surface)
    assert occ is not None
    xs = ops.conv3d_split(grid.contiguous())
    g = torch.Generator(device="cuda").manual_seed(5)
    w = torch.randn(cout, cin, 3, 3, 3, device="cuda", generator=g) * 0.05
    bias = torch.randn(cout, device="cuda", generator=g)
    img = ops.conv3d_prep_weight(w, False)
    y0 = ops.conv3d_igemm_split(xs, img, bias, b, cin, cout, r, "conv3d_fwd")
    y1 = ops.conv3d_igemm_split(xs, img, bias, b, cin, cout, r, "conv3d_fwd", occ=occ,
                                occ_mode=1)
    assert torch.equal(y0, y1)
    dy = torch.randn(b, cout, r, r, r, device="cuda", generator=g)
    gys = ops.conv3d_split(dy)
    imgt = ops.conv3d_prep_weight(w, True)
    dx0 = ops.conv3d_igemm_split(gys, imgt, None, b, cout, cin, r, "conv3d_bwd_data")
    dx1 = ops.conv3d_igemm_split(gys, imgt, None, b, cout, cin, r, "conv3d_bwd_data", occ=occ,
                                 occ_mode=2)
    occupied = (cnt.view(b, 1, -1) > 0).expand(b, cin, r ** 3)
    assert torch.equal(dx0.view(b, cin, -1)[occupied], dx1.view(b, cin, -1)[occupied])
    tiles = (cnt.view(b, -1, 256) > 0).any(-1)                     # (b, tiles)
    dw0 = ops.conv3d_wgrad_split(xs, gys, b, cin, cout, r)
    dw1 = ops.conv3d_wgrad_split(xs, gys, b, cin, cout, r, occ=occ)
    assert torch.equal(dw0, dw1)
    # fp64 reference of the weight gradient (the new strided step order)
    ref = torch.nn.grad.conv3d_weight(grid.double(), w.shape, dy.double(), padding=1)
    err = ((dw1.double() - ref).abs().max() / ref.pow(2).mean().sqrt()).item()
    assert err < 1e-4
    m = occ[: b * (r ** 3 // 256)]
    active = sum(bin(int(v) & 0x7FFFFFF).count("1") for v in m.tolist()) / (27.0 * m.numel())
    report(f"conv_occupancy_c{cin}_r{r}{'_surface' if surface else ''}",
           {"fwd_active_tap_fraction": active,
            "bwd_active_tile_fraction": float(tiles.float().mean()), "wgrad_rel_err": err})


def test_pvconv_occupancy_end_to_end(ops, monkeypatch):
    """A PVConv layer's output and every gradient are bit-identical with the
    occupancy skipping on and off (pcfm.plans.OCCUPANCY)."""
    import modules.pvconv as pv
    from pcfm import plans
    torch.manual_seed(0)
    mod = pv.PVConv(128, 128, 3, 32, with_se=True, normalize=True).cuda().train()
    feats = torch.randn(2, 128, 8000, device="cuda")
    coords = torch.randn(2, 3, 8000, device="cuda")
    state = {k: v.clone() for k, v in mod.state_dict().items()}

    def run():
        mod.load_state_dict(state)
        f = feats.clone().requires_grad_(True)
        out, _ = mod((f, coords.clone()))
        out.backward(torch.randn(out.shape, device="cuda",
                                 generator=torch.Generator(device="cuda").manual_seed(1)))
        grads = [f.grad] + [p.grad.clone() for p in mod.parameters()]
        mod.zero_grad(set_to_none=True)
        return out.detach(), grads

    monkeypatch.setattr(plans, "OCCUPANCY", True)
    o1, g1 = run()
    monkeypatch.setattr(plans, "OCCUPANCY", False)
    o0, g0 = run()
    assert torch.equal(o0, o1)
    for a, b_ in zip(g0, g1):
        assert torch.equal(a, b_)


@pytest.mark.parametrize("b,r,n,surface", [(4, 32, 6000, False), (3, 16, 5000, True),
                                           (2, 8, 3000, False)])
def test_conv_voxel_lists(ops, b, r, n, surface):
    """pcfm_conv3d_vlist against torch: list 0 = the 32-voxel chunks holding an
    occupied voxel, list 1 = the chunks holding a voxel with an occupied voxel in
    its 3x3x3 neighbourhood, both as ascending global chunk indices
    (b r^3 + v) / 32; list 2 = the occupied voxels, ascending b r^3 + v; the
    device-side counts first."""
    _, cnt, _ = _voxelized(ops, b, 8, r, n, 3 * r, surface)
    lists = ops.conv3d_vlists(cnt, r)
    assert lists is not None
    v = r ** 3
    occ = (cnt.view(b, 1, r, r, r) > 0).float()
    act = torch.nn.functional.max_pool3d(occ, 3, stride=1, padding=1) > 0
    want0 = torch.nonzero(occ.view(-1, 32).amax(1) > 0).view(-1).int()
    want1 = torch.nonzero(act.reshape(-1, 32).any(1)).view(-1).int()
    tiles = b * v // 256
    want2 = torch.nonzero(occ.view(-1) > 0).view(-1).int()
    want3 = torch.nonzero(act.reshape(-1)).view(-1).int()
    counts = lists[:4].tolist()
    assert counts == [want0.numel(), want1.numel(), want2.numel(), want3.numel()]
    nch = b * v // 32
    l0 = lists[64 + 2 * tiles: 64 + 2 * tiles + nch]
    l1 = lists[64 + 2 * tiles + nch: 64 + 2 * tiles + 2 * nch]
    l2 = lists[64 + 4 * tiles + 2 * nch: 64 + 4 * tiles + 2 * nch + b * v]
    l3 = lists[64 + 4 * tiles + 2 * nch + b * v: 64 + 4 * tiles + 2 * nch + 2 * b * v]
    assert torch.equal(l0[: counts[0]], want0)
    assert torch.equal(l1[: counts[1]], want1)
    assert torch.equal(l2[: counts[2]], want2)
    assert torch.equal(l3[: counts[3]], want3)


@pytest.mark.parametrize("b,cin,cout,r,surface", [(4, 128, 128, 32, False),
                                                  (4, 128, 256, 16, False),
                                                  (4, 128, 128, 32, True),
                                                  (8, 256, 256, 16, False),
                                                  (4, 256, 256, 8, False)])
def test_conv_voxel_list_gemm_is_exact(ops, monkeypatch, b, cin, cout, r, surface, report):
    """The voxel-list form of PVConv's first conv: the forward bit-identical to
    the dense GEMM at every voxel (bias where no occupied voxel is near), the
    backward-data bit-identical at every occupied voxel and 0 in chunks without one
    (split-K shapes -- r = 8, and r = 16 at b = 4 -- have no list form: the
    dense GEMM runs; b = 8, r = 16 takes the 128-entry list tiles)."""
    grid, cnt, _ = _voxelized(ops, b, cin, r, 6000, r + cin + 7, surface)
    lists = ops.conv3d_vlists(cnt, r)
    xs = ops.conv3d_split(grid.contiguous())
    g = torch.Generator(device="cuda").manual_seed(11)
    w = torch.randn(cout, cin, 3, 3, 3, device="cuda", generator=g) * 0.05
    bias = torch.randn(cout, device="cuda", generator=g)
    img = ops.conv3d_prep_weight(w, False)
    y0 = ops.conv3d_igemm_split(xs, img, bias, b, cin, cout, r, "conv3d_fwd")
    for vox in ("3", "0"):  # voxel list 3 (default), chunk list 1
        monkeypatch.setenv("PCFM_LIST_VOX", vox)
        y1 = ops.conv3d_igemm_split(xs, img, bias, b, cin, cout, r, "conv3d_fwd", occ_mode=1,
                                    vlists=lists, cnt=cnt)
        assert torch.equal(y0, y1), vox
    monkeypatch.delenv("PCFM_LIST_VOX")
    dy = torch.randn(b, cout, r, r, r, device="cuda", generator=g)
    gys = ops.conv3d_split(dy)
    imgt = ops.conv3d_prep_weight(w, True)
    dx0 = ops.conv3d_igemm_split(gys, imgt, None, b, cout, cin, r, "conv3d_bwd_data")
    occupied = (cnt.view(b, 1, -1) > 0).expand(b, cin, r ** 3)
    # the voxel-list form (default) and the chunk-list form (PCFM_LIST_VOX=0)
    for vox in ("1", "0"):
        monkeypatch.setenv("PCFM_LIST_VOX", vox)
        dx1 = ops.conv3d_igemm_split(gys, imgt, None, b, cout, cin, r, "conv3d_bwd_data",
                                     occ_mode=2, vlists=lists, cnt=cnt)
        assert torch.equal(dx0.view(b, cin, -1)[occupied], dx1.view(b, cin, -1)[occupied]), vox
        # at the other voxels: 0 (voxel list: everywhere; chunk list: in the chunks
        # without an occupied voxel), else the dense value (and everywhere on
        # shapes without the list form)
        rest1, rest0 = dx1.view(b, cin, -1)[~occupied], dx0.view(b, cin, -1)[~occupied]
        assert bool(((rest1 == 0) | (rest1 == rest0)).all()), vox
    monkeypatch.delenv("PCFM_LIST_VOX")
    report(f"conv_voxel_lists_b{b}_c{cin}_r{r}{'_surface' if surface else ''}",
           {"occupied_fraction": float((cnt > 0).float().mean()),
            "listed_fwd_chunk_fraction": int(lists[1]) * 32 / float(b * r ** 3),
            "listed_bwd_chunk_fraction": int(lists[0]) * 32 / float(b * r ** 3)})


@pytest.mark.parametrize("cin,cout,r,n", [(128, 128, 32, 20000), (256, 256, 16, 8000),
                                          (256, 256, 8, 5000)])
def test_voxel_branch_node_matches_two_node_form(ops, monkeypatch, cin, cout, r, n):
    """The PVConv voxel branch as one node (_VoxelBranchSEDevox: BN2's activation
    never written, SE pooling and BN2 backward sums from single passes) against
    the round-4 two-node form (_Conv3dBnActPair + _SEDevoxAdd) at the C2 stage
    shapes: outputs, every gradient and the running statistics to fp32
    summation order (SE's pooling and BN2's backward sums are taken in another
    order)."""
    import modules.pvconv as pv
    torch.manual_seed(r)
    mod = pv.PVConv(cin, cout, 3, r, with_se=True, normalize=True).cuda().train()
    g = torch.Generator(device="cuda").manual_seed(r)
    feats = torch.randn(2, cin, n, device="cuda", generator=g)
    coords = torch.randn(2, 3, n, device="cuda", generator=g)
    gy = torch.randn(2, cout, n, device="cuda", generator=g)
    state = {k: v.clone() for k, v in mod.state_dict().items()}

    def run():
        mod.load_state_dict(state)
        f = feats.clone().requires_grad_(True)
        out, _ = mod((f, coords))
        node = type(out.grad_fn).__name__
        out.backward(gy)
        grads = [("input", f.grad)] + [(k, p.grad.clone()) for k, p in mod.named_parameters()]
        bufs = {k: v.clone() for k, v in mod.state_dict().items()}
        mod.zero_grad(set_to_none=True)
        return out.detach(), grads, bufs, node

    o1, g1, b1, n1 = run()
    monkeypatch.setattr(pv, "_PV_FUSED", False)
    o0, g0, b0, n0 = run()
    assert n1 == "_VoxelBranchSEDevoxBackward" and n0 != n1, (n1, n0)
    assert _rel(o1, o0) < 1e-5
    zero_grad = {"voxel_layers.0.bias", "voxel_layers.3.bias", "point_features.layers.0.bias"}
    for (name, a), (_, b) in zip(g1, g0):
        if name in zero_grad:
            assert (a - b).abs().max().item() < 1e-3, name
        else:
            assert _rel(a, b) < 1e-4, (name, _rel(a, b))
    for k in b0:  # running statistics (and the unchanged parameters)
        if b0[k].dtype.is_floating_point:
            torch.testing.assert_close(b1[k], b0[k], rtol=1e-6, atol=1e-7, msg=k)
        else:
            assert torch.equal(b1[k], b0[k]), k
