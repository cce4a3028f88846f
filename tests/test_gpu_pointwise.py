"""bf16x3 pointwise convolution (csrc/pointwise.hip) against fp64.

Tolerance as for the voxel convolution: max |err| / rms(reference) < 1e-4
(~2^-16 relative per product; TF32 -- the reference's cuDNN default -- is 2^-11)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _rel(a, ref):
    a = a.detach().double().cpu()
    return ((a - ref).abs().max() / ref.pow(2).mean().sqrt()).item()


@pytest.fixture(scope="module")
def ops():
    from pcfm import _lib, ops
    _lib.load()
    return ops


@pytest.mark.parametrize("b,cin,cout,n", [(2, 262, 128, 1000), (1, 896, 256, 777), (3, 256, 64, 129),
                                          (2, 128, 128, 64), (1, 5, 3, 7), (8, 256, 256, 20000),
                                          # streaming form (M <= 128, K <= 256, multiples of 32):
                                          # ragged point tiles, 8 K-chunks in the backward-data
                                          (2, 128, 256, 1000), (1, 96, 32, 45),
                                          (8, 128, 128, 20000)])
def test_pointwise_vs_fp64(ops, b, cin, cout, n):
    g = torch.Generator(device="cuda").manual_seed(cin * 7 + cout + n)
    x = torch.randn(b, cin, n, device="cuda", generator=g)
    w = torch.randn(cout, cin, 1, device="cuda", generator=g) / cin ** 0.5
    bias = torch.randn(cout, device="cuda", generator=g)
    gy = torch.randn(b, cout, n, device="cuda", generator=g)
    bs = slice(0, min(b, 2))
    x64, w64, g64 = x[bs].double().cpu(), w[:, :, 0].double().cpu(), gy[bs].double().cpu()
    y64 = torch.einsum("oc,bcn->bon", w64, x64) + bias.double().cpu()[:, None]
    assert _rel(ops.pointwise_forward(x, w, bias)[bs], y64) < TOL
    dx64 = torch.einsum("oc,bon->bcn", w64, g64)
    assert _rel(ops.pointwise_backward_data(gy, w)[bs], dx64) < TOL
    dw64 = torch.einsum("bon,bcn->oc", g64, x64)
    dw = ops.pointwise_backward_weight(x[bs].contiguous(), gy[bs].contiguous())
    assert _rel(dw, dw64) < TOL


def test_pointwise_module_matches_conv1d(ops):
    from modules.shared_mlp import PointwiseConv1d
    torch.manual_seed(0)
    ref = torch.nn.Conv1d(262, 128, 1).cuda()
    mod = PointwiseConv1d(262, 128, 1).cuda()
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(2, 262, 3000, device="cuda")
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = ref(xa), mod(xb)
    gy = torch.randn_like(ya)
    ya.backward(gy)
    yb.backward(gy)
    for a, b in ((ya, yb), (xa.grad, xb.grad), (ref.weight.grad, mod.weight.grad),
                 (ref.bias.grad, mod.bias.grad)):
        assert _rel(b, a.detach().double().cpu()) < 2 * TOL


def test_pointwise_module_keeps_autocast(ops):
    from modules.shared_mlp import PointwiseConv1d
    mod = PointwiseConv1d(64, 32, 1).cuda()
    x = torch.randn(2, 64, 100, device="cuda")
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert mod(x).dtype == torch.bfloat16
    assert mod(x).dtype == torch.float32


@pytest.mark.parametrize("widths,cout,n,b", [((128, 256, 256), 256, 2000, 2), ((128, 96), 64, 333, 2),
                                             ((32, 32, 32, 7), 130, 65, 2),
                                             ((128, 256, 256), 256, 20000, 4)])
def test_pointwise_parts_vs_fp64(ops, widths, cout, n, b):
    """Channel-segmented GEMMs (ContextNet head_pre without the concat); the last
    case is large enough for the 256-row tile."""
    g = torch.Generator(device="cuda").manual_seed(sum(widths) + cout + n)
    xs = [torch.randn(b, w, n, device="cuda", generator=g) for w in widths]
    cin = sum(widths)
    w = torch.randn(cout, cin, device="cuda", generator=g) / cin ** 0.5
    bias_b = torch.randn(b, cout, device="cuda", generator=g)
    gy = torch.randn(b, cout, n, device="cuda", generator=g)
    x64 = torch.cat(xs, 1).double().cpu()
    w64, g64 = w.double().cpu(), gy.double().cpu()
    y64 = torch.einsum("oc,bcn->bon", w64, x64) + bias_b.double().cpu()[:, :, None]
    assert _rel(ops.pointwise_forward_parts(xs, w, bias_b, bias_per_batch=True), y64) < TOL
    dx64 = torch.einsum("oc,bon->bcn", w64, g64)
    if all(v % 128 == 0 for v in widths[:-1]):
        dxs = ops.pointwise_backward_data_parts(gy, w, list(widths))
        assert [d.shape[1] for d in dxs] == list(widths)
        assert _rel(torch.cat(dxs, 1), dx64) < TOL
    dw64 = torch.einsum("bon,bcn->oc", g64, x64)
    assert _rel(ops.pointwise_backward_weight_parts(xs, gy), dw64) < TOL


def test_context_head_pre_parts_matches_concat(ops):
    from pcfm.models import ContextNet
    torch.manual_seed(3)
    net = ContextNet(3, 0, emb_dim=32, ctx_dim=16).cuda()
    b, n = 2, 1500
    scales = [torch.randn(b, c, n, device="cuda", requires_grad=True) for c in net.stage_channels]
    g = torch.randn(b, net.stage_channels[-1], device="cuda", requires_grad=True)
    y = net._head_pre(scales, g)
    gy = torch.randn_like(y)
    grads = torch.autograd.grad(y, [*scales, g, net.head_pre.weight, net.head_pre.bias], gy)
    ref_in = torch.cat([s.detach().double() for s in scales]
                       + [g.detach().double()[:, :, None].expand(b, -1, n)], 1).requires_grad_(True)
    w64 = net.head_pre.weight.detach().double().requires_grad_(True)
    b64 = net.head_pre.bias.detach().double().requires_grad_(True)
    y64 = torch.nn.functional.conv1d(ref_in, w64, b64)
    r = torch.autograd.grad(y64, [ref_in, w64, b64], gy.double())
    cs = sum(net.stage_channels)
    refs = list(torch.split(r[0][:, :cs], net.stage_channels, 1)) + [r[0][:, cs:].sum(2), r[1], r[2]]
    assert _rel(y, y64.detach().cpu()) < TOL
    for a, ref in zip(grads, refs):
        assert _rel(a, ref.detach().cpu()) < 2 * TOL


def test_context_stem_fold_matches_concat(ops, monkeypatch):
    """ContextNet's stage-1 lift with the embedding columns folded into a per-cloud
    bias (ContextNet._stem_proj).  (1) The fold itself against the fp64 conv over
    the built stem cat([emb broadcast, xyz, rgb]), forward and backward.  (2) The
    whole (training-mode) ContextNet against its module path, forward.  Network-level
    parameter gradients are not compared: behind training-mode BatchNorms they are
    sums that cancel (BN's backward sums to zero over the points), so a 1e-7
    change in the lift's rounding moves them by up to a few percent in either path;
    (1) checks the fold's own gradients against fp64.)"""
    from pcfm.models import ContextNet, _PointwiseParts
    g = torch.Generator(device="cuda").manual_seed(11)
    b, n, e = 2, 3000, 64
    pts = torch.randn(b, 6, n, device="cuda", generator=g).requires_grad_(True)
    emb = torch.randn(b, e, device="cuda", generator=g).requires_grad_(True)
    w = (torch.randn(128, e + 6, device="cuda", generator=g) / 8).requires_grad_(True)
    bias = torch.randn(128, device="cuda", generator=g).requires_grad_(True)
    gy = torch.randn(b, 128, n, device="cuda", generator=g)
    pre = _PointwiseParts.apply(w[:, e:], torch.addmm(bias, emb, w[:, :e].t()), pts)
    got = torch.autograd.grad(pre, [pts, emb, w, bias], gy)
    d = [t.detach().double().requires_grad_(True) for t in (pts, emb, w, bias)]
    stem = torch.cat([d[1][:, :, None].expand(b, e, n), d[0]], dim=1)
    ref = torch.nn.functional.conv1d(stem, d[2][:, :, None], d[3])
    want = torch.autograd.grad(ref, d, gy.double())
    assert _rel(pre, ref.detach().cpu()) < TOL
    for a, r in zip(got, want):
        assert _rel(a, r.detach().cpu()) < TOL

    torch.manual_seed(5)
    net = ContextNet(6, 1, emb_dim=64, ctx_dim=16, stage_channels=(128, 128, 128),
                     stage_blocks=(1, 1, 1), stage_res=(8, 8, 8)).cuda().train()
    with torch.no_grad():
        net.head_out.weight.normal_(0.0, 0.1)
    x = torch.randn(b, n, 6, device="cuda")
    t = torch.rand(b, device="cuda")
    cond = torch.rand(b, 1, device="cuda")
    state = {k: v.clone() for k, v in net.state_dict().items()}

    def run():
        net.load_state_dict(state)
        with torch.no_grad():
            return net(x, t, cond)

    o1 = run()
    monkeypatch.setattr(ContextNet, "_stem_proj", lambda self, *a: None)
    o0 = run()
    assert _rel(o1, o0.double().cpu()) < 1e-4


@pytest.mark.parametrize("b,cin,cout,n", [(8, 256, 256, 20000), (8, 128, 256, 20000),
                                          (8, 256, 128, 20000),  # backward-data: M = cin = 256
                                          (5, 200, 256, 16388),  # channel tail, ragged tile
                                          (16, 64, 256, 4100)])  # one K-step, more tiles than CUs
def test_pointwise_256_row_shapes(ops, b, cin, cout, n):
    """The 256-row tile (pw_gemm256_kernel) over shapes with a channel tail, a
    ragged point tile and one K-step: forward against fp64, the BatchNorm group
    statistics present for the 256-row output, backward-data through the same
    path.  (Its persistent LDS-DMA twin, bit-identical here in round 5 and
    slower, was removed in round 6.)"""
    g = torch.Generator(device="cuda").manual_seed(b + cin + cout + n)
    x = torch.randn(b, cin, n, device="cuda", generator=g)
    w = torch.randn(cout, cin, 1, device="cuda", generator=g) / cin ** 0.5
    bias = torch.randn(cout, device="cuda", generator=g)
    gy = torch.randn(b, cout, n, device="cuda", generator=g)
    y = ops.pointwise_forward(x, w, bias)
    fs = ops.pointwise_forward_bnstats(x, w, bias)
    assert fs is not None or cout != 256
    if fs is not None:  # per (channel, 64-point group): the group's mean and centred sum of squares
        assert torch.equal(fs[0], y)
        st = fs[1]
        ng = st.shape[1] // b
        G = (n + ng - 1) // ng
        yd = torch.nn.functional.pad(y.double(), (0, ng * G - n)).view(b, cout, ng, G)
        cnt = torch.full((ng,), float(G), device="cuda", dtype=torch.float64)
        cnt[-1] = n - (ng - 1) * G
        mean = yd.sum(-1) / cnt
        valid = (torch.arange(G, device="cuda")[None, :]
                 + G * torch.arange(ng, device="cuda")[:, None]) < n
        m2 = (((yd - mean[..., None]) ** 2) * valid).sum(-1)
        ref = torch.stack([mean, m2], -1).permute(1, 0, 2, 3).reshape(cout, b * ng, 2)
        scale = y.double().abs().max()
        assert torch.allclose(st[..., 0].double(), ref[..., 0], rtol=1e-5, atol=1e-6 * scale)
        assert torch.allclose(st[..., 1].double(), ref[..., 1], rtol=1e-4,
                              atol=1e-5 * scale ** 2 * G)
    dx = ops.pointwise_backward_data(gy, w)
    x64, w64 = x[:1].double().cpu(), w[:, :, 0].double().cpu()
    y64 = torch.einsum("oc,bcn->bon", w64, x64) + bias.double().cpu()[:, None]
    assert _rel(y[:1], y64) < TOL
    dx64 = torch.einsum("oc,bon->bcn", w64, gy[:1].double().cpu())
    assert _rel(dx[:1], dx64) < TOL