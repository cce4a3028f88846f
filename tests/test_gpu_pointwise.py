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
                                          (2, 128, 128, 64), (1, 5, 3, 7), (8, 256, 256, 20000)])
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
