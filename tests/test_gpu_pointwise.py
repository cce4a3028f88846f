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
