"""bf16x3 voxel convolution (csrc/conv3d.hip) against an fp64 reference.

Tolerance: max |err| / rms(reference) < 1e-4.  The split-bf16 products carry
~2^-16 relative error each (measured ~2.5e-5 of the output rms at C=128..256,
K = 27*C terms; MIOpen fp32 measures 1e-6..1.7e-5 on the same data); the
reference's own cuDNN path runs TF32 (2^-11 per product) by default.
"""
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


@pytest.mark.parametrize("b,cin,cout,r", [(2, 128, 128, 8), (1, 128, 256, 8), (1, 256, 128, 8),
                                          (2, 128, 128, 16), (1, 256, 256, 8), (1, 128, 128, 32),
                                          (1, 128, 128, 24), (8, 256, 256, 8)])
def test_conv3d_fwd_bwd_vs_fp64(ops, b, cin, cout, r):
    g = torch.Generator(device="cuda").manual_seed(b * 1000 + cin + r)
    x = torch.randn(b, cin, r, r, r, device="cuda", generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, device="cuda", generator=g) / (27 * cin) ** 0.5
    bias = torch.randn(cout, device="cuda", generator=g)
    gy = torch.randn(b, cout, r, r, r, device="cuda", generator=g)
    x64, w64, g64 = x.double().cpu(), w.double().cpu(), gy.double().cpu()
    y64 = torch.nn.functional.conv3d(x64, w64, bias.double().cpu(), padding=1)
    assert _rel(ops.conv3d_forward(x, w, bias), y64) < TOL
    dx64 = torch.nn.grad.conv3d_input(x64.shape, w64, g64, padding=1)
    assert _rel(ops.conv3d_backward_data(gy, w), dx64) < TOL
    if cin % 128 == 0:
        dw64 = torch.nn.grad.conv3d_weight(x64, w64.shape, g64, padding=1)
        assert _rel(ops.conv3d_backward_weight(x, gy), dw64) < TOL
        if cout % 128 == 0:  # split-operand path (what VoxelConv3d's autograd runs)
            xs, gys = ops.conv3d_split(x), ops.conv3d_split(gy)
            assert _rel(ops.conv3d_wgrad_split(xs, gys, b, cin, cout, r), dw64) < TOL
            img = ops.conv3d_prep_weight(w, False)
            y = ops.conv3d_igemm_split(xs, img, bias, b, cin, cout, r, "t")
            assert _rel(y, y64) < TOL


def test_conv3d_padding_is_zero(ops):
    """All-ones input and kernel: each output = number of in-grid neighbours * C."""
    r, c = 8, 128
    x = torch.ones(1, c, r, r, r, device="cuda")
    w = torch.ones(c, c, 3, 3, 3, device="cuda")
    y = ops.conv3d_forward(x, w, None)
    idx = torch.arange(r, device="cuda")
    n1 = 3 - (idx == 0).int() - (idx == r - 1).int()
    cnt = (n1[:, None, None] * n1[None, :, None] * n1[None, None, :]).float() * c
    assert torch.equal(y[0, 0], cnt) and torch.equal(y[0, c - 1], cnt)


@pytest.mark.parametrize("b,r", [(2, 16), (1, 8), (1, 24)])
def test_conv3d_wgrad_padding_counts(ops, b, r):
    """All-ones x and grad_y: dW[co, ci, tap] = b * prod over axes of (r - |d|) exactly
    (the three-tap kernel's halo rows and z/y/x edge masking)."""
    c = 128
    x = torch.ones(b, c, r, r, r, device="cuda")
    gy = torch.ones(b, c, r, r, r, device="cuda")
    xs, gys = ops.conv3d_split(x), ops.conv3d_split(gy)
    dw = ops.conv3d_wgrad_split(xs, gys, b, c, c, r).view(c, c, 3, 3, 3)
    n = torch.tensor([r - 1, r, r - 1], dtype=torch.float32, device="cuda")
    want = b * n[:, None, None] * n[None, :, None] * n[None, None, :]
    assert torch.equal(dw[0, 0], want) and torch.equal(dw[c - 1, 5], want)
    assert torch.equal(dw, want.expand_as(dw))


def test_conv3d_unsupported_shape_rejected(ops):
    from pcfm import _lib
    assert _lib.query("pcfm_conv3d_supported", 1, 16, 16, 8) == 0
    x = torch.randn(1, 16, 8, 8, 8, device="cuda")
    w = torch.randn(16, 16, 3, 3, 3, device="cuda")
    assert not ops.conv3d_supported(x, w)
    with pytest.raises(_lib.PcfmError, match="unsupported"):
        ops.conv3d_forward(x, w, None)


def test_voxel_conv_module_matches_conv3d(ops):
    """VoxelConv3d (x3 path) vs nn.Conv3d (MIOpen fp32) with the same parameters:
    output, input grad and weight/bias grads."""
    from modules.voxel_conv import VoxelConv3d
    torch.manual_seed(0)
    ref = torch.nn.Conv3d(128, 128, 3, padding=1).cuda()
    mod = VoxelConv3d(128, 128, 3, padding=1).cuda()
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(2, 128, 16, 16, 16, device="cuda")
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = ref(xa), mod(xb)
    gy = torch.randn_like(ya)
    ya.backward(gy)
    yb.backward(gy)
    for a, b in ((ya, yb), (xa.grad, xb.grad), (ref.weight.grad, mod.weight.grad),
                 (ref.bias.grad, mod.bias.grad)):
        a64 = a.detach().double().cpu()
        assert _rel(b, a64) < 2 * TOL


@pytest.mark.parametrize("b,cin,cout,r", [(2, 128, 128, 32), (2, 256, 256, 16), (1, 128, 256, 16),
                                          (1, 256, 128, 32)])
def test_slab_form_is_bit_identical(ops, monkeypatch, b, cin, cout, r):
    """The slab form of the dense r = 32 / 16 GEMM (conv3_igemm_slab_kernel: B from a
    per-(chunk, dx) 2-D slab in LDS) runs the LDS-DMA kernel's K-steps in the same
    order with the same operands: forward and backward-data outputs bit-identical,
    including the volume's border voxels (zero rows of the slab)."""
    g = torch.Generator(device="cuda").manual_seed(7 * r + cin)
    x = torch.randn(b, cin, r, r, r, device="cuda", generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, device="cuda", generator=g) / (27 * cin) ** 0.5
    bias = torch.randn(cout, device="cuda", generator=g)
    xs = ops.conv3d_split(x)
    img, imgt = ops.conv3d_prep_weight(w, False), ops.conv3d_prep_weight(w, True)
    gys = ops.conv3d_split(torch.randn(b, cout, r, r, r, device="cuda", generator=g))
    out = {}
    for slab in ("1", "0"):
        monkeypatch.setenv("PCFM_CONV_SLAB", slab)
        out[slab] = (ops.conv3d_igemm_split(xs, img, bias, b, cin, cout, r, "t"),
                     ops.conv3d_igemm_split(gys, imgt, None, b, cout, cin, r, "t"))
    assert torch.equal(out["1"][0], out["0"][0])
    assert torch.equal(out["1"][1], out["0"][1])
    y64 = torch.nn.functional.conv3d(x.double().cpu(), w.double().cpu(), bias.double().cpu(),
                                     padding=1)
    assert _rel(out["1"][0], y64) < TOL


@pytest.mark.parametrize("r", [16, 32])
def test_slab_form_padding_counts(ops, r):
    """All-ones input and kernel at the slab form's resolutions: every output is the
    number of in-grid neighbours times C (zero rows at all six faces)."""
    c = 128
    x = torch.ones(1, c, r, r, r, device="cuda")
    w = torch.ones(c, c, 3, 3, 3, device="cuda")
    y = ops.conv3d_forward(x, w, None)
    idx = torch.arange(r, device="cuda")
    n1 = 3 - (idx == 0).int() - (idx == r - 1).int()
    cnt = (n1[:, None, None] * n1[None, :, None] * n1[None, None, :]).float() * c
    assert torch.equal(y[0, 0], cnt) and torch.equal(y[0, c - 1], cnt)


@pytest.mark.parametrize("b,cin,cout,r", [(8, 256, 256, 8), (2, 256, 128, 8), (4, 128, 256, 8),
                                          (3, 128, 128, 8)])
def test_window_form_is_bit_identical(ops, monkeypatch, b, cin, cout, r):
    """The window form of the small-grid split-K GEMM (conv3_igemm_win_kernel: B
    for all 27 taps from one staged window of the input per 32-channel chunk) runs
    the LDS-DMA kernel's K-steps in the same order with the same operands (zeroed
    fragments where that kernel reads its zero row): forward and backward-data
    outputs bit-identical, incl. the border voxels, and the fp64 pin."""
    g = torch.Generator(device="cuda").manual_seed(11 * r + cin + cout)
    x = torch.randn(b, cin, r, r, r, device="cuda", generator=g)
    w = torch.randn(cout, cin, 3, 3, 3, device="cuda", generator=g) / (27 * cin) ** 0.5
    bias = torch.randn(cout, device="cuda", generator=g)
    xs = ops.conv3d_split(x)
    img, imgt = ops.conv3d_prep_weight(w, False), ops.conv3d_prep_weight(w, True)
    gys = ops.conv3d_split(torch.randn(b, cout, r, r, r, device="cuda", generator=g))
    out = {}
    for win in ("1", "0"):
        monkeypatch.setenv("PCFM_CONV_WIN", win)
        out[win] = (ops.conv3d_igemm_split(xs, img, bias, b, cin, cout, r, "t"),
                    ops.conv3d_igemm_split(gys, imgt, None, b, cout, cin, r, "t"))
    assert torch.equal(out["1"][0], out["0"][0])
    assert torch.equal(out["1"][1], out["0"][1])
    y64 = torch.nn.functional.conv3d(x.double().cpu(), w.double().cpu(), bias.double().cpu(),
                                     padding=1)
    assert _rel(out["1"][0], y64) < TOL


def test_window_form_padding_counts(ops):
    """All-ones input and kernel at r = 8: every output is the number of in-grid
    neighbours times C (the masked linear-index neighbours at all six faces)."""
    c, r = 256, 8
    x = torch.ones(2, c, r, r, r, device="cuda")
    w = torch.ones(c, c, 3, 3, 3, device="cuda")
    y = ops.conv3d_forward(x, w, None)
    idx = torch.arange(r, device="cuda")
    n1 = 3 - (idx == 0).int() - (idx == r - 1).int()
    cnt = (n1[:, None, None] * n1[None, :, None] * n1[None, None, :]).float() * c
    assert torch.equal(y[0, 0], cnt) and torch.equal(y[1, c - 1], cnt)

