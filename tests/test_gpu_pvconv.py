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
    # the voxelization's scatter sums are order-nondeterministic at the last bit
    # (segsum.hpp, like the reference's float atomics): compare at fp32 rounding
    assert _rel(o1, o0) < 1e-4
    assert _rel(g1, g0) < 1e-4
