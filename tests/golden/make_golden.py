"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own code.

Run in the build container, where the reference tree is mounted read-only:

    python tests/golden/make_golden.py /root/reference

It never runs on the GPU box (the reference is not there) and nothing under
tests/ reads the reference at test time -- only these .npz files.

What is pinned by what:
  * chamfer_python.npz   -- reference ChamferDistancePytorch/chamfer_python.py
    (distChamfer: float64 expanded-form pairwise distances; the reference's
    own CUDA unit test asserts its kernel against exactly this,
    unit_test.py:14-35).  Seeded versions of the unit test's shapes plus
    duplicate-point (tie) and near-duplicate cases.
  * emd_known.npz        -- reference PyTorchEMD/test_emd_loss.py known answer:
    its inputs and its exact-assignment ground truth `gt_dist` and gradients
    (the script's own arithmetic, restated here because the script imports the
    JIT-built extension at import time).
  * pvconv_r8.npz / model_hybrid_c1.npz / model_hybrid_c1_perturbed.npz --
    the reference's Python modules
    (pvcnn modules.PVConv; models.HybridMLP) run on the CPU with the native
    `_pvcnn_backend` replaced by this build's C oracle (oracle/pcfm_oracle.c).
    These pin the Python composition (coordinate normalisation and rounding,
    layer order, mixed precision, parameter initialisation order from a seed)
    -- not the CUDA kernels, which cannot be built here (DESIGN.md "Oracle").
"""
from __future__ import annotations

import os
import sys
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def chamfer_fixtures(ref: str) -> None:
    sys.path.insert(0, os.path.join(ref, "third_party", "ChamferDistancePytorch"))
    import chamfer_python  # reference, pure torch

    cases = {}
    g = torch.Generator().manual_seed(20251024)
    shapes = [("unit", 4, 100, 200, "rand"), ("wide", 2, 257, 1025, "randn"),
              ("small", 3, 7, 5, "randn"), ("timing_shape", 2, 2000, 1000, "rand")]
    for name, b, n, m, kind in shapes:
        f = torch.rand if kind == "rand" else torch.randn
        a = f(b, n, 3, generator=g)
        c = f(b, m, 3, generator=g)
        cases[name] = (a, c)
    # ties: exact duplicates in xyz2 -> lowest index must win
    a = torch.randn(2, 64, 3, generator=g)
    c = torch.randn(2, 32, 3, generator=g)
    c = torch.cat([c, c, c[:, :8]], dim=1)
    cases["ties"] = (a, c)
    out = {}
    for name, (a, c) in cases.items():
        d1, d2, i1, i2 = chamfer_python.distChamfer(a, c)
        out[f"{name}_xyz1"] = a.numpy()
        out[f"{name}_xyz2"] = c.numpy()
        out[f"{name}_dist1"] = d1.numpy()
        out[f"{name}_dist2"] = d2.numpy()
        out[f"{name}_idx1"] = i1.numpy()
        out[f"{name}_idx2"] = i2.numpy()
    np.savez_compressed(os.path.join(HERE, "chamfer_python.npz"), **out)
    sys.path.pop(0)


def emd_fixture() -> None:
    # test_emd_loss.py:6-21: two 2-point clouds, batch of 3, weights 1/2, 2, 1/3
    p1 = torch.tensor([[[1.7, -0.1, 0.1], [0.1, 1.2, 0.3]]], dtype=torch.float32).repeat(3, 1, 1)
    p2 = torch.tensor([[[0.3, 1.8, 0.2], [1.2, -0.2, 0.3]]], dtype=torch.float32).repeat(3, 1, 1)
    p1.requires_grad_(True)
    p2.requires_grad_(True)
    per = (((p1[:, 0] - p2[:, 1]) ** 2).sum(-1) + ((p1[:, 1] - p2[:, 0]) ** 2).sum(-1))
    gt = per[0] / 2 + per[1] * 2 + per[2] / 3
    gt.backward()
    np.savez_compressed(
        os.path.join(HERE, "emd_known.npz"),
        p1=p1.detach().numpy(), p2=p2.detach().numpy(),
        weights=np.array([0.5, 2.0, 1.0 / 3.0], np.float32),
        gt_dist=np.float32(gt.item()), gt_per_element=(per.detach() / 2).numpy(),
        gt_grad1=p1.grad.numpy(), gt_grad2=p2.grad.numpy())


def _install_oracle_backend():
    sys.path.insert(0, REPO)
    from oracle.oracle import TorchBackend
    stub = types.ModuleType("modules.functional.backend")
    stub._backend = TorchBackend()
    sys.modules["modules.functional.backend"] = stub


def _param_sums(module):
    return np.array([p.detach().double().sum().item() for _, p in module.named_parameters()],
                    np.float64)


def pvcnn_fixtures(ref: str) -> None:
    _install_oracle_backend()
    sys.path.insert(0, os.path.join(ref, "third_party", "pvcnn"))
    sys.path.insert(0, ref)
    from modules.pvconv import PVConv  # reference
    import models  # reference models.py

    # --- one PVConv block (R=8, with SE), train mode, forward + backward ---
    torch.manual_seed(7)
    blk = PVConv(16, 16, kernel_size=3, resolution=8, with_se=True, normalize=True, eps=1e-6)
    feats = torch.randn(2, 16, 300, requires_grad=True)
    coords = torch.randn(2, 3, 300)
    out, _ = blk((feats, coords))
    loss = (out * torch.linspace(-1, 1, out.numel()).view_as(out)).sum()
    loss.backward()
    np.savez_compressed(
        os.path.join(HERE, "pvconv_r8.npz"), seed=7, feats=feats.detach().numpy(),
        coords=coords.numpy(), out=out.detach().numpy(), grad_feats=feats.grad.numpy(),
        param_sums=_param_sums(blk),
        grad_sums=np.array([p.grad.double().sum().item() for p in blk.parameters()]))

    # --- full default HybridMLP at C1 size (B=2, N=1024, xyz+rgb) ---
    torch.manual_seed(1234)
    pf = models.HybridMLP(cond_dim=129, point_dim=6)
    pf.train()
    g = torch.Generator().manual_seed(99)
    x = torch.randn(2, 1024, 6, generator=g)
    t = torch.rand(2, generator=g)
    cond = torch.randn(2, 129, generator=g)
    mask = torch.tensor([[0.0], [1.0]])
    v = pf(x, t, cond, cond_drop_mask=mask)
    target = torch.randn(2, 1024, 6, generator=g)
    loss = torch.nn.functional.mse_loss(v, target)
    loss.backward()
    names = [n for n, _ in pf.named_parameters()]
    np.savez_compressed(
        os.path.join(HERE, "model_hybrid_c1.npz"), seed=1234, x=x.numpy(), t=t.numpy(),
        cond=cond.numpy(), mask=mask.numpy(), target=target.numpy(),
        v=v.detach().numpy(), loss=np.float32(loss.item()), param_names=np.array(names),
        param_sums=_param_sums(pf),
        grad_sums=np.array([p.grad.double().sum().item() if p.grad is not None else 0.0
                            for p in pf.parameters()]),
        grad_norms=np.array([p.grad.double().norm().item() if p.grad is not None else 0.0
                             for p in pf.parameters()]))


def perturb_zero_init_(module, seed: int = 5, std: float = 0.05) -> None:
    """Give every all-zero parameter (zero-initialised FiLM affines, head_out,
    output biases, ...) seeded N(0, std^2) values, in named_parameters order.  At
    the reference's initialisation ContextNet.head_out is zero, so the velocity
    does not depend on the PVConv pyramid at all (models.py:450-451); the
    perturbed golden makes every branch visible in v.  tests/ restate this
    helper (same generator, same order)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for _, p in module.named_parameters():
            if not bool(p.detach().abs().sum()):
                p.copy_(torch.randn(p.shape, generator=g) * std)


def hybrid_perturbed_fixture(ref: str) -> None:
    """model_hybrid_c1_perturbed.npz: as model_hybrid_c1.npz, with the zero-init
    parameters perturbed (perturb_zero_init_) so v depends on every branch."""
    import models  # reference (already on sys.path from pvcnn_fixtures)
    torch.manual_seed(1234)
    pf = models.HybridMLP(cond_dim=129, point_dim=6)
    perturb_zero_init_(pf)
    pf.train()
    g = torch.Generator().manual_seed(77)
    x = torch.randn(2, 1024, 6, generator=g)
    t = torch.rand(2, generator=g)
    cond = torch.randn(2, 129, generator=g)
    mask = torch.tensor([[1.0], [0.0]])
    v = pf(x, t, cond, cond_drop_mask=mask)
    target = torch.randn(2, 1024, 6, generator=g)
    loss = torch.nn.functional.mse_loss(v, target)
    loss.backward()
    np.savez_compressed(
        os.path.join(HERE, "model_hybrid_c1_perturbed.npz"), seed=1234, perturb_seed=5,
        x=x.numpy(), t=t.numpy(), cond=cond.numpy(), mask=mask.numpy(), target=target.numpy(),
        v=v.detach().numpy(), loss=np.float32(loss.item()), param_sums=_param_sums(pf),
        grad_norms=np.array([p.grad.double().norm().item() if p.grad is not None else 0.0
                             for p in pf.parameters()]))


def main() -> None:
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    torch.set_num_threads(1)  # deterministic CPU reductions
    only = sys.argv[2:]  # optional subset, e.g. `hybrid_perturbed`
    if not only:
        chamfer_fixtures(ref)
        emd_fixture()
        pvcnn_fixtures(ref)
    else:
        _install_oracle_backend()
        sys.path.insert(0, os.path.join(ref, "third_party", "pvcnn"))
        sys.path.insert(0, ref)
    hybrid_perturbed_fixture(ref)
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))


if __name__ == "__main__":
    main()
