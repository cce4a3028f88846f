"""GPU: the drop-in modules and the flow model on the HIP path against the
reference-Python goldens, and the train step at small scale."""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _fp32_exact():
    # cuDNN/MIOpen and hipBLASLt must not trade fp32 for a reduced format here,
    # and MIOpen picks its solvers by heuristic, not by a timed search (which
    # can choose per run, so the gradient norms below moved 4.6e-4 -> 1.2e-3
    # between two runs of the same suite); conftest restores the flags
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cudnn.benchmark = False
    yield


def _param_sums(module):
    return np.array([p.detach().double().sum().item() for _, p in module.named_parameters()])


def test_native_library_is_what_runs():
    import modules.functional.backend as be
    from pcfm import _lib, ops
    if os.environ.get("PCFM_TORCH_BACKEND") == "1":  # the torch-extension binding
        assert be._backend.extension is be._torch_backend is not None
    else:
        assert be._backend is ops.backend
    lib = _lib.load()
    assert lib._name.endswith("libpcfm_hip.so")


def _rel_max(got, ref):
    """max |got - ref| / max |ref|: the norm-wise relative error the tolerances use."""
    return float(np.abs(got - ref).max() / np.abs(ref).max())


# biases of convolutions that feed a BatchNorm: analytically zero gradient
_NOISE_BIAS = ("layers.0.bias", "voxel_layers.0.bias", "voxel_layers.3.bias")


@pytest.mark.parametrize("mode", ["exact_fp32", "bf16x3"])
def test_pvconv_gpu_matches_reference(golden, report, mode):
    """PVConv(16, 16, r=8, SE) vs the reference module's output (pvconv_r8.npz):
    exact-fp32 convolutions within 1e-5, the bf16x3 default within 1e-4."""
    from modules.pvconv import PVConv
    from pcfm.precision import exact_fp32
    g = golden("pvconv_r8.npz")
    torch.manual_seed(int(g["seed"]))
    blk = PVConv(16, 16, kernel_size=3, resolution=8, with_se=True, normalize=True, eps=1e-6)
    np.testing.assert_allclose(_param_sums(blk), g["param_sums"], rtol=1e-12, atol=1e-12)
    blk = blk.to(DEV)
    feats = torch.from_numpy(g["feats"]).to(DEV).requires_grad_(True)
    with exact_fp32(mode == "exact_fp32"):
        out, _ = blk((feats, torch.from_numpy(g["coords"]).to(DEV)))
        loss = (out * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum()
        loss.backward()
    e_out = _rel_max(out.detach().cpu().numpy(), g["out"])
    e_grad = _rel_max(feats.grad.cpu().numpy(), g["grad_feats"])
    # every parameter gradient element by element (pvconv_r8_grads.npz), normalised
    # by the parameter's max |gradient|; the two conv biases that feed a BatchNorm
    # have an analytically zero gradient (noise) and are left out
    from golden_util import grad_errors_full, worst
    e_pg, w_pg = worst(grad_errors_full(blk, golden("pvconv_r8_grads.npz")))
    report(f"pvconv_r8_{mode}", {"out": e_out, "grad_feats": e_grad, "param_grads": e_pg,
                                 "param_grads_worst": w_pg})
    tol = 1e-5 if mode == "exact_fp32" else 1e-4
    assert e_out < tol and e_grad < tol and e_pg < tol, (e_out, e_grad, e_pg, w_pg)


@pytest.mark.parametrize("perturbed", [False, True])
@pytest.mark.parametrize("mode", ["exact_fp32", "bf16x3"])
def test_hybrid_gpu_matches_reference(golden, report, mode, perturbed):
    """HybridMLP (C1, fp32) vs the reference model's velocity, loss and gradient
    norms (model_hybrid_c1.npz).  exact-fp32: v and the loss within 1e-5
    (north_star); bf16x3: v and the loss within 1e-4.  Gradient-norm bounds
    below (reductions that cancel).  `perturbed`:
    model_hybrid_c1_perturbed.npz, the zero-init parameters perturbed so that v
    depends on the PVConv pyramid (at the reference's init ContextNet.head_out
    is zero and v does not see it)."""
    from golden_util import perturb_zero_init_
    from pcfm.models import HybridMLP
    from pcfm.precision import exact_fp32
    g = golden("model_hybrid_c1_perturbed.npz" if perturbed else "model_hybrid_c1.npz")
    torch.manual_seed(int(g["seed"]))
    pf = HybridMLP(cond_dim=129, point_dim=6)
    if perturbed:
        perturb_zero_init_(pf, int(g["perturb_seed"]))
    # same seed -> same weights (float64 sums: summation order may differ per host CPU)
    np.testing.assert_allclose(_param_sums(pf), g["param_sums"], rtol=1e-12, atol=1e-12)
    pf = pf.to(DEV).train()
    x = torch.from_numpy(g["x"]).to(DEV)
    with exact_fp32(mode == "exact_fp32"):
        v = pf(x, torch.from_numpy(g["t"]).to(DEV), torch.from_numpy(g["cond"]).to(DEV),
               cond_drop_mask=torch.from_numpy(g["mask"]).to(DEV))
        loss = torch.nn.functional.mse_loss(v, torch.from_numpy(g["target"]).to(DEV))
        loss.backward()
    e_v = _rel_max(v.detach().cpu().numpy(), g["v"])
    e_loss = abs(loss.item() - float(g["loss"])) / abs(float(g["loss"]))
    names = [n for n, _ in pf.named_parameters()]
    norms = np.array([p.grad.double().norm().item() if p.grad is not None else 0.0
                      for p in pf.parameters()])
    live = np.array([not n.endswith(_NOISE_BIAS) for n in names])
    # Gradient norms are reductions over 2k-160k terms that cancel (BatchNorm
    # biases: sums of dy; SE3d's MLP weights: ds = sum_v grid * g over R^3
    # voxels), so summation order alone moves them by far more than the forward
    # -- measured on MI355X, exact-fp32: 3.6e-4 (BN biases), 4.6e-4 (SE);
    # bf16x3: 4.1e-3, 1.1e-2.  Bounds: 1e-3 / 2e-3 exact, 1e-2 / 3e-2 bf16x3.
    se = np.array(["voxel_layers.6.fc." in n for n in names])
    gdev = np.abs(norms - g["grad_norms"]) / np.maximum(g["grad_norms"], 1e-30)
    e_g = float(gdev[live & ~se].max())
    e_se = float(gdev[live & se].max())
    worst = [names[i] for i in np.argsort(-np.where(live, gdev, 0))[:3]]
    rep = {"v": e_v, "loss": e_loss, "grad_norms": e_g, "grad_norms_se": e_se, "worst": worst}
    if perturbed:
        # elementwise at 64 seeded positions per parameter, normalised by the
        # parameter's max |gradient| (model_hybrid_c1_perturbed_grads.npz).  The
        # ContextNet's backward is itself this sensitive: on the CPU path alone, rgb
        # inputs moved by 1e-6 relative (coordinates untouched) move the gradients
        # at the stage outputs by 7.5e-4 (stage 2) to 1.5e-2 (stage 0) -- ReLU
        # masks that flip (profiles/r05_grad_sensitivity.json, tools/
        # grad_localize.py MODE=sensitivity) -- while the GPU forward differs
        # from the reference by ~1e-6 (v).  So the bounds are on the
        # distribution: median, 99th percentile and max over the 10.9 k sampled
        # elements.  Measured on MI355X (profiles/r05_hybrid_grads_elementwise.json):
        # exact fp32 2.5e-5 / 1.2e-3 / 1.2e-2, bf16x3 3.3e-4 / 2.0e-2 / 7.3e-2.
        # The PVConv block test above holds every gradient element to 1e-5 / 1e-4.
        from golden_util import grad_errors_sampled
        from golden_util import worst as worst_of
        per, el = grad_errors_sampled(pf, golden("model_hybrid_c1_perturbed_grads.npz"),
                                      elements=True)
        e_el, w_el = worst_of(per)
        rep.update(grads_elementwise=e_el, grads_elementwise_worst=w_el,
                   grads_elementwise_quantiles={q: float(np.quantile(el, q))
                                                for q in (0.5, 0.9, 0.99, 0.999)},
                   grads_elementwise_over_1e4=int((el > 1e-4).sum()), grads_sampled=int(el.size),
                   grads_elementwise_top={k: v for k, v in sorted(
                       per.items(), key=lambda kv: -kv[1]) if not k.endswith(_NOISE_BIAS)})
    report(f"hybrid_c1{'_perturbed' if perturbed else ''}_{mode}", rep)
    if perturbed:
        q = rep["grads_elementwise_quantiles"]
        med, p99, mx = (1e-4, 5e-3, 5e-2) if mode == "exact_fp32" else (1e-3, 5e-2, 2e-1)
        assert q[0.5] < med and q[0.99] < p99 and e_el < mx, (q, e_el, w_el)
        # per parameter where the ReLU-mask sensitivity does not reach: the head
        # (measured <= 1.9e-6 in both modes, profiles/r05_hybrid_grads_elementwise.json)
        # and the ContextNet parameters outside its PVConv stages (<= 1.5e-4 exact,
        # 2.5e-3 bf16x3) -- a wrong gradient confined to a few of them fails here
        head = {k: v for k, v in per.items() if k.startswith("head.")}
        rest = {k: v for k, v in per.items() if k.startswith("ctx_net.")
                and ".stages." not in k and not k.endswith(_NOISE_BIAS)}
        assert len(head) > 30 and len(rest) > 8, (len(head), len(rest))
        assert max(head.values()) < 1e-4, sorted(head.items(), key=lambda kv: -kv[1])[:3]
        bound = 1e-3 if mode == "exact_fp32" else 1e-2
        assert max(rest.values()) < bound, sorted(rest.items(), key=lambda kv: -kv[1])[:3]
    if mode == "exact_fp32":
        assert e_v < 1e-5 and e_loss < 1e-5 and e_g < 1e-3 and e_se < 2e-3, (e_v, e_loss, e_g,
                                                                             e_se, worst)
    else:
        # bf16x3 products (~2^-16 each): v / loss measured 2.4e-6 / 2.6e-6 on
        # MI355X, held to north_star's 1e-5
        assert e_v < 1e-5 and e_loss < 1e-5 and e_g < 1e-2 and e_se < 3e-2, (e_v, e_loss, e_g,
                                                                             e_se, worst)


def test_train_step_gpu_small():
    from pcfm.train import TrainConfig, Trainer, synthetic_batch
    cfg = TrainConfig(batch_size=2, num_points=2048, steps_per_epoch=10, epochs=2)
    tr = Trainer(cfg, DEV)
    tr.train_mode()
    batch = synthetic_batch(cfg, DEV)
    for ep in (1, 201):
        out = tr.step(batch, epoch=ep)
        assert math.isfinite(out["loss_point"].item()) and math.isfinite(out["loss_latent"].item())
