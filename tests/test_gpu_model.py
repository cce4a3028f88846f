"""GPU: the drop-in modules and the flow model on the HIP path against the
reference-Python goldens, and the train step at small scale."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _fp32_exact():
    # cuDNN/MIOpen and hipBLASLt must not trade fp32 for a reduced format here
    old = (torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    yield
    torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = old


def _param_sums(module):
    return np.array([p.detach().double().sum().item() for _, p in module.named_parameters()])


def test_native_library_is_what_runs():
    import modules.functional.backend as be
    from pcfm import _lib, ops
    assert be._backend is ops.backend
    lib = _lib.load()
    assert lib._name.endswith("libpcfm_hip.so")


def test_pvconv_gpu_matches_reference(golden):
    from modules.pvconv import PVConv
    g = golden("pvconv_r8.npz")
    torch.manual_seed(int(g["seed"]))
    blk = PVConv(16, 16, kernel_size=3, resolution=8, with_se=True, normalize=True, eps=1e-6)
    np.testing.assert_allclose(_param_sums(blk), g["param_sums"], rtol=1e-12, atol=1e-12)
    blk = blk.to(DEV)
    feats = torch.from_numpy(g["feats"]).to(DEV).requires_grad_(True)
    out, _ = blk((feats, torch.from_numpy(g["coords"]).to(DEV)))
    np.testing.assert_allclose(out.detach().cpu().numpy(), g["out"], rtol=1e-4, atol=1e-5)
    loss = (out * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum()
    loss.backward()
    np.testing.assert_allclose(feats.grad.cpu().numpy(), g["grad_feats"], rtol=1e-3, atol=1e-4)


def test_hybrid_gpu_matches_reference(golden):
    from pcfm.models import HybridMLP
    g = golden("model_hybrid_c1.npz")
    torch.manual_seed(int(g["seed"]))
    pf = HybridMLP(cond_dim=129, point_dim=6)
    # same seed -> same weights (float64 sums: summation order may differ per host CPU)
    np.testing.assert_allclose(_param_sums(pf), g["param_sums"], rtol=1e-12, atol=1e-12)
    pf = pf.to(DEV).train()
    x = torch.from_numpy(g["x"]).to(DEV)
    v = pf(x, torch.from_numpy(g["t"]).to(DEV), torch.from_numpy(g["cond"]).to(DEV),
           cond_drop_mask=torch.from_numpy(g["mask"]).to(DEV))
    np.testing.assert_allclose(v.detach().cpu().numpy(), g["v"], rtol=1e-3, atol=1e-4)
    loss = torch.nn.functional.mse_loss(v, torch.from_numpy(g["target"]).to(DEV))
    np.testing.assert_allclose(loss.item(), float(g["loss"]), rtol=1e-4)
    loss.backward()
    norms = np.array([p.grad.double().norm().item() if p.grad is not None else 0.0
                      for p in pf.parameters()])
    # fp32 GPU convolutions vs CPU: gradients agree to ~1e-3 relative per tensor
    np.testing.assert_allclose(norms, g["grad_norms"], rtol=1e-2, atol=1e-5)


def test_train_step_gpu_small():
    from pcfm.train import TrainConfig, Trainer, synthetic_batch
    cfg = TrainConfig(batch_size=2, num_points=2048, steps_per_epoch=10, epochs=2)
    tr = Trainer(cfg, DEV)
    tr.train_mode()
    batch = synthetic_batch(cfg, DEV)
    for ep in (1, 201):
        out = tr.step(batch, epoch=ep)
        assert math.isfinite(out["loss_point"].item()) and math.isfinite(out["loss_latent"].item())
