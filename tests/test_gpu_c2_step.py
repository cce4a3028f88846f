"""GPU: one train step at the headline configuration (BASELINE.json configs[1],
SURVEY.md C2: hybrid backbone, B=8, N=20000, xyz+rgb) in the production
arithmetic -- the ContextNet's Conv3d / 1x1 convolutions as bf16x3 matrix-core
products (modules/voxel_conv.py, modules/shared_mlp.py) -- against the same
step with exact fp32 convolutions (MIOpen / hipBLASLt fp32, pcfm.precision),
on the same weights, batch and random draws (reference step: train.py:553-673).

Every zero-initialised parameter is perturbed first (tests/golden_util.py), so
the velocity depends on the whole PVConv pyramid: at the reference's
initialisation ContextNet.head_out is zero and v would not see the voxel path.

  * amp off (fp32 head): the context ctx, the velocity v and both losses
    within 1e-4 (max-norm relative).
  * amp on (the reference's GPU training config: bf16 autocast on the head):
    ctx -- the fp32 ContextNet's output -- within 1e-4; v and the losses go
    through the bf16 head, reported and held to 2e-2.
Measured values are reported (PCFM_REPORT -> profiles/r04_parity.json)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy()
    return float(np.abs(a - b).max() / np.abs(b).max())


@pytest.fixture(scope="module")
def c2_setup():
    from golden_util import perturb_zero_init_
    from pcfm.train import TrainConfig, Trainer, synthetic_batch
    dev = torch.device("cuda", 0)
    cfg = TrainConfig(batch_size=8, num_points=20000, tunableop=False, miopen_find=False)
    tr = Trainer(cfg, dev)
    tr.train_mode()
    perturb_zero_init_(tr.pf, seed=11)
    g = torch.Generator().manual_seed(1234)
    batch = {k: v.to(dev) for k, v in synthetic_batch(cfg, "cpu", generator=g).items()}
    b, n = cfg.batch_size, cfg.num_points
    beta = torch.distributions.Beta(torch.tensor(cfg.t_beta_a), torch.tensor(1.0))
    torch.manual_seed(77)
    draws = {"z_pts": torch.cat([torch.randn(b, n, 3, generator=g), torch.rand(b, n, 3, generator=g)],
                                -1),
             "t_pts": beta.sample((b,)), "drop_u": torch.rand(b, generator=g),
             "eps_z": torch.randn(b, cfg.latent_dim, generator=g), "t_z": beta.sample((b,))}
    return tr, batch, draws, cfg.geom_warmup_epochs + 1


def _one(tr, batch, draws, epoch, exact, amp):
    from pcfm.precision import exact_fp32
    seen = {}
    h1 = tr.pf.ctx_net.register_forward_hook(lambda m, i, o: seen.__setitem__("ctx", o.detach()))
    h2 = tr.pf.register_forward_hook(lambda m, i, o: seen.__setitem__("v", o.detach().float()))
    old_amp = tr.cfg.amp
    tr.cfg.amp = amp
    try:
        tr.opt.zero_grad(set_to_none=True)
        with exact_fp32(exact):
            out = tr.forward_backward(batch, epoch, draws)
        torch.cuda.synchronize()
    finally:
        tr.cfg.amp = old_amp
        h1.remove()
        h2.remove()
    tr.opt.zero_grad(set_to_none=True)
    return {"ctx": seen["ctx"], "v": seen["v"], "loss_point": out["loss_point"].float(),
            "loss_latent": out["loss_latent"].float()}


@pytest.mark.parametrize("amp", [False, True])
def test_c2_step_bf16x3_matches_exact_fp32(c2_setup, report, amp):
    tr, batch, draws, epoch = c2_setup
    ref = _one(tr, batch, draws, epoch, exact=True, amp=amp)
    got = _one(tr, batch, draws, epoch, exact=False, amp=amp)
    dev = {k: _rel(got[k], ref[k]) for k in ("ctx", "v", "loss_point", "loss_latent")}
    # the perturbed head_out makes v depend on ctx: a ctx of zeros would pass vacuously
    dev["ctx_rms"] = float(ref["ctx"].double().pow(2).mean().sqrt())
    report(f"c2_step_bf16x3_vs_exact_fp32_{'amp' if amp else 'fp32'}", dev)
    assert dev["ctx_rms"] > 1e-3, dev
    assert dev["ctx"] <= 1e-4, dev
    bound = 2e-2 if amp else 1e-4
    for k in ("v", "loss_point", "loss_latent"):
        assert dev[k] <= bound, (k, dev)
