"""Train-step plumbing on the CPU (config C1: B=2, N=1024, xyz+rgb, hybrid) on the
product's pure-PyTorch CPU backend (no oracle involved)."""
import math

import torch

from pcfm.train import EMA, TrainConfig, Trainer, cosine_lr, synthetic_batch


def small_cfg(**kw):
    base = dict(batch_size=2, num_points=1024, ctx_stage_channels=[32, 64, 64],
                ctx_stage_res=[8, 4, 4], pf_width=64, lf_width=64, enc_width=32, latent_dim=16,
                steps_per_epoch=10, epochs=2)
    base.update(kw)
    return TrainConfig(**base)


def test_train_step_c1_full_size_model():
    """C1 with the default (full-width) hybrid model: one step, finite losses."""
    torch.manual_seed(0)
    cfg = TrainConfig(batch_size=2, num_points=1024, steps_per_epoch=1, epochs=1)
    tr = Trainer(cfg, "cpu")
    tr.train_mode()
    out = tr.step(synthetic_batch(cfg, "cpu"), epoch=201)
    assert math.isfinite(out["loss_point"].item()) and math.isfinite(out["loss_latent"].item())


def test_train_steps_reduce_loss():
    cfg = small_cfg(lr_pf=1e-3, lr_enc=1e-3, lr_lf=1e-3, warmup_steps=0, use_cosine_lr=False)
    tr = Trainer(cfg, "cpu")
    tr.train_mode()
    g = torch.Generator().manual_seed(1)
    batch = synthetic_batch(cfg, "cpu", generator=g)
    losses = [tr.step(batch, epoch=1)["loss_latent"].item() for _ in range(8)]
    assert losses[-1] < losses[0]


def test_warmup_epoch_uses_geometry_only():
    cfg = small_cfg()
    tr = Trainer(cfg, "cpu")
    tr.train_mode()
    out = tr.step(synthetic_batch(cfg, "cpu"), epoch=1)  # ep <= geom_warmup_epochs
    assert out["loss_point"].ndim == 0


def test_ema_foreach_equals_loop():
    m = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.BatchNorm1d(4))
    a, b = EMA(m, 0.9, foreach=True), EMA(m, 0.9, foreach=False)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(1.0)
    a.update(m)
    b.update(m)
    for k in a.shadow:
        assert torch.equal(a.shadow[k], b.shadow[k])


def test_cosine_lr_schedule():
    assert cosine_lr(0, 100, 1.0, 0.0, 10) == 0.0
    assert abs(cosine_lr(10, 100, 1.0, 0.0, 10) - 1.0) < 1e-12
    assert abs(cosine_lr(100, 100, 1.0, 0.0, 10)) < 1e-12
