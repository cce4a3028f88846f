"""GPU: the fused parameter update (pcfm.optim.FusedAdamWEMA, csrc/optim.hip)
against the reference's own sequence on the same tensors: GradScaler unscale,
clip_grad_norm_, torch.optim.AdamW (foreach, the reference's default,
train.py:249-253) and util.EMA's mul_/add_ (util.py:17-21)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
SHAPES = [(256, 128, 3, 3, 3), (7,), (3,), (513, 9), (4096,), (4097,), (64, 64), (1,)]


def _setup(seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    ps = [torch.randn(s, device=DEV, generator=g) * 0.1 for s in SHAPES]
    shadows = [p.clone() + 0.01 for p in ps]
    return g, ps, shadows


def _reference_step(ps, grads, shadows, opt, scale, max_norm, decay, ema_mask):
    for p, gr in zip(ps, grads):
        p.grad = None if gr is None else gr.clone()
    live = [p for p in ps if p.grad is not None]
    inv = 1.0 / scale  # a power of two, as GradScaler's scales are
    found = any(not torch.isfinite(p.grad).all() for p in live)
    torch._foreach_mul_([p.grad for p in live], inv)
    # the Trainer clips only for grad_clip_norm > 0 (train.py:653-656)
    total = torch.nn.utils.clip_grad_norm_(live, max_norm) if max_norm > 0 else 0.0
    if not found:
        opt.step()
    with torch.no_grad():
        for p, s, on in zip(ps, shadows, ema_mask):
            if on:
                s.mul_(decay).add_(p, alpha=1.0 - decay)
    return float(total), found


class _Scaler:
    """The GradScaler attributes FusedAdamWEMA.step reads and updates."""

    def __init__(self, scale):
        self._scale = torch.full((1,), float(scale), device=DEV)
        self._growth_tracker = torch.zeros(1, dtype=torch.int32, device=DEV)
        self._growth_factor, self._backoff_factor, self._growth_interval = 2.0, 0.5, 2000

    def is_enabled(self):
        return True


@pytest.mark.parametrize("max_norm", [1.0, 1e4, 0.0])
def test_fused_adamw_ema_matches_torch(max_norm):
    from pcfm.optim import FusedAdamWEMA
    g, ps, shadows = _setup(1)
    ref_ps = [p.clone() for p in ps]
    ref_sh = [s.clone() for s in shadows]
    lrs, wd, decay = (3e-4, 1e-3, 5e-4), 1e-4, 0.999
    split = [slice(0, 3), slice(3, 6), slice(6, len(ps))]
    ema_mask = [i % 3 != 1 for i in range(len(ps))]
    fused = FusedAdamWEMA(
        [{"params": ps[s], "lr": lr, "weight_decay": wd} for s, lr in zip(split, lrs)],
        ema_shadows={p: sh for p, sh, on in zip(ps, shadows, ema_mask) if on},
        ema_decay=decay)
    ref_opt = torch.optim.AdamW([{"params": ref_ps[s], "lr": lr} for s, lr in zip(split, lrs)],
                                weight_decay=wd, foreach=True)
    scale = 2.0 ** 10
    scaler = _Scaler(scale)
    for step in range(4):
        grads = [torch.randn(p.shape, device=DEV, generator=g) * scale * 0.05 for p in ps]
        grads[5] = None if step == 2 else grads[5]  # a parameter without gradient
        for p, gr in zip(ps, grads):
            p.grad = gr
        # the cosine schedule rewrites the group lrs between steps
        for grp, rgrp in zip(fused.param_groups, ref_opt.param_groups):
            grp["lr"] = rgrp["lr"] = grp["lr"] * 0.9
        norm = fused.step(max_norm, scaler)
        tot, _ = _reference_step(ref_ps, grads, ref_sh, ref_opt, scale, max_norm, decay, ema_mask)
        if max_norm > 0:
            assert abs(float(norm) - tot) <= 1e-5 * tot
        for a, b in zip(ps, ref_ps):
            torch.testing.assert_close(a, b, rtol=2e-6, atol=1e-8)
        for a, b in zip(shadows, ref_sh):
            torch.testing.assert_close(a, b, rtol=2e-6, atol=1e-8)
        for a, b in zip(ps, ref_ps):  # keep the two on identical values
            a.copy_(b)
        for a, b in zip(shadows, ref_sh):
            a.copy_(b)
    steps = fused.steps.cpu().tolist()
    assert steps[5] == 3.0 and all(v == 4.0 for i, v in enumerate(steps) if i != 5)
    assert float(scaler._scale) == scale  # no inf: no backoff (growth after 2000)


def test_fused_adamw_skips_on_inf_and_backs_off():
    from pcfm.optim import FusedAdamWEMA
    g, ps, shadows = _setup(2)
    fused = FusedAdamWEMA([{"params": ps, "lr": 1e-3, "weight_decay": 1e-4}],
                          ema_shadows=dict(zip(ps, shadows)), ema_decay=0.9)
    scaler = _Scaler(2.0 ** 16)
    before = [p.clone() for p in ps]
    sh_before = [s.clone() for s in shadows]
    for p in ps:
        p.grad = torch.randn(p.shape, device=DEV, generator=g)
    ps[3].grad[0, 0] = float("inf")
    fused.step(1.0, scaler)
    for a, b in zip(ps, before):
        assert torch.equal(a, b)  # update skipped
    for s, s0, p in zip(shadows, sh_before, before):  # the EMA still moves
        torch.testing.assert_close(s, s0 * 0.9 + 0.1 * p, rtol=1e-6, atol=1e-7)
    assert float(fused.steps.max()) == 0.0 and float(fused.found_inf) == 1.0
    assert float(scaler._scale) == 2.0 ** 15
    for p in ps:
        p.grad = torch.randn(p.shape, device=DEV, generator=g)
    fused.step(1.0, scaler)
    assert float(fused.steps.min()) == 1.0 and float(fused.found_inf) == 0.0
    assert not all(torch.equal(a, b) for a, b in zip(ps, before))


def test_trainer_fused_step_matches_torch_path():
    """Two Trainer steps at a small config: fused update vs torch AdamW + clip +
    foreach EMA from the same initial state and batch."""
    from pcfm.train import TrainConfig, Trainer, synthetic_batch
    cfg = dict(batch_size=2, num_points=1024, steps_per_epoch=4, epochs=1, tunableop=False,
               miopen_find=False, device_rng=False)
    out = {}
    lr_max = 0.0
    for fused in (True, False):
        tr = Trainer(TrainConfig(fused_step=fused, **cfg), DEV)
        lr_max = max([lr_max] + [float(gr["lr"]) for gr in tr.opt.param_groups])
        tr.train_mode()
        batch = synthetic_batch(tr.cfg, DEV, generator=torch.Generator(device=DEV).manual_seed(3))
        torch.manual_seed(5)
        for _ in range(2):
            tr.step(batch, epoch=201)
        out[fused] = ([p.detach().double().sum().item() for p in tr._clip_params],
                      [v.double().sum().item() for v in tr.ema_pf.shadow.values()
                       if v.dtype.is_floating_point], float(tr.last_grad_norm))
    pf, ef, nf = out[True]
    pt, et, nt = out[False]
    # identical forward/backward (same seeds, deterministic kernels); the updates
    # differ only in rounding -- except where AdamW's m / (sqrt(v) + eps) is
    # rounding-sensitive: an element whose gradient is ~eps can take a different
    # full-size step (up to lr each), so a parameter's sum may differ by a few
    # lr over the two steps (measured: 2.0e-4 with the per-cloud layers in bf16,
    # 4.2e-4 in fp32, lr 3e-4) besides the relative rounding term
    assert abs(nf - nt) <= 1e-4 * nt
    d = np.abs(np.array(pf) - np.array(pt))
    bound = max(1e-3 * 3e-4 * 2 * max(1.0, np.abs(pt).max()), 2 * 2 * lr_max)
    assert d.max() <= bound, (d.max(), bound)
    np.testing.assert_allclose(ef, et, rtol=1e-6, atol=1e-6)


def test_fused_adamw_without_scaler_steps_through_nan():
    """amp off (no GradScaler): torch's clip_grad_norm_ + AdamW step anyway and
    the NaN reaches the parameters; the fused update must not skip."""
    from pcfm.optim import FusedAdamWEMA
    g, ps, shadows = _setup(4)
    ref_ps = [p.clone() for p in ps]
    fused = FusedAdamWEMA([{"params": ps, "lr": 1e-3, "weight_decay": 1e-4}])
    ref_opt = torch.optim.AdamW([{"params": ref_ps, "lr": 1e-3}], weight_decay=1e-4,
                                foreach=True)
    grads = [torch.randn(p.shape, device=DEV, generator=g) for p in ps]
    grads[2][1] = float("nan")
    for p, gr in zip(ps, grads):
        p.grad = gr.clone()
    fused.step(1.0, None)
    for p, gr in zip(ref_ps, grads):
        p.grad = gr.clone()
    torch.nn.utils.clip_grad_norm_(ref_ps, 1.0)
    ref_opt.step()
    for a, b in zip(ps, ref_ps):
        assert torch.equal(torch.isnan(a), torch.isnan(b))
    assert all(torch.isnan(p).all() for p in ps)  # the NaN norm scales every gradient
    assert float(fused.steps.min()) == 1.0 and float(fused.found_inf) == 0.0


def test_fused_adamw_state_dict_round_trips_with_torch():
    """state_dict / load_state_dict in torch.optim.AdamW's layout (the reference
    checkpoints opt.state_dict(), train.py:501, :701): torch -> fused and
    fused -> torch, then one more step on both must agree."""
    from pcfm.optim import FusedAdamWEMA
    g, ps, _ = _setup(5)
    split = [slice(0, 4), slice(4, len(ps))]
    lrs, wd = (3e-4, 1e-3), 1e-4
    ref_ps = [p.clone() for p in ps]
    ref_opt = torch.optim.AdamW([{"params": ref_ps[s], "lr": lr} for s, lr in zip(split, lrs)],
                                weight_decay=wd, foreach=True)
    for step in range(2):
        for p in ref_ps:
            p.grad = None if (step == 1 and p is ref_ps[6]) else torch.randn(
                p.shape, device=DEV, generator=g)
        ref_opt.step()
    fused = FusedAdamWEMA([{"params": ps[s], "lr": 0.5, "weight_decay": 0.5} for s in split])
    with torch.no_grad():
        for a, b in zip(ps, ref_ps):
            a.copy_(b)
    fused.load_state_dict(ref_opt.state_dict())
    assert [g_["lr"] for g_ in fused.param_groups] == list(lrs)
    sd = fused.state_dict()
    for k, st in ref_opt.state_dict()["state"].items():
        assert float(sd["state"][k]["step"]) == float(st["step"])
        assert torch.equal(sd["state"][k]["exp_avg"], st["exp_avg"])
        assert torch.equal(sd["state"][k]["exp_avg_sq"], st["exp_avg_sq"])
    grads = [torch.randn(p.shape, device=DEV, generator=g) for p in ps]
    for a, b, gr in zip(ps, ref_ps, grads):
        a.grad, b.grad = gr.clone(), gr.clone()
    fused.step(0.0, None)
    ref_opt.step()
    for a, b in zip(ps, ref_ps):
        torch.testing.assert_close(a, b, rtol=2e-6, atol=1e-8)
    # fused -> a fresh torch AdamW
    ref2 = [p.detach().clone() for p in ps]
    opt2 = torch.optim.AdamW([{"params": ref2[s], "lr": 9.0} for s in split], weight_decay=wd,
                             foreach=True)
    opt2.load_state_dict(fused.state_dict())
    for a, b in zip(ps, ref2):
        gr = torch.randn(a.shape, device=DEV, generator=g)
        a.grad, b.grad = gr.clone(), gr.clone()
    fused.step(0.0, None)
    opt2.step()
    for a, b in zip(ps, ref2):
        torch.testing.assert_close(a, b, rtol=2e-6, atol=1e-8)


def test_trainer_fused_first_step_elementwise():
    """One Trainer step, fused vs torch path, compared element by element
    (ADVICE r2): the moments at 1e-5, and the parameters within 1e-6 relative +
    1e-3 lr except where the unscaled, clipped gradient is below 1e-6 -- there
    AdamW's first step m / (sqrt(v) + eps) = g / (|g| + eps) depends on eps and
    on the gradient's last bits, so the step itself (up to lr) is rounding."""
    from pcfm.train import TrainConfig, Trainer, synthetic_batch
    cfg = dict(batch_size=2, num_points=1024, steps_per_epoch=4, epochs=1, tunableop=False,
               miopen_find=False, device_rng=False)
    res = {}
    for fused in (True, False):
        tr = Trainer(TrainConfig(fused_step=fused, **cfg), DEV)
        tr.train_mode()
        batch = synthetic_batch(tr.cfg, DEV, generator=torch.Generator(device=DEV).manual_seed(3))
        torch.manual_seed(5)
        p0 = [p.detach().clone() for p in tr._clip_params]
        tr.forward_backward(batch, epoch=201)
        inv = 1.0 / tr.scaler.get_scale()
        gr = [None if p.grad is None else p.grad.detach().clone() * inv for p in tr._clip_params]
        tr._update_params()
        sd = tr.opt.state_dict()["state"]
        res[fused] = (p0, gr, [p.detach().clone() for p in tr._clip_params], sd,
                      float(tr.last_grad_norm))
    p0f, gf, pf, sdf, nf = res[True]
    p0t, gt, pt, sdt, nt = res[False]
    assert all(torch.equal(a, b) for a, b in zip(p0f, p0t))
    assert abs(nf - nt) <= 1e-5 * nt
    coef = min(1.0, 1.0 / (nt + 1e-6))
    lr = 3e-4  # the groups' initial lr (the schedule is applied after the step)
    for i, (g1, g2) in enumerate(zip(gf, gt)):
        if g1 is None:
            assert g2 is None and i not in sdf and i not in sdt
            continue
        torch.testing.assert_close(g1, g2, rtol=0, atol=0)  # same forward / backward bits
        torch.testing.assert_close(sdf[i]["exp_avg"], sdt[i]["exp_avg"], rtol=1e-5, atol=1e-12)
        torch.testing.assert_close(sdf[i]["exp_avg_sq"], sdt[i]["exp_avg_sq"], rtol=1e-5,
                                   atol=1e-18)
        live = (g1 * coef).abs() >= 1e-6
        d = (pf[i] - pt[i]).abs()
        bound = 1e-6 * pt[i].abs() + 1e-3 * lr
        assert bool((d[live] <= bound[live]).all()), (i, float(d[live].max()))
