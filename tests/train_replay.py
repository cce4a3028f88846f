"""Replay the reference's recorded train steps (tests/golden/train_step_c1.npz,
made by tests/golden/make_train_golden.py from /root/reference/train.py:553-673)
through this build's Trainer.step with the same batches and random draws, and
measure how far every recorded quantity lands from the reference's.

Used by tests/test_train_golden.py (CPU, the product's pure-PyTorch backend)
and tests/test_gpu_train_golden.py (MI355X, the HIP kernels).
"""
from __future__ import annotations

import contextlib
import re

import numpy as np
import torch

from pcfm.train import TrainConfig, Trainer

LR = 3e-4
# biases of the convolutions that feed a BatchNorm (SharedMLP layers.0, PVConv
# voxel_layers.0 / .3): their gradient is analytically zero (the BN removes any
# per-channel shift), so what autograd returns is rounding noise
_NOISE = re.compile(r"(layers\.0|voxel_layers\.[03])\.bias$")


def golden_config(**kw) -> TrainConfig:
    """The TrainConfig equal to make_train_golden.ARGS (+ argparse defaults)."""
    base = dict(batch_size=2, num_points=1024, cond_dim=1, latent_dim=128, epochs=1,
                steps_per_epoch=2, geom_warmup_epochs=0, color_prior="uniform",
                cfg_drop_p=0.5, cfg_drop_warmup_epochs=1, seed=123, tunableop=False,
                miopen_find=False)
    base.update(kw)
    return TrainConfig(**base)


@contextlib.contextmanager
def _record_update(tr, store):
    """Record, around Trainer._update_params, the per-parameter norms of the
    unscaled gradients (what clip_grad_norm_ sees) and the total norm it returns."""
    orig = tr._update_params
    params = _params(tr)

    def update():
        inv = 1.0 / tr.scaler.get_scale() if tr.scaler.is_enabled() else 1.0
        store["grad_norms"] = np.array([p.grad.double().norm().item() * inv
                                        if p.grad is not None else 0.0 for p in params])
        orig()
        store["total_norm"] = float(tr.last_grad_norm)
    tr._update_params = update
    try:
        yield
    finally:
        del tr._update_params


def _params(tr):
    return list(tr.enc.parameters()) + list(tr.pf.parameters()) + list(tr.lf.parameters())


def _names(tr):
    return ([f"enc.{n}" for n, _ in tr.enc.named_parameters()]
            + [f"pf.{n}" for n, _ in tr.pf.named_parameters()]
            + [f"lf.{n}" for n, _ in tr.lf.named_parameters()])


def _ema(tr):
    """(names, sums, numels) of the floating EMA shadows, pf then lf (the
    reference's order)."""
    names, sums, numel = [], [], []
    for tag, sh in (("pf", tr.ema_pf.shadow), ("lf", tr.ema_lf.shadow)):
        for k, t in sh.items():
            if t.dtype.is_floating_point:
                names.append(f"{tag}.{k}")
                sums.append(t.double().sum().item())
                numel.append(t.numel())
    return names, np.array(sums), np.array(numel)


def _rel(a, b):
    return float(abs(a - b) / max(abs(b), 1e-30))


def replay(g, device, n_steps=None, **cfg_kw):
    """Run the recorded steps; return a list (one dict per step) of deviations:
      loss_point / loss_latent / total_norm: relative error;
      v: max |v - v_ref| / max |v_ref|;
      grad_norm: max relative error of the per-parameter gradient norms over the
        parameters whose gradient is not rounding noise (_NOISE: conv biases in
        front of a BatchNorm have analytic gradient 0);
      update: max over parameters of |d_sum - d_sum_ref| / (lr * numel), d_sum the
        change of the parameter's sum in the AdamW step (0 = identical update;
        AdamW's first steps move every element by ~lr, so 1 means the sums
        differ by one full step of every element), same noise exclusion;
      ema: max |sum - sum_ref| of the EMA shadows in units of one EMA-weighted
        first step, (1 - decay) * lr * numel, over the non-noise parameters
        (BatchNorm running statistics, which inherit the noise biases' steps,
        and the noise biases themselves excluded).
    Also "init": max relative error of the initial parameter sums (same seed ->
    same weights).  Returns (init, steps, trainer)."""
    cfg = golden_config(**cfg_kw)
    tr = Trainer(cfg, device)
    tr.train_mode()
    params = _params(tr)
    names = _names(tr)
    numel = g["s0_numel"]
    assert [p.numel() for p in params] == list(numel)
    init = np.array([p.detach().double().sum().item() for p in params])
    out = []
    init_dev = float(np.max(np.abs(init - g["s0_pre_param_sums"]) /
                            np.maximum(np.abs(g["s0_pre_param_sums"]), 1e-12)))
    captured = {}
    hook = tr.pf.register_forward_hook(lambda m, i, o: captured.__setitem__("v", o.detach()))
    steps = int(g["n_steps"]) if n_steps is None else n_steps
    for i in range(steps):
        p = f"s{i}_"
        batch = {"train_points": torch.from_numpy(g[p + "train_points"]),
                 "train_rgb": torch.from_numpy(g[p + "train_rgb"]),
                 "cond": torch.from_numpy(g[p + "cond"])}
        draws = {k: torch.from_numpy(g[p + k]) for k in ("z_pts", "t_pts", "drop_u", "eps_z",
                                                         "t_z")}
        pre = np.array([q.detach().double().sum().item() for q in params])
        rec = {}
        with _record_update(tr, rec):
            losses = tr.step(batch, epoch=1, draws=draws)
        post = np.array([q.detach().double().sum().item() for q in params])
        mse = g[p + "mse"]
        lp_ref = float(np.float32(mse[0]) + np.float32(mse[1]))  # lambda_color = 1
        v = captured["v"].float().cpu().numpy()
        v_ref = g[p + "v"]
        gn_ref = g[p + "grad_norms"]
        live = np.array([not _NOISE.search(nm) for nm in names])
        gn_dev = np.abs(rec["grad_norms"] - gn_ref) / np.maximum(gn_ref, 1e-30)
        step_lr = float(g[p + "lrs"][0])  # the lr AdamW.step used (recorded inside it)
        d_got = post - pre
        d_ref = g[p + "post_param_sums"] - g[p + "pre_param_sums"]
        upd = np.abs(d_got - d_ref) / (step_lr * numel)
        ema_ref = np.concatenate([g[p + "ema_pf"], g[p + "ema_lf"]])
        ema_names, ema_got, ema_numel = _ema(tr)
        ema_live = np.array([not (_NOISE.search(nm) or "running_" in nm) for nm in ema_names])
        ema_dev = np.abs(ema_got - ema_ref) / ((1.0 - tr.cfg.ema_decay) * LR * ema_numel)
        out.append({
            "loss_point": _rel(float(losses["loss_point"]), lp_ref),
            "loss_latent": _rel(float(losses["loss_latent"]), float(mse[2])),
            "total_norm": _rel(rec["total_norm"], float(g[p + "total_norm"])),
            "v": float(np.abs(v - v_ref).max() / np.abs(v_ref).max()),
            "grad_norm": float(gn_dev[live].max()),
            "update": float(upd[live].max()),
            "update_noise": float(upd[~live].max()) if (~live).any() else 0.0,
            "ema": float(ema_dev[ema_live].max()),
            "worst_grad": names[int(np.argmax(np.where(live, gn_dev, 0)))],
            "worst_ema": ema_names[int(np.argmax(np.where(ema_live, ema_dev, 0)))],
        })
    hook.remove()
    return init_dev, out, tr


def replay_sampling(g, tr, amp: bool = False):
    """The reference's post-epoch Heun sampling (train.py:282-429, EMA weights,
    --sample_steps 2) through pcfm.sample.heun on the Trainer after replay():
    same prior draws, same conditions.  Returns max-abs relative deviations of
    every velocity evaluation ("recon_v", "samples_lf_v", "samples_v"), of the
    final clouds ("recon_xyz", "samples_xyz") and of the latent z ("samples_z")."""
    from pcfm.sample import heun
    dev = tr.device
    tr.ema_pf.copy_to(tr.pf)
    tr.ema_lf.copy_to(tr.lf)
    tr.pf.eval()
    tr.lf.eval()
    steps = g["recon_pf_t"].shape[0] // 2

    def rel(a, b):
        return float(np.abs(a - b).max() / np.abs(b).max())

    def run_pf(x0, cond, vs):
        def vel(x, t):
            v = tr.pf.guided_velocity(x, t, cond, guidance_scale=0.0)
            vs.append(v.float().cpu().numpy())
            return v
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            return heun(vel, x0, steps)

    out = {}
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    vs = []
    x = run_pf(t(g["recon_x0"]), t(g["recon_cond"]), vs)
    out["recon_v"] = max(rel(a, b) for a, b in zip(vs, g["recon_pf_v"]))
    out["recon_xyz"] = rel(x[..., :3].float().cpu().numpy(), g["recon_final_xyz"])
    lvs = []

    def lvel(y, tt):
        v = tr.lf(y, tt, cond=None)
        lvs.append(v.float().cpu().numpy())
        return v
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        z = heun(lvel, t(g["samples_z0"]), steps)
    latent = g["samples_z0"].shape[1]
    out["samples_lf_v"] = max(rel(a, b) for a, b in zip(lvs, g["samples_lf_v"]))
    out["samples_z"] = rel(z.float().cpu().numpy(), g["samples_cond"][:, :latent])
    vs = []
    x = run_pf(t(g["samples_x0"]), t(g["samples_cond"]), vs)
    out["samples_v"] = max(rel(a, b) for a, b in zip(vs, g["samples_pf_v"]))
    out["samples_xyz"] = rel(x[..., :3].float().cpu().numpy(), g["samples_final_xyz"])
    return out


def replay_dopri5(gd, g, tr, names=("hybrid_c1_3", "hybrid_c1_5")):
    """The golden's dopri5 cases of the C1 hybrid flow (tests/golden/
    dopri5_torchdiffeq.npz, made by the reference's vendored torchdiffeq 0.2.2)
    through pcfm.sample.dopri5 on the Trainer after replay() + replay_sampling()
    (EMA weights, eval mode).  Returns {case: {nfe, nfe_ref, times (max abs
    difference of the evaluation times, when the counts agree), y1 (max |dy| /
    max |y_ref|)}}."""
    from pcfm.sample import dopri5
    dev = tr.device
    cond = torch.from_numpy(g["recon_cond"]).to(dev)
    out = {}
    for name in names:
        rtol, atol = (float(v) for v in gd[f"{name}_tol"])
        times = []
        y1, nfe = dopri5(lambda x, t: tr.pf.guided_velocity(x, t, cond),
                         torch.from_numpy(gd[f"{name}_y0"]).to(dev), rtol=rtol, atol=atol,
                         trace=times)
        ref = gd[f"{name}_y1"]
        t_ref = gd[f"{name}_times"]
        out[name] = {"nfe": nfe, "nfe_ref": int(gd[f"{name}_nfe"]),
                     "times": float(np.abs(np.array(times) - t_ref).max())
                     if len(times) == len(t_ref) else None,
                     "y1": float(np.abs(y1.float().cpu().numpy() - ref).max()
                                 / np.abs(ref).max())}
    return out
