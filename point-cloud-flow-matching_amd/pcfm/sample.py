"""Point-cloud generation and the Chamfer metric of the flow model (SURVEY.md
section 8 f3; BASELINE.json configs[3]).

* `heun` -- the reference's predictor-corrector loop (train.py:332-341, 385-415):
  t_k = k / steps, x <- x + dt/2 (v(x, t_k) + v(x + dt v(x, t_k), t_{k+1})).
* `dopri5` -- adaptive Dormand-Prince 5(4) with FSAL, the method the reference
  vendors (third_party/torchdiffeq, `odeint(..., method='dopri5')`) but never
  calls; restated here from the published tableau (Dormand & Prince 1980) with
  torchdiffeq's step control: RMS error norm over the whole state scaled by
  atol + rtol * max(|y0|, |y1|), safety 0.9, growth in [0.2, 10], and Hairer's
  initial step selection.  `fixed_steps=k` runs k equal steps instead.
* `generate` -- save_val_samples (train.py:361-429): latent flow (Heun) from
  N(0, latent_prior_std^2), cond = [z | joint cond], then the point flow from
  the xyz(+rgb) prior with Heun or dopri5, CFG through `guided_velocity`.
* `chamfer_l2` -- train.py:80-84 (mean squared nearest-neighbour distance both
  ways, per cloud) on the gfx950 Chamfer kernel for HIP tensors.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch

Velocity = Callable[[torch.Tensor, torch.Tensor], torch.Tensor]


def _tvec(x: torch.Tensor, t: float) -> torch.Tensor:
    return torch.full((x.shape[0],), t, device=x.device, dtype=x.dtype)


@torch.no_grad()
def heun(velocity: Velocity, x: torch.Tensor, steps: int) -> torch.Tensor:
    """The reference's Heun (RK2) integration from t = 0 to 1 (train.py:332-341)."""
    steps = max(1, int(steps))
    dt = 1.0 / steps
    for k in range(steps):
        v1 = velocity(x, _tvec(x, k * dt))
        x_hat = x + v1 * dt
        v2 = velocity(x_hat, _tvec(x, (k + 1) * dt))
        x = x + 0.5 * dt * (v1 + v2)
    return x


# Dormand-Prince 5(4) tableau
_C = (0.0, 1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0, 1.0)
_A = ((),
      (1 / 5,),
      (3 / 40, 9 / 40),
      (44 / 45, -56 / 15, 32 / 9),
      (19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729),
      (9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656),
      (35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84))
_B5 = (35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84, 0.0)
_B4 = (5179 / 57600, 0.0, 7571 / 16695, 393 / 640, -92097 / 339200, 187 / 2100, 1 / 40)


def _rms(x: torch.Tensor) -> float:
    return float(x.pow(2).mean().sqrt())


def _initial_step(f, t0, y0, f0, rtol, atol) -> float:
    """Hairer, Norsett & Wanner II.4 (torchdiffeq's _select_initial_step), order 5."""
    scale = atol + y0.abs() * rtol
    d0, d1 = _rms(y0 / scale), _rms(f0 / scale)
    h0 = 1e-6 if d0 < 1e-5 or d1 < 1e-5 else 0.01 * d0 / d1
    f1 = f(y0 + h0 * f0, t0 + h0)
    d2 = _rms((f1 - f0) / scale) / h0
    if d1 <= 1e-15 and d2 <= 1e-15:
        h1 = max(1e-6, h0 * 1e-3)
    else:
        h1 = (0.01 / max(d1, d2)) ** (1.0 / 5)
    return min(100 * h0, h1)


@torch.no_grad()
def dopri5(velocity: Velocity, x: torch.Tensor, t0: float = 0.0, t1: float = 1.0,
           rtol: float = 1e-5, atol: float = 1e-5, fixed_steps: Optional[int] = None,
           max_steps: int = 10000) -> Tuple[torch.Tensor, int]:
    """Integrate dx/dt = velocity(x, t) from t0 to t1; returns (x(t1), NFE)."""
    nfe = 0

    def f(y, t):
        nonlocal nfe
        nfe += 1
        return velocity(y, _tvec(y, t))

    t, y = float(t0), x
    k1 = f(y, t)
    if fixed_steps is not None:
        h = (t1 - t0) / max(1, int(fixed_steps))
    else:
        h = _initial_step(f, t, y, k1, rtol, atol)
    steps = 0
    while t1 - t > 1e-12 * max(1.0, abs(t1)) and steps < max_steps:
        h = min(h, t1 - t)
        ks = [k1]
        for i in range(1, 7):
            yi = y
            for j, a in enumerate(_A[i]):
                if a != 0.0:
                    yi = yi + (h * a) * ks[j]
            ks.append(f(yi, t + _C[i] * h))
        y_new = yi  # stage 7 input is the 5th-order solution (FSAL)
        steps += 1
        if fixed_steps is not None:
            t, y, k1 = t + h, y_new, ks[6]
            continue
        err = sum((h * (b5 - b4)) * k for b5, b4, k in zip(_B5, _B4, ks) if b5 != b4)
        scale = atol + rtol * torch.maximum(y.abs(), y_new.abs())
        e = _rms(err / scale)
        if e <= 1.0:
            t, y, k1 = t + h, y_new, ks[6]
        factor = 10.0 if e == 0.0 else min(10.0, max(0.2, 0.9 * e ** (-1.0 / 5)))
        h = h * factor
    return y, nfe


def pf_prior_like(data_pf: torch.Tensor, point_prior_std: float = 1.0,
                  color_prior: str = "uniform", color_prior_std: float = 1.0) -> torch.Tensor:
    """make_pf_prior_like (train.py:266-279)."""
    b, n, d = data_pf.shape
    if d == 3:
        return torch.randn_like(data_pf) * point_prior_std
    z = data_pf.new_empty(b, n, 6)
    z[..., :3] = torch.randn(b, n, 3, device=data_pf.device, dtype=data_pf.dtype) * point_prior_std
    if color_prior == "gauss":
        z[..., 3:] = torch.randn(b, n, 3, device=data_pf.device, dtype=data_pf.dtype) * color_prior_std
    elif color_prior == "uniform":
        z[..., 3:] = torch.rand(b, n, 3, device=data_pf.device, dtype=data_pf.dtype)
    else:
        z[..., 3:] = 0.0
    return z


@torch.no_grad()
def generate(pf, lf, batch_size: int, num_points: int, point_dim: int, latent_dim: int,
             cond: Optional[torch.Tensor] = None, cond_dim: int = 0, steps: int = 50,
             method: str = "heun", guidance_scale: float = 0.0, latent_prior_std: float = 1.0,
             point_prior_std: float = 1.0, color_prior: str = "uniform", rtol: float = 1e-5,
             atol: float = 1e-5, device=None, dtype=torch.float32) -> Tuple[torch.Tensor, int]:
    """Random-z generation as save_val_samples (train.py:361-429); returns
    (points (B, N, point_dim), point-flow NFE).  Models are used as given
    (call .eval() and swap in EMA weights first, as the reference does)."""
    dev = device if device is not None else next(pf.parameters()).device
    b = int(batch_size)
    z = torch.randn((b, latent_dim), device=dev, dtype=dtype) * latent_prior_std
    z = heun(lambda y, t: lf(y, t, cond=None), z, steps)
    if cond is not None:
        cond_full = torch.cat([z, cond.to(dev, dtype)], dim=1)
    elif cond_dim > 0:
        cond_full = torch.cat([z, torch.zeros((b, cond_dim), device=dev, dtype=dtype)], dim=1)
    else:
        cond_full = z
    x0 = pf_prior_like(torch.empty((b, num_points, point_dim), device=dev, dtype=dtype),
                       point_prior_std, color_prior)

    def vel(x, t):
        return pf.guided_velocity(x, t, cond_full, guidance_scale=guidance_scale)

    if method == "heun":
        return heun(vel, x0, steps), 2 * max(1, int(steps))
    if method == "dopri5":
        return dopri5(vel, x0, rtol=rtol, atol=atol)
    if method == "dopri5_fixed":
        return dopri5(vel, x0, fixed_steps=steps)
    raise ValueError(f"unknown method {method!r}")


@torch.no_grad()
def chamfer_l2(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Per-cloud mean squared NN distance both ways (train.py:80-84); (B,)."""
    if pred.is_cuda and pred.dtype == torch.float32 and target.dtype == torch.float32:
        from chamfer3D.dist_chamfer_3D import chamfer_3DDist
        d1, d2, _, _ = chamfer_3DDist()(pred.contiguous(), target.contiguous())
        return d1.mean(dim=1) + d2.mean(dim=1)
    d2 = torch.cdist(pred, target, p=2).pow(2)
    return d2.min(dim=2).values.mean(dim=1) + d2.min(dim=1).values.mean(dim=1)


__all__ = ["heun", "dopri5", "pf_prior_like", "generate", "chamfer_l2"]
