"""Point-cloud generation and the Chamfer metric of the flow model (SURVEY.md
section 8 f3; BASELINE.json configs[3]).

* `heun` -- the reference's predictor-corrector loop (train.py:332-341, 385-415):
  t_k = k / steps, x <- x + dt/2 (v(x, t_k) + v(x + dt v(x, t_k), t_{k+1})).
* `dopri5` -- adaptive Dormand-Prince 5(4), the solver the reference vendors
  (third_party/torchdiffeq 0.2.2, `odeint(..., method='dopri5')`) but never
  calls, restated step for step: Hairer's initial step, RMS error ratio,
  accepted steps never shrink the next one, and x(t1) read off the last step's
  dense-output quartic (pinned against the vendored solver's own outputs:
  tests/golden/dopri5_torchdiffeq.npz).  `fixed_steps=k` runs k equal steps.
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


# Dormand-Prince 5(4) as torchdiffeq 0.2.2 runs it (the version the reference
# vendors: third_party/torchdiffeq/torchdiffeq/_impl/dopri5.py:5-36 tableau and
# dense-output midpoint weights, rk_common.py:40-93 / :235-319 step and state
# machine, misc.py:31-102 initial step / error ratio / step-size update,
# interp.py:1-48 the quartic dense output).  The published coefficients:
_DP_ALPHA = (1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0, 1.0)
_DP_BETA = ((1 / 5,),
            (3 / 40, 9 / 40),
            (44 / 45, -56 / 15, 32 / 9),
            (19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729),
            (9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656),
            (35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84))
# 5th-order weights minus the embedded 4th-order ones (Shampine's error estimate)
_DP_ERR = (35 / 384 - 1951 / 21600, 0.0, 500 / 1113 - 22642 / 50085, 125 / 192 - 451 / 720,
           -2187 / 6784 - -12231 / 42400, 11 / 84 - 649 / 6300, -1.0 / 60.0)
# y(t0 + dt/2) = y0 + dt * sum_i mid_i k_i (Shampine 1986), for the dense output
_DP_MID = (6025192743 / 30085553152 / 2, 0.0, 51252292925 / 65400821598 / 2,
           -2691868925 / 45128329728 / 2, 187940372067 / 1594534317056 / 2,
           -1776094331 / 19743644256 / 2, 11237099 / 235043384 / 2)
_SAFETY, _IFACTOR, _DFACTOR, _ORDER = 0.9, 10.0, 0.2, 5


def _rms(x: torch.Tensor) -> torch.Tensor:
    """torchdiffeq's default norm (misc.py:19-20): RMS over the whole state."""
    return x.pow(2).mean().sqrt()


class _Tableau:
    """The coefficients in the state's dtype, as the solver casts them
    (rk_common.py:212-216): float64 values rounded once to y's dtype."""

    def __init__(self, dtype, device):
        def t(v):
            return torch.tensor(v, dtype=torch.float64).to(device=device, dtype=dtype)
        self.alpha = t(_DP_ALPHA)
        self.beta = [t(b) for b in _DP_BETA]
        self.err = t(_DP_ERR)
        self.mid = t(_DP_MID)


def _initial_step(f, t0, y0, f0, rtol, atol) -> torch.Tensor:
    """Hairer, Norsett & Wanner I, II.4 with the solver's order - 1 = 4 (misc.py:31-72);
    evaluated in y's dtype, returned in the time dtype."""
    dtype, t_dtype = y0.dtype, t0.dtype
    t0 = t0.to(dtype)
    scale = atol + torch.abs(y0) * rtol
    d0, d1 = _rms(y0 / scale), _rms(f0 / scale)
    if d0 < 1e-5 or d1 < 1e-5:
        h0 = torch.tensor(1e-6, dtype=dtype, device=y0.device)
    else:
        h0 = 0.01 * d0 / d1
    f1 = f(t0 + h0, y0 + h0 * f0)
    d2 = _rms((f1 - f0) / scale) / h0
    if d1 <= 1e-15 and d2 <= 1e-15:
        h1 = torch.max(torch.tensor(1e-6, dtype=dtype, device=y0.device), h0 * 1e-3)
    else:
        h1 = (0.01 / max(d1, d2)) ** (1.0 / float(_ORDER))
    return torch.min(100 * h0, h1).to(t_dtype)


def _rk_step(f, tab: _Tableau, y0, f0, t0, dt, t1):
    """One Dormand-Prince step from (t0, y0) with FSAL slope f0 (rk_common.py:40-93):
    stages accumulated as matmuls over the slope stack k (..., 7); the stages at
    alpha = 1 are evaluated just below t1 (Perturb.PREV).  Returns (y1, f1,
    error estimate, k)."""
    t0, dt, t1 = t0.to(y0.dtype), dt.to(y0.dtype), t1.to(y0.dtype)
    k = torch.empty(*f0.shape, len(_DP_ALPHA) + 1, dtype=y0.dtype, device=y0.device)
    k[..., 0] = f0
    yi = y0
    for i, (alpha_i, beta_i) in enumerate(zip(tab.alpha, tab.beta)):
        if alpha_i == 1.0:
            ti, prev = t1, True
        else:
            ti, prev = t0 + alpha_i * dt, False
        yi = y0 + k[..., :i + 1].matmul(beta_i * dt).view_as(f0)
        k[..., i + 1] = f(ti, yi, prev)
    # the 5th-order weights equal the last stage's (FSAL): y1 is that stage's input
    return yi, k[..., -1], k.matmul(dt * tab.err), k


def _interp_fit(tab: _Tableau, y0, y1, k, dt):
    """Quartic through y0, y_mid, y1 with slopes f0, f1 (rk_common.py:313-319,
    interp.py:1-23); coefficients lowest power first."""
    dt = dt.type_as(y0)
    y_mid = y0 + k.matmul(dt * tab.mid).view_as(y0)
    f0, f1 = k[..., 0], k[..., -1]
    a = 2 * dt * (f1 - f0) - 8 * (y1 + y0) + 16 * y_mid
    b = dt * (5 * f0 - 3 * f1) + 18 * y0 + 14 * y1 - 32 * y_mid
    c = dt * (f1 - 4 * f0) - 11 * y0 - 5 * y1 + 16 * y_mid
    return [y0, dt * f0, c, b, a]


def _interp_eval(coeffs, t0, t1, t):
    """interp.py:26-48."""
    assert (t0 <= t) & (t <= t1), f"invalid interpolation {t0} <= {t} <= {t1}"
    x = ((t - t0) / (t1 - t0)).to(coeffs[0].dtype)
    total = coeffs[0] + x * coeffs[1]
    xp = x
    for c in coeffs[2:]:
        xp = xp * x
        total = total + xp * c
    return total


def _next_step(dt, ratio, safety, ifactor, dfactor):
    """misc.py:79-89: grow by up to 10x; shrink (down to 0.2x) only after a
    rejected step -- an accepted step never shrinks the next one."""
    if ratio == 0:
        return dt * ifactor
    if ratio < 1:
        dfactor = torch.ones((), dtype=dt.dtype, device=dt.device)
    ratio = ratio.type_as(dt)
    exponent = torch.tensor(_ORDER, dtype=dt.dtype, device=dt.device).reciprocal()
    return dt * torch.min(ifactor, torch.max(safety / ratio ** exponent, dfactor))


@torch.no_grad()
def dopri5(velocity: Velocity, x: torch.Tensor, t0: float = 0.0, t1: float = 1.0,
           rtol: float = 1e-5, atol: float = 1e-5, fixed_steps: Optional[int] = None,
           max_steps: int = 2 ** 31 - 1, trace: Optional[list] = None
           ) -> Tuple[torch.Tensor, int]:
    """Integrate dx/dt = velocity(x, t) from t0 to t1 < ... as
    `torchdiffeq.odeint(f, x, torch.tensor([t0, t1]), rtol=rtol, atol=atol,
    method='dopri5')[1]` computes it; returns (x(t1), NFE).

    Times are float64 tensors on x's device, the state and the coefficients in
    x's dtype; error ratio = RMS(err / (atol + rtol max(|y0|, |y1|))); a step is
    accepted at ratio <= 1; the last step overshoots t1 and x(t1) is read off
    the step's dense-output quartic.  `trace`, if given, collects the time of
    every velocity evaluation (as torchdiffeq's func sees it, in x's dtype).
    `fixed_steps=k` instead takes k equal Dormand-Prince steps ending exactly on
    t1, no error control (this build's fixed-grid variant; 1 + 6k evaluations)."""
    if float(t1) == float(t0):  # torchdiffeq rejects a degenerate grid (misc.py:101, :286)
        raise AssertionError("t must be strictly increasing or decreasing")
    if float(t1) < float(t0):
        # decreasing time as torchdiffeq integrates it (misc.py:259-269): t -> -t and
        # f -> -f(-t, y) over the increasing grid [-t0, -t1]
        def rev(y, s):
            if trace is not None:
                trace.append(float(-s[0]))
            return -velocity(y, -s)
        return dopri5(rev, x, -float(t0), -float(t1), rtol, atol, fixed_steps, max_steps, None)
    nfe = 0

    def f(t, y, prev=False):
        nonlocal nfe
        nfe += 1
        t = t.to(y.dtype)
        if prev:  # Perturb.PREV: the previous representable time (misc.py:212-228)
            t = torch.nextafter(t, t - 1)
        if trace is not None:
            trace.append(float(t))
        return velocity(y, t.reshape(1).expand(y.shape[0]))

    dev = x.device
    t_dtype = torch.promote_types(torch.float64, x.dtype)
    tab = _Tableau(x.dtype, dev)
    ta = torch.tensor(float(t0), dtype=t_dtype, device=dev)
    tb = torch.tensor(float(t1), dtype=t_dtype, device=dev)
    f0 = f(ta, x)
    if fixed_steps is not None:
        n = max(1, int(fixed_steps))
        y = x
        for i in range(n):
            s = ta + (tb - ta) * i / n
            e = tb if i == n - 1 else ta + (tb - ta) * (i + 1) / n
            y, f0, _, _ = _rk_step(f, tab, y, f0, s, e - s, e)
        return y, nfe
    rtol_t = torch.as_tensor(rtol, dtype=t_dtype, device=dev)
    atol_t = torch.as_tensor(atol, dtype=t_dtype, device=dev)
    safety = torch.as_tensor(_SAFETY, dtype=t_dtype, device=dev)
    ifactor = torch.as_tensor(_IFACTOR, dtype=t_dtype, device=dev)
    dfactor = torch.as_tensor(_DFACTOR, dtype=t_dtype, device=dev)
    dt = _initial_step(f, ta, x, f0, rtol_t, atol_t)
    # state of the last step: (y1, f1, its start, its end, next dt, dense output)
    y, fy, s0, s1, coeffs = x, f0, ta, ta, [x] * 5
    n_steps = 0
    while tb > s1:
        assert n_steps < max_steps, f"max_num_steps exceeded ({n_steps}>={max_steps})"
        start = s1
        end = start + dt
        assert end > start, f"underflow in dt {dt.item()}"
        assert torch.isfinite(y).all(), "non-finite values in state `y`"
        y1, f1, err, k = _rk_step(f, tab, y, fy, start, dt, end)
        ratio = _rms(err / (atol_t + rtol_t * torch.max(y.abs(), y1.abs())))
        if ratio <= 1:
            coeffs = _interp_fit(tab, y, y1, k, dt)
            y, fy, s1 = y1, f1, end
        s0 = start
        dt = _next_step(dt, ratio, safety, ifactor, dfactor)
        n_steps += 1
    return _interp_eval(coeffs, s0, s1, tb), nfe


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
