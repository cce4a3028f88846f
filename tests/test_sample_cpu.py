"""Samplers (pcfm/sample.py) on closed-form ODEs, the CPU Chamfer fallback,
and an end-to-end generation on CPU through the drop-in modules."""
import math

import pytest
import torch

from pcfm import sample


def test_heun_matches_its_recurrence():
    # dx/dt = -x: one Heun step multiplies by 1 - dt + dt^2 / 2 (train.py:332-341)
    x0 = torch.tensor([[1.0, -2.0]], dtype=torch.float64)
    steps = 7
    dt = 1.0 / steps
    x = sample.heun(lambda x, t: -x, x0, steps)
    assert torch.allclose(x, x0 * (1 - dt + dt * dt / 2) ** steps, rtol=1e-14, atol=0)


def test_heun_uses_the_reference_time_grid():
    seen = []
    sample.heun(lambda x, t: (seen.append(float(t[0])), torch.zeros_like(x))[1],
                torch.zeros(2, 3), 4)
    assert seen == [0.0, 0.25, 0.25, 0.5, 0.5, 0.75, 0.75, 1.0]


@pytest.mark.parametrize("rtol", [1e-5, 1e-8])
def test_dopri5_adaptive_accuracy(rtol):
    x0 = torch.tensor([[1.0, 0.5, -3.0]], dtype=torch.float64)
    x, nfe = sample.dopri5(lambda x, t: -x, x0, rtol=rtol, atol=rtol)
    assert torch.allclose(x, x0 * math.exp(-1.0), rtol=20 * rtol, atol=0)
    assert nfe > 6


def test_dopri5_is_exact_on_polynomials_in_t():
    # dx/dt = 4 t^3 -> x(1) = x0 + 1; a 5th-order method is exact for degree <= 4
    x0 = torch.zeros(1, 2, dtype=torch.float64)
    f = lambda x, t: (4 * t[:, None] ** 3).expand_as(x)  # noqa: E731
    x, _ = sample.dopri5(f, x0, fixed_steps=1)
    assert torch.allclose(x, x0 + 1.0, rtol=0, atol=1e-14)


def test_dopri5_fixed_steps_nfe():
    _, nfe = sample.dopri5(lambda x, t: -x, torch.ones(1, 1), fixed_steps=10)
    assert nfe == 1 + 10 * 6  # FSAL: 6 new evaluations per step


def test_chamfer_l2_cpu_formula():
    g = torch.Generator().manual_seed(0)
    a, b = torch.randn(2, 50, 3, generator=g), torch.randn(2, 40, 3, generator=g)
    d = ((a[:, :, None] - b[:, None]) ** 2).sum(-1)
    exp = d.min(2).values.mean(1) + d.min(1).values.mean(1)
    assert torch.allclose(sample.chamfer_l2(a, b), exp, rtol=1e-5, atol=1e-6)


def test_generate_end_to_end_cpu(oracle_backend):
    from pcfm.models import ConditionalLatentVelocityNet, HybridMLP
    torch.manual_seed(0)
    pf = HybridMLP(cond_dim=9, point_dim=6, ctx_dim=16, ctx_emb_dim=32, stage_channels=(16, 32),
                   stage_blocks=(1, 1), stage_res=(8, 4), pf_width=32, pf_depth=3,
                   pf_emb_dim=32).eval()
    lf = ConditionalLatentVelocityNet(8, cond_dim=0, width=32, depth=3, emb_dim=32).eval()
    cond = torch.rand(2, 1)
    x, nfe = sample.generate(pf, lf, 2, 200, point_dim=6, latent_dim=8, cond=cond, steps=3,
                             guidance_scale=1.5)
    assert x.shape == (2, 200, 6) and nfe == 6 and torch.isfinite(x).all()
    x2, nfe2 = sample.generate(pf, lf, 2, 200, point_dim=6, latent_dim=8, cond=cond, steps=2,
                               method="dopri5_fixed")
    assert x2.shape == (2, 200, 6) and nfe2 == 1 + 2 * 6
