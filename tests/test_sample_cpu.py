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


def test_dopri5_degenerate_and_reversed_spans():
    # torchdiffeq: equal times are rejected (misc.py:101, :286); a decreasing span is
    # integrated as -f(-t, y) over the negated grid (misc.py:259-269)
    x0 = torch.tensor([[1.0, 0.5]], dtype=torch.float64)
    with pytest.raises(AssertionError, match="strictly increasing or decreasing"):
        sample.dopri5(lambda x, t: -x, x0, t0=0.5, t1=0.5)
    seen = []
    x, nfe = sample.dopri5(lambda x, t: (seen.append(float(t[0])), -x)[1], x0, t0=1.0, t1=0.0,
                           rtol=1e-9, atol=1e-9)
    assert torch.allclose(x, x0 * math.e, rtol=1e-7, atol=0)
    assert len(seen) == nfe and seen[0] == 1.0 and max(seen) == 1.0  # the user sees t, not -t


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


# ---------------------------------------------------------------------------
# dopri5 against the reference's vendored torchdiffeq 0.2.2 (the golden's own
# outputs: tests/golden/make_dopri5_golden.py)
# ---------------------------------------------------------------------------
def _golden_case(golden, name):
    import numpy as np
    g = golden("dopri5_torchdiffeq.npz")
    return (torch.from_numpy(g[f"{name}_y0"]), g[f"{name}_y1"], g[f"{name}_times"],
            int(g[f"{name}_nfe"]), tuple(float(v) for v in g[f"{name}_tol"]), np)


def _field(name):
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_dopri5_golden as M
    if name == "decay_f64":
        return lambda y, t: -(1.0 + t[:, None]) * y
    dtype = torch.float64 if "_f64_" in name else torch.float32
    return M.tanh_field(dtype)[0]


@pytest.mark.parametrize("name", ["decay_f64", "tanh_f64_3", "tanh_f64_5", "tanh_f32_3",
                                  "tanh_f32_5"])
def test_dopri5_matches_vendored_torchdiffeq(golden, name):
    """Same NFE, the same evaluation times (the accepted / rejected step
    sequence) and y(1) within 1e-5 of the vendored solver's (in practice
    bit-equal: the same tensor operations in the same order)."""
    y0, y1_ref, times_ref, nfe_ref, (rtol, atol), np = _golden_case(golden, name)
    times = []
    y1, nfe = sample.dopri5(_field(name), y0, rtol=rtol, atol=atol, trace=times)
    assert nfe == nfe_ref
    np.testing.assert_array_equal(np.array(times), times_ref)
    y1 = y1.numpy()
    assert np.abs(y1 - y1_ref).max() <= 1e-5 * np.abs(y1_ref).max()
    np.testing.assert_array_equal(y1, y1_ref)


def test_dopri5_decay_closed_form(golden):
    y0, y1_ref, _, _, _, np = _golden_case(golden, "decay_f64")
    exact = y0.numpy() * math.exp(-1.5)
    assert np.abs(y1_ref - exact).max() < 1e-5


@pytest.fixture(scope="module")
def c1_ema_flow():
    """The C1 hybrid point flow with the EMA weights after replaying the
    reference's two recorded steps on the product CPU backend."""
    import os
    import sys
    import numpy as np
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from train_replay import replay
    g = np.load(os.path.join(here, "golden", "train_step_c1.npz"), allow_pickle=False)
    _, _, tr = replay(g, "cpu")
    tr.ema_pf.copy_to(tr.pf)
    tr.pf.eval()
    return tr.pf


def test_dopri5_hybrid_flow_matches_vendored_torchdiffeq(golden, c1_ema_flow):
    """The C1 hybrid flow through dopri5 (BASELINE configs[3]'s sampler) at
    rtol = atol = 1e-3: NFE and evaluation times equal to torchdiffeq's, y(1)
    within 1e-5.  (The golden's 1e-5 case runs on the GPU only,
    test_gpu_sample.py: at ~3.7 s per CPU velocity its 38 evaluations do not
    fit the CPU suite.  At that tolerance an fp32 state's error estimate,
    ~1e-5 |y|, is a difference of stage slopes that carries their rounding, so
    velocities that differ in their last bits -- the CPU GEMMs' thread count --
    move the accepted step sizes by ~1e-4 relative; same-thread-count runs
    reproduce the golden bit for bit.)"""
    x0, y1_ref, times_ref, nfe_ref, (rtol, atol), np = _golden_case(golden, "hybrid_c1_3")
    cond = torch.from_numpy(golden("train_step_c1.npz")["recon_cond"])
    times = []
    y1, nfe = sample.dopri5(lambda x, t: c1_ema_flow.guided_velocity(x, t, cond), x0,
                            rtol=rtol, atol=atol, trace=times)
    assert nfe == nfe_ref
    np.testing.assert_allclose(np.array(times), times_ref, rtol=1e-6, atol=0)
    assert np.abs(y1.numpy() - y1_ref).max() <= 1e-5 * np.abs(y1_ref).max()
