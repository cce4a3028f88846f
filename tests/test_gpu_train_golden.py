"""GPU: the train step against the REFERENCE's executed train step
(tests/golden/train_step_c1.npz, /root/reference/train.py:553-673 at C1),
replayed through Trainer.step on the MI355X with the same weights, batches and
random draws (tests/train_replay.py).

  * exact-fp32 mode (pcfm.precision.exact_fp32, amp off -- the reference's CPU
    step is plain fp32): the HIP voxel/devox/BN/GN kernels plus exact fp32
    convolutions.  Step 1's losses, velocity, clip norm and gradient norms
    within 1e-5 relative (north_star), AdamW update sums within 1e-4 lr steps.
    Step 2 starts from weights that differ where step 1's gradient was ~0
    (AdamW moves such elements by ~lr * sign(rounding noise)): losses and v
    within 1e-5, gradient norms within 2e-2 (measured 6.6e-3 on MI355X, 8.7e-4
    on the CPU path), updates within 5e-2 lr steps.
  * bf16x3 mode (the default fp32 convolutions on the matrix cores, amp off):
    the measured deviation is reported and bounded at 1e-4 (step 1; step 2's
    AdamW-amplified gradient norms at 5e-2, as in exact fp32 plus the bf16x3
    rounding -- bounds in the test).
  * the reference's post-epoch Heun sampling with the EMA weights
    (train.py:282-429) replayed through pcfm.sample.heun: 1e-5 exact-fp32,
    1e-4 bf16x3.
  * dopri5 through pcfm.sample on the same EMA flow against the reference's
    vendored torchdiffeq 0.2.2 (tests/golden/dopri5_torchdiffeq.npz).
  * the production step (bf16 autocast on the head as the reference trains on
    GPU, train.py:580-645): reported and bounded at 2e-2 -- bf16 rounding.
"""
import numpy as np
import pytest
import torch

import train_replay

pytestmark = pytest.mark.gpu


def _run(golden, **kw):
    torch.manual_seed(0)
    return train_replay.replay(golden("train_step_c1.npz"), "cuda", **kw)


def test_exact_fp32_step_matches_reference(golden, report):
    from pcfm.precision import exact_fp32
    with exact_fp32():
        init, steps, tr = _run(golden, amp=False)
    report("train_golden_exact_fp32", steps)
    assert init < 1e-12
    s = steps[0]
    for k in ("loss_point", "loss_latent", "v", "total_norm", "grad_norm"):
        assert s[k] < 1e-5, (k, s)
    assert s["update"] < 1e-4 and s["ema"] < 1e-4, s
    s = steps[1]
    for k in ("loss_point", "loss_latent", "v"):
        assert s[k] < 1e-5, (k, s)
    assert s["grad_norm"] < 2e-2 and s["update"] < 5e-2 and s["ema"] < 1e-3, s
    with exact_fp32():
        smp = train_replay.replay_sampling(golden("train_step_c1.npz"), tr)
    report("sampling_golden_exact_fp32", smp)
    for k, v in smp.items():
        assert v < 1e-5, (k, smp)
    # dopri5 (BASELINE configs[3]) against the reference's vendored torchdiffeq
    # on the same EMA flow: NFE and step sequence equal at rtol = atol = 1e-3,
    # y(1) within 1e-5.  At 1e-5 the fp32 error estimate carries the slopes'
    # rounding (test_sample_cpu.py): the accepted step sizes move by ~1e-2
    # relative (measured on MI355X: same NFE 38, evaluation times 1.2e-2 apart),
    # so y(1) is held to three times the tolerance the solver was asked for
    # (measured 1.1e-5) and the NFE to within one step.
    with exact_fp32():
        d5 = train_replay.replay_dopri5(golden("dopri5_torchdiffeq.npz"),
                                        golden("train_step_c1.npz"), tr)
    report("dopri5_golden_exact_fp32", d5)
    r = d5["hybrid_c1_3"]
    assert r["nfe"] == r["nfe_ref"] and r["times"] < 1e-6 and r["y1"] < 1e-5, d5
    r = d5["hybrid_c1_5"]
    assert abs(r["nfe"] - r["nfe_ref"]) <= 6 and r["y1"] < 3e-5, d5


def test_bf16x3_step_deviation(golden, report):
    _, steps, tr = _run(golden, amp=False)
    report("train_golden_bf16x3", steps)
    s = steps[0]
    for k in ("loss_point", "loss_latent", "v", "total_norm"):
        assert s[k] < 1e-4, (k, s)
    # step 2 starts from AdamW-updated weights: elements whose step-1 gradient was
    # ~0 moved by ~lr * sign(rounding noise), which the SE MLP's weight gradients
    # (ds = sum over R^3 voxels of grid * g, cancelling) amplify -- measured on
    # MI355X: losses <= 3.5e-7, v 4.6e-6, grad norms 3.3e-2 (SE fc.0 weight;
    # 8.2e-4 in exact fp32), update 8.4e-3 lr steps, EMA 3.8e-5
    s = steps[1]
    for k in ("loss_point", "loss_latent", "v", "total_norm"):
        assert s[k] < 1e-4, (k, s)
    assert s["grad_norm"] < 5e-2 and s["update"] < 5e-2 and s["ema"] < 1e-3, s
    smp = train_replay.replay_sampling(golden("train_step_c1.npz"), tr)
    report("sampling_golden_bf16x3", smp)
    for k, v in smp.items():
        assert v < 1e-4, (k, smp)


def test_production_step_deviation(golden, report):
    _, steps, _ = _run(golden)  # amp=True: bf16 autocast head, as the reference on GPU
    report("train_golden_bf16_autocast", steps)
    s = steps[0]
    for k in ("loss_point", "loss_latent", "v"):
        assert np.isfinite(s[k]) and s[k] < 2e-2, (k, s)
