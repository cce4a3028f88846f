"""The train step against the REFERENCE's own executed train step
(tests/golden/train_step_c1.npz: /root/reference/train.py:553-673 run for two
steps at C1 by tests/golden/make_train_golden.py), replayed on the CPU through
this build's Trainer.step and its pure-PyTorch backend (BASELINE configs[0]).

Tolerances (deviation measures: tests/train_replay.py):
  * step 1 -- same weights, same batch and draws: losses, velocity (max-abs
    relative to max |v|), clip total norm and every non-noise gradient norm
    within 1e-5 relative (north_star's fp32 bound); the AdamW update sums
    within 1e-4 of one full lr step per element;
  * step 2 starts from weights that already differ where step 1's gradient
    was ~0 (AdamW moves an element by ~lr * sign(g) whatever |g| is, so
    rounding-level gradients flip whole-lr steps): losses and velocity still
    within 1e-5; gradient norms within 5e-3, updates within 2e-2 lr steps;
  * the reference's post-epoch Heun sampling with the EMA weights
    (train.py:282-429): every velocity evaluation and the final clouds within
    1e-5.
"""
import numpy as np
import pytest
import torch

import train_replay


@pytest.fixture(scope="module")
def replay_cpu(golden):
    torch.manual_seed(0)
    return train_replay.replay(golden("train_step_c1.npz"), "cpu")


def test_same_seed_same_initial_weights(replay_cpu):
    init = replay_cpu[0]
    assert init < 1e-12


def test_first_step_matches_reference(replay_cpu):
    s = replay_cpu[1][0]
    for k in ("loss_point", "loss_latent", "v", "total_norm", "grad_norm"):
        assert s[k] < 1e-5, (k, s)
    assert s["update"] < 1e-4 and s["ema"] < 1e-4, s


def test_second_step_matches_reference(replay_cpu):
    s = replay_cpu[1][1]
    for k in ("loss_point", "loss_latent", "v"):
        assert s[k] < 1e-5, (k, s)
    assert s["grad_norm"] < 5e-3 and s["update"] < 2e-2 and s["ema"] < 1e-3, s


def test_golden_records_the_reference_draw_sequence(golden):
    """The recorded step consumed exactly the reference's draws (train.py:271-276,
    :604-605, :617, :637, :639-640) and the drop mask follows drop_u < p."""
    g = golden("train_step_c1.npz")
    for i in range(int(g["n_steps"])):
        p = f"s{i}_"
        u = g[p + "drop_u"]
        assert np.array_equal(g[p + "mask"][:, 0], (u < 0.5).astype(np.float32))
        z = g[p + "z_pts"]
        assert z.shape == (2, 1024, 6) and 0.0 <= z[..., 3:].min() and z[..., 3:].max() < 1.0
        t = g[p + "t_pts"].astype(np.float32)[:, None, None]
        data = np.concatenate([g[p + "train_points"], g[p + "train_rgb"]], -1)
        np.testing.assert_allclose(g[p + "x_t"], (1 - t) * z + t * data, rtol=1e-6, atol=1e-6)


def test_heun_sampling_matches_reference(replay_cpu, golden):
    """After the epoch the reference samples with its EMA weights (Heun,
    train.py:282-429): the same prior draws through pcfm.sample.heun and the
    Trainer's EMA models give the same velocities and clouds within 1e-5."""
    dev = train_replay.replay_sampling(golden("train_step_c1.npz"), replay_cpu[2])
    for k, v in dev.items():
        assert v < 1e-5, (k, dev)
