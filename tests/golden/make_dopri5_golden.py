"""Generate tests/golden/dopri5_torchdiffeq.npz by running the REFERENCE's vendored
ODE solver -- torchdiffeq 0.2.2 (/root/reference/third_party/torchdiffeq,
`odeint(func, y0, t=[0, 1], rtol, atol, method='dopri5')`) -- on the CPU.

Run in the build container, where the reference tree is mounted read-only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_dopri5_golden.py /root/reference

Nothing is copied out of the reference: torchdiffeq is imported by path and
run; the script records numbers.  Recorded per case: the initial state, the
number of velocity evaluations (NFE), the time of every evaluation as the
solver's func receives it, and the solution y(1).  Cases:
  * decay_f64: y' = -(1 + t) y, fp64 (closed form exp(-(t + t^2/2)));
  * tanh{32,64}_{f64,f32}_{3,5}: y' = tanh(y W + t b) on a (2, 32) state with a
    seeded W, b (fp64 / fp32 state; rtol = atol = 1e-3 / 1e-5);
  * hybrid_c1: the C1 hybrid point flow (HybridMLP.guided_velocity in eval
    mode) with the EMA weights after replaying the reference's two recorded
    train steps (tests/golden/train_step_c1.npz, tests/train_replay.py, the
    product's CPU backend), from that golden's `recon_x0` / `recon_cond`,
    rtol = atol = 1e-3 and 1e-5.  The velocity is this build's -- the case pins
    the solver around a real flow, the velocity itself is pinned elsewhere.
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd"),
                os.path.join(REPO, "tests")]


def tanh_field(dtype):
    g = torch.Generator().manual_seed(64)
    w = (torch.randn(32, 32, generator=g, dtype=torch.float64) * 0.6).to(dtype)
    b = torch.randn(32, generator=g, dtype=torch.float64).to(dtype)
    y0 = torch.randn(2, 32, generator=g, dtype=torch.float64).to(dtype)
    return (lambda y, t: torch.tanh(y @ w + t[:, None] * b)), y0


def cases():
    """(name, velocity(y, t_vec), y0, rtol, atol); velocity(y, t) with t (B,)."""
    out = []
    y0 = torch.tensor([[1.0, -0.5, 2.0, 0.25], [3.0, 0.1, -1.0, 0.0], [0.5, 0.5, 0.5, -2.0]],
                      dtype=torch.float64)
    out.append(("decay_f64", lambda y, t: -(1.0 + t[:, None]) * y, y0, 1e-6, 1e-6))
    for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        f, y0 = tanh_field(dtype)
        for tol, ttag in ((1e-3, "3"), (1e-5, "5")):
            out.append((f"tanh_{tag}_{ttag}", f, y0, tol, tol))
    return out


def hybrid_velocity():
    """The C1 hybrid flow with its post-replay EMA weights (CPU backend)."""
    from train_replay import replay
    g = np.load(os.path.join(HERE, "train_step_c1.npz"), allow_pickle=False)
    _, _, tr = replay(g, "cpu")
    tr.ema_pf.copy_to(tr.pf)
    tr.pf.eval()
    cond = torch.from_numpy(g["recon_cond"])
    x0 = torch.from_numpy(g["recon_x0"])
    return (lambda x, t: tr.pf.guided_velocity(x, t, cond, guidance_scale=0.0)), x0


def run(odeint, f, y0, rtol, atol):
    times = []

    def func(t, y):  # torchdiffeq calls func(t, y) with t a 0-dim tensor of y.dtype
        times.append(float(t))
        return f(y, t.reshape(1).expand(y.shape[0]))
    with torch.no_grad():
        sol = odeint(func, y0, torch.tensor([0.0, 1.0], dtype=torch.float64), rtol=rtol,
                     atol=atol, method="dopri5")
    return sol[1], np.array(times)


def main(ref_root: str) -> None:
    sys.path.insert(0, os.path.join(ref_root, "third_party", "torchdiffeq"))
    import torchdiffeq
    assert torchdiffeq.__version__ == "0.2.2", torchdiffeq.__version__
    from torchdiffeq import odeint
    torch.set_num_threads(1)
    rec = {"torchdiffeq_version": np.array(torchdiffeq.__version__)}
    names = []
    todo = cases()
    fh, xh = hybrid_velocity()
    todo += [("hybrid_c1_3", fh, xh, 1e-3, 1e-3), ("hybrid_c1_5", fh, xh, 1e-5, 1e-5)]
    for name, f, y0, rtol, atol in todo:
        y1, times = run(odeint, f, y0, rtol, atol)
        names.append(name)
        rec[f"{name}_y0"] = y0.numpy()
        rec[f"{name}_y1"] = y1.numpy()
        rec[f"{name}_times"] = times
        rec[f"{name}_nfe"] = np.array(len(times))
        rec[f"{name}_tol"] = np.array([rtol, atol])
        print(f"{name}: nfe {len(times)}, |y1| max {float(y1.abs().max()):.4g}")
    rec["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "dopri5_torchdiffeq.npz"), **rec)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
