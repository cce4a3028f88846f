"""BASELINE.json configs[3]: point-cloud generation (inference path) on one
MI355X -- latent Heun + point-flow Heun (50 steps = 100 NFE, the reference's
sampler) or dopri5 -- with random-init hybrid models in eval mode.  Prints one
JSON line (generated points/s, ms per velocity evaluation).

    python tools/sample_bench.py [--batch 32] [--points 20000] [--method heun]
        [--steps 50] [--amp]   (--amp: bf16 autocast as in training; default fp32
                                as the reference's save_val_samples)
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

from pcfm import _lib  # noqa: E402
from pcfm.sample import chamfer_l2, generate  # noqa: E402
from pcfm.train import TrainConfig, build_models  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--points", type=int, default=20000)
    p.add_argument("--method", default="heun", choices=["heun", "dopri5", "dopri5_fixed"])
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--rtol", type=float, default=1e-3)
    p.add_argument("--atol", type=float, default=1e-3)
    p.add_argument("--guidance", type=float, default=0.0)
    p.add_argument("--amp", action="store_true")
    a = p.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = TrainConfig(batch_size=a.batch, num_points=a.points)
    _, pf, lf = build_models(cfg, dev)
    pf.eval()
    lf.eval()
    cond = torch.rand(a.batch, cfg.cond_dim, device=dev)
    kw = dict(point_dim=cfg.pf_point_dim, latent_dim=cfg.latent_dim, cond=cond,
              steps=a.steps, method=a.method, guidance_scale=a.guidance, rtol=a.rtol,
              atol=a.atol)
    ctx = torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.amp)
    with ctx:  # warm-up at the full shape (MIOpen/hipBLASLt selection)
        generate(pf, lf, a.batch, a.points, **{**kw, "steps": 1,
                                               "method": "heun" if a.method == "heun"
                                               else "dopri5_fixed"})
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with ctx:
        x, nfe = generate(pf, lf, a.batch, a.points, **kw)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    cd = float(chamfer_l2(x[..., :3].float().contiguous(),
                          torch.randn_like(x[..., :3].float())).mean())
    print(json.dumps({
        "metric": "generated points/s (BASELINE configs[3] sampling)", "value": a.batch * a.points / dt,
        "unit": "points/s", "seconds": dt, "nfe": nfe, "ms_per_nfe": dt * 1e3 / max(1, nfe),
        "config": {"batch": a.batch, "points": a.points, "method": a.method, "steps": a.steps,
                   "rtol": a.rtol, "atol": a.atol, "guidance": a.guidance,
                   "precision": "bf16 autocast head" if a.amp else "fp32 (reference eval)"},
        "finite": bool(torch.isfinite(x).all()), "chamfer_vs_gaussian": cd}), flush=True)


if __name__ == "__main__":
    main()
