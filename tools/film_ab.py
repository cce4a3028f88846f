"""A/B timing of the head FiLM backward row pass at the C2 train-step shape
(B=8, N=20000, W=512; dev tool): u read back vs u recomputed (u=None), plus
the forward pass.  JSON line."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402
from tools.scatter_ab import timeit  # noqa: E402


def main():
    b, n, w = 8, 20000, 512
    g = torch.Generator(device="cuda").manual_seed(0)
    rnd = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
    gamma, beta = 1.0 + 0.2 * rnd(w), 0.2 * rnd(w)
    sp1, sh = (1.0 + 0.1 * rnd(b, w)).bfloat16(), (0.1 * rnd(b, w)).bfloat16()
    uprev, gprev = rnd(b * n, w), rnd(b * n, w).bfloat16()
    u, a, mean, rstd = ops.head_film_fwd(None, uprev, gprev, gamma, beta, sp1, sh, n, 1e-5)
    dhn, da = rnd(b * n, w), rnd(b * n, w).bfloat16()
    res = {"tag": sys.argv[1] if len(sys.argv) > 1 else "main",
           "fwd_ms": timeit(lambda: ops.head_film_fwd(None, uprev, gprev, gamma, beta, sp1, sh, n,
                                                      1e-5)),
           "bwd_u_ms": timeit(lambda: ops.head_film_bwd(dhn, da, u, None, uprev, gprev, mean, rstd,
                                                        gamma, beta, sp1, n, want_dh=True)),
           "bwd_recompute_ms": timeit(lambda: ops.head_film_bwd(
               dhn, da, None, None, uprev, gprev, mean, rstd, gamma, beta, sp1, n, want_dh=True,
               shift=sh))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
