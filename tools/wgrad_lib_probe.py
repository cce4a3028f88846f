"""rows_wgrad vs the tuned library GEMM for the head's weight gradients (dev tool)."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402
from pcfm.train import enable_tunableop  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


enable_tunableop("gpurun_out/tunable_probe.csv", tune=True)
R = 160000
for m, n in [(512, 512), (512, 72), (128, 128)]:
    g = torch.Generator(device="cuda").manual_seed(m + n)
    dy = torch.randn(R, m, device="cuda", generator=g).bfloat16()
    x = torch.randn(R, n, device="cuda", generator=g).bfloat16()
    t1 = timeit(lambda: ops.rows_wgrad_bf16(dy, x))
    t2 = timeit(lambda: torch.mm(dy.t(), x))
    print(f"{m}x{n} over {R} rows: rows_wgrad {t1 * 1e3:.1f} us, tuned library mm {t2 * 1e3:.1f} us",
          flush=True)
