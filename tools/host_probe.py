"""Is the bench train step host-bound?  Per step after a sync: the time the
host takes to issue the step (tr.step returns) and the GPU tail after it.
If issue ~ wall, the kernels wait on Python/launch overhead.  Dev tool."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import _lib  # noqa: E402
from pcfm.train import TrainConfig, Trainer, synthetic_batch  # noqa: E402


def main():
    _lib.load()
    dev = torch.device("cuda", 0)
    cfg = TrainConfig(batch_size=8, num_points=20000, pf_backbone="hybrid")
    tr = Trainer(cfg, dev)
    tr.train_mode()
    gen = torch.Generator(device=dev).manual_seed(1234)
    batch = synthetic_batch(cfg, dev, generator=gen)
    epoch = cfg.geom_warmup_epochs + 1
    for _ in range(5):
        tr.step(batch, epoch)
    torch.cuda.synchronize()
    iss, tail = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step(batch, epoch)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        iss.append(t1 - t0)
        tail.append(t2 - t1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        tr.step(batch, epoch)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 10
    iss.sort()
    tail.sort()
    print(f"issue {1e3 * iss[5]:.2f} ms (min {1e3 * iss[0]:.2f})  tail {1e3 * tail[5]:.2f} ms  "
          f"isolated {1e3 * (iss[5] + tail[5]):.2f} ms  pipelined wall {1e3 * wall:.2f} ms")


if __name__ == "__main__":
    main()
