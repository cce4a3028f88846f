"""Attribute the bench train step's device time to aten ops / autograd nodes
(torch.profiler, shapes recorded), to find which model-level op each kernel
belongs to.  Dev tool: `python tools/aten_profile.py [steps] [key filter] > out.txt`."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from pcfm import _lib  # noqa: E402
from pcfm.train import TrainConfig, Trainer, synthetic_batch  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    _lib.load()
    cfg = TrainConfig()
    tr = Trainer(cfg, dev)
    tr.train_mode()
    batch = synthetic_batch(cfg, dev, generator=torch.Generator(device=dev).manual_seed(1234))
    for _ in range(3):
        tr.step(batch, 201)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        for _ in range(steps):
            tr.step(batch, 201)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    rows = sorted(ka, key=lambda e: -e.self_device_time_total)
    tot = sum(e.self_device_time_total for e in ka)
    print(f"total self device time {tot / 1e3 / steps:.2f} ms/step")
    pat = sys.argv[2].lower() if len(sys.argv) > 2 else None  # optional key filter
    for e in (rows if pat else rows[:120]):
        if e.self_device_time_total <= 0 or (pat and pat not in e.key.lower()):
            continue
        print(f"{e.self_device_time_total / 1e3 / steps:8.3f} ms {e.count // steps:4d}x  "
              f"{e.key[:60]:60s} {str(e.input_shapes)[:150]}")


if __name__ == "__main__":
    main()
