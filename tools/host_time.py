"""Host (enqueue) time per train step vs device time per step (dev tool): if
the host needs as long as the device, the step is launch-bound."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
import torch  # noqa: E402

from pcfm.train import TrainConfig, Trainer, synthetic_batch  # noqa: E402

dev = torch.device("cuda", 0)
cfg = TrainConfig()
tr = Trainer(cfg, dev)
tr.train_mode()
batch = synthetic_batch(cfg, dev, generator=torch.Generator(device=dev).manual_seed(1))
for _ in range(5):
    tr.step(batch, 201)
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for _ in range(20):
    h0 = time.perf_counter()
    tr.step(batch, 201)
    host.append(time.perf_counter() - h0)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 20
host.sort()
print(f"wall {wall * 1e3:.2f} ms/step; host enqueue median {host[10] * 1e3:.2f} ms, "
      f"min {host[0] * 1e3:.2f}, max {host[-1] * 1e3:.2f}")
# a step the device has to wait for: enqueue with the queue empty
torch.cuda.synchronize()
h0 = time.perf_counter()
tr.step(batch, 201)
h1 = time.perf_counter()
torch.cuda.synchronize()
h2 = time.perf_counter()
print(f"single step: host {1e3 * (h1 - h0):.2f} ms, device tail after host {1e3 * (h2 - h1):.2f} ms")
