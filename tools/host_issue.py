"""Is the train step host-bound? (dev tool)  Times the bench's default step
(B=8, N=20000, hybrid) two ways over K steps after warm-up: the host time to
issue them (perf_counter before the final synchronize) and the wall time to
finish them.  When the issue time is close to the wall time, the GPU waits on
Python; when it is well below, the GPU queue stays full.  One JSON line."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm.train import TrainConfig, Trainer, synthetic_batch  # noqa: E402

K = int(os.environ.get("STEPS", "20"))
dev = torch.device("cuda", 0)
cfg = TrainConfig(batch_size=8, num_points=20000, pf_backbone="hybrid")
tr = Trainer(cfg, dev)
tr.train_mode()
batch = synthetic_batch(cfg, dev, generator=torch.Generator(device=dev).manual_seed(1234))
epoch = cfg.geom_warmup_epochs + 1
for _ in range(3):
    tr.step(batch, epoch)
torch.cuda.synchronize(dev)
res = {}
for rep in range(2):
    t0 = time.perf_counter()
    per = []
    for _ in range(K):
        s = time.perf_counter()
        tr.step(batch, epoch)
        per.append(time.perf_counter() - s)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    t_wall = time.perf_counter() - t0
    per.sort()
    res[f"rep{rep}"] = {"issue_ms_per_step": t_issue * 1e3 / K, "wall_ms_per_step": t_wall * 1e3 / K,
                        "host_step_ms_median": per[K // 2] * 1e3, "host_step_ms_min": per[0] * 1e3}
# the host's own cost of one step with the GPU idle before it (the queue empty)
torch.cuda.synchronize(dev)
t0 = time.perf_counter()
tr.step(batch, epoch)
res["host_ms_one_step_from_idle"] = (time.perf_counter() - t0) * 1e3
torch.cuda.synchronize(dev)
print(json.dumps(res), flush=True)
