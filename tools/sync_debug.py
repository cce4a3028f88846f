"""Report host<->device synchronisations inside one train step (dev tool)."""
import os
import sys
import traceback
import warnings

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
import torch  # noqa: E402

from pcfm.train import TrainConfig, Trainer, synthetic_batch  # noqa: E402

dev = torch.device("cuda", 0)
cfg = TrainConfig()
tr = Trainer(cfg, dev)
tr.train_mode()
batch = synthetic_batch(cfg, dev, generator=torch.Generator(device=dev).manual_seed(1))
for _ in range(3):
    tr.step(batch, 201)
torch.cuda.synchronize()
seen = {}


def show(message, category, filename, lineno, file=None, line=None):
    stack = "".join(traceback.format_stack(limit=12)[:-2])
    key = stack[-600:]
    seen[key] = seen.get(key, 0) + 1


warnings.showwarning = show
torch.cuda.set_sync_debug_mode("warn")
tr.step(batch, 201)
torch.cuda.set_sync_debug_mode(0)
for k, v in seen.items():
    print(f"--- {v}x\n{k}")
print("syncs:", sum(seen.values()))
