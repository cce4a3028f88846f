"""Which torch (non-pcfm) kernels run in the bench train step, and from where
(dev tool): one profiled step of the bench workload under torch.profiler, the
aten ops that launch device work, grouped by op + input shapes, with the
innermost repo frames of their Python stacks.  Prints JSON lines."""
import json
import os
import sys
from collections import defaultdict

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]


_OURS = ("point-cloud-flow-matching_amd", "pcfm/", "modules/", "PyTorchEMD/", "chamfer3D/")


def main():
    from pcfm import _lib
    from pcfm.train import TrainConfig, Trainer, synthetic_batch
    _lib.load()
    dev = torch.device("cuda", 0)
    cfg = TrainConfig(batch_size=8, num_points=20000, pf_backbone="hybrid")
    tr = Trainer(cfg, dev)
    tr.train_mode()
    batch = synthetic_batch(cfg, dev, generator=torch.Generator(device=dev).manual_seed(1234))
    epoch = cfg.geom_warmup_epochs + 1
    for _ in range(3):
        tr.step(batch, epoch)
    torch.cuda.synchronize(dev)
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    cfgx = torch._C._profiler._ExperimentalConfig(verbose=True)  # populates e.stack
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True,
                                experimental_config=cfgx) as prof:
        tr.step(batch, epoch)
        torch.cuda.synchronize(dev)
    agg = defaultdict(lambda: {"calls": 0, "dev_us": 0.0})
    for e in prof.events():
        if not e.name.startswith("aten::") or e.device_type != torch.autograd.DeviceType.CPU:
            continue
        dev_us = sum(k.duration for k in e.kernels) if e.kernels else 0.0
        if dev_us <= 0:
            continue
        # the box runs a snapshot whose path differs from REPO: keep the package's frames
        frames = [f for f in (e.stack or []) if any(m in f for m in _OURS)
                  and "torch_ops.py" not in f and "site-packages" not in f]
        where = " <- ".join(f.split("/")[-1] for f in frames[:3])
        if not where:  # backward ops run on the autograd thread: name the node instead
            p = e.cpu_parent
            while p is not None and not p.name.startswith("autograd::engine"):
                p = p.cpu_parent
            where = p.name.split(": ")[-1] if p is not None else ""
        key = (e.name, str(e.input_shapes)[:120], where)
        agg[key]["calls"] += 1
        agg[key]["dev_us"] += dev_us
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["dev_us"])
    tot = sum(v["dev_us"] for _, v in rows)
    print(json.dumps({"total_aten_device_us": tot, "groups": len(rows)}))
    for (name, shapes, where), v in rows[:60]:
        print(json.dumps({"op": name, "us": round(v["dev_us"], 1), "calls": v["calls"],
                          "shapes": shapes, "where": where}))


if __name__ == "__main__":
    main()
