"""Dev probe: does any kernel of the train step read memory it never wrote?
After one warm-up step (the caching allocator then holds blocks of the step's
sizes), every free cached block is filled with NaN: tensors are allocated in
decreasing chunk sizes until the reserved-but-unallocated bytes are covered,
filled with NaN and freed.  Then one forward + backward runs with every
pcfm.ops call and module output checked; the first one whose floating output
holds a non-finite value read uninitialised memory (or propagated it: the
first in program order is the culprit).  JSON lines."""
import functools
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402

from pcfm import ops  # noqa: E402
from pcfm.train import TrainConfig, Trainer, synthetic_batch  # noqa: E402

BAD = []
ORDER = [0]


def _tensors(x):
    if isinstance(x, torch.Tensor):
        return [x]
    if isinstance(x, (list, tuple)):
        return [t for e in x for t in _tensors(e)]
    return []


def _check(where, out):
    ORDER[0] += 1
    for k, t in enumerate(_tensors(out)):
        if t.is_floating_point() and t.numel() and not (0 in t.stride() and t.numel() > 1):
            bad = ~torch.isfinite(t.detach().float())
            if bool(bad.any()):
                BAD.append({"order": ORDER[0], "where": where, "output": k,
                            "shape": list(t.shape), "n_bad": int(bad.sum()),
                            "first_idx": bad.nonzero()[:4].tolist()})


def wrap(name, fn):
    @functools.wraps(fn)
    def inner(*a, **k):
        out = fn(*a, **k)
        _check("ops." + name, out)
        return out
    return inner


def poison(dev):
    torch.cuda.synchronize(dev)
    free = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    held, total = [], 0
    for mb in (256, 64, 16, 4, 1):
        sz = mb << 20
        while total + sz <= free:
            try:
                t = torch.empty(sz // 4, dtype=torch.float32, device=dev)
            except torch.cuda.OutOfMemoryError:
                break
            t.fill_(float("nan"))
            held.append(t)
            total += sz
    # small pool (< 1 MiB blocks)
    for kb in (512, 128, 32, 8, 2):
        for _ in range(64):
            t = torch.empty((kb << 10) // 4, dtype=torch.float32, device=dev)
            t.fill_(float("nan"))
            held.append(t)
    torch.cuda.synchronize(dev)
    del held
    return free, total


def main():
    dev = torch.device("cuda", 0)
    b, n = int(os.environ.get("B", "8")), int(os.environ.get("N", "4096"))
    cfg = TrainConfig(batch_size=b, num_points=n, tunableop=False, miopen_find=False)
    tr = Trainer(cfg, dev)
    tr.train_mode()
    batch = synthetic_batch(cfg, dev, generator=torch.Generator(device=dev).manual_seed(3))
    torch.manual_seed(5)
    tr.opt.zero_grad(set_to_none=True)
    tr.forward_backward(batch, 201)  # warm-up: the allocator caches the step's block sizes
    tr.opt.zero_grad(set_to_none=True)
    free, filled = poison(dev)
    for name in dir(ops):
        f = getattr(ops, name)
        if callable(f) and not name.startswith("_") and getattr(f, "__module__", "") == ops.__name__:
            setattr(ops, name, wrap(name, f))
    for name, mod in list(tr.enc.named_modules()) + list(tr.pf.named_modules()):
        mod.register_forward_hook(lambda m, i, o, name=name: _check("module " + name, o))
    torch.manual_seed(5)
    losses = tr.forward_backward(batch, 201)
    torch.cuda.synchronize()
    grads_bad = [nm for nm, p in list(tr.pf.named_parameters()) + list(tr.enc.named_parameters())
                 if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
    print(json.dumps({"free_cached": free, "poisoned": filled, "n_bad": len(BAD),
                      "first_bad": BAD[:8], "nonfinite_grads": grads_bad[:12],
                      "losses": {k: float(v) for k, v in losses.items()}}), flush=True)


if __name__ == "__main__":
    main()
