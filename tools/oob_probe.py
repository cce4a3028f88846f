"""Dev probe: does any kernel read BatchNorm running statistics (which, in
training mode, only the statistics publisher may touch)?  Sets every BN's
momentum to 0 and its running_mean / running_var to 1e30, runs a forward +
backward, and reports the first pcfm.ops call / module whose float output
holds a value beyond 1e20 or a non-finite one (the op that read them, e.g. past
the end of a neighbouring allocation).  JSON lines."""
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


def _tensors(x):
    if isinstance(x, torch.Tensor):
        return [x]
    if isinstance(x, (list, tuple)):
        return [t for e in x for t in _tensors(e)]
    return []


def _check(where, out):
    for k, t in enumerate(_tensors(out)):
        if t.is_floating_point() and t.numel() and not (0 in t.stride() and t.numel() > 1):
            a = t.detach().float()
            bad = (~torch.isfinite(a)) | (a.abs() > 1e20)
            if bool(bad.any()):
                idx = bad.nonzero()[:4].tolist()
                BAD.append({"where": where, "output": k, "shape": list(t.shape),
                            "n_bad": int(bad.sum()), "first_idx": idx})


def wrap(name, fn):
    @functools.wraps(fn)
    def inner(*a, **k):
        out = fn(*a, **k)
        _check("ops." + name, out)
        return out
    return inner


def main():
    for name in dir(ops):
        f = getattr(ops, name)
        if callable(f) and not name.startswith("_") and getattr(f, "__module__", "") == ops.__name__:
            setattr(ops, name, wrap(name, f))
    dev = torch.device("cuda", 0)
    b, n = int(os.environ.get("B", "8")), int(os.environ.get("N", "4096"))
    cfg = TrainConfig(batch_size=b, num_points=n, tunableop=False, miopen_find=False)
    tr = Trainer(cfg, dev)
    tr.train_mode()
    nbn = 0
    for m in list(tr.enc.modules()) + list(tr.pf.modules()) + list(tr.lf.modules()):
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.momentum = 0.0
            with torch.no_grad():
                m.running_mean.fill_(1e30)
                m.running_var.fill_(3e30)
            nbn += 1
    for name, mod in list(tr.enc.named_modules()) + list(tr.pf.named_modules()):
        mod.register_forward_hook(lambda m, i, o, name=name: _check("module " + name, o))
    batch = synthetic_batch(cfg, dev, generator=torch.Generator(device=dev).manual_seed(3))
    torch.manual_seed(5)
    tr.opt.zero_grad(set_to_none=True)
    losses = tr.forward_backward(batch, 201)
    torch.cuda.synchronize()
    grads_bad = [nm for nm, p in tr.pf.named_parameters()
                 if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
    print(json.dumps({"bn_modules": nbn, "n_bad": len(BAD), "first_bad": BAD[:6],
                      "nonfinite_grads": grads_bad[:10],
                      "losses": [float(x) for x in losses] if isinstance(losses, (list, tuple))
                      else str(losses)}), flush=True)


if __name__ == "__main__":
    main()
