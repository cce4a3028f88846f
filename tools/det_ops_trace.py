"""Dev probe: trace every pcfm.ops call of the point flow's forward (inputs and
outputs cloned), run it several times on identical inputs, and report the
first op call whose inputs are bitwise equal to run 0's but whose outputs are
not -- the op that is not reproducible in context.  Run two copies at once to
put the GPU under contention.  JSON lines."""
import functools
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402

from pcfm import ops  # noqa: E402
from pcfm.train import TrainConfig, Trainer  # noqa: E402

TRACE = []


def _tensors(x):
    if isinstance(x, torch.Tensor):
        # expanded stand-ins (stride 0, e.g. shape probes of an empty scalar) hold no data
        return [] if 0 in x.stride() and x.numel() > 1 else [x]
    if isinstance(x, (list, tuple)):
        return [t for e in x for t in _tensors(e)]
    if hasattr(x, "__dict__") and not isinstance(x, type):
        return [v for v in vars(x).values() if isinstance(v, torch.Tensor)]
    return []


def wrap(name, fn):
    @functools.wraps(fn)
    def inner(*a, **k):
        ins = [t.detach().clone() for t in _tensors(list(a) + list(k.values()))]
        out = fn(*a, **k)
        outs = [t.detach().clone() for t in _tensors(out)]
        # in-place ops: the inputs after the call too
        post = [t.detach().clone() for t in _tensors(list(a))]
        TRACE.append((name, ins, outs, post))
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
    for m in tr.pf.modules():  # running statistics frozen: every run sees the same inputs
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.momentum = 0.0
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(b, n, 6, device=dev, generator=g)
    t = torch.rand(b, device=dev, generator=g)
    cond = torch.randn(b, cfg.latent_dim + cfg.cond_dim, device=dev, generator=g)
    runs = []
    for _ in range(int(os.environ.get("RUNS", "6"))):
        TRACE.clear()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            tr.pf(x, t, cond, cond_drop_mask=None)
        torch.cuda.synchronize()
        runs.append(list(TRACE))

    def eq(a, c):
        # uint8 images / workspaces carry uninitialised padding; int64 counters
        # (num_batches_tracked) advance by design
        return len(a) == len(c) and all(
            u.dtype in (torch.uint8, torch.int64) or (u.shape == v.shape and torch.equal(u, v))
            for u, v in zip(a, c))
    for k in range(1, len(runs)):
        first = None
        for i, ((n0, i0, o0, p0), (n1, i1, o1, p1)) in enumerate(zip(runs[0], runs[k])):
            if n0 != n1:
                first = {"call": i, "op": n0, "other": n1, "why": "sequence differs"}
                break
            if not eq(i0, i1):
                bad = [(j, list(u.shape), str(u.dtype), float((u.double() - v.double()).abs().max()))
                       for j, (u, v) in enumerate(zip(i0, i1))
                       if u.dtype not in (torch.uint8, torch.int64) and not torch.equal(u, v)]
                first = {"call": i, "op": n0, "why": "inputs differ (an earlier op or a race)",
                         "inputs": bad, "prev_ops": [runs[0][q][0] for q in range(max(0, i - 4), i)]}
                break
            if not eq(o0, o1) or not eq(p0, p1):
                det = []
                for j, (u, v) in enumerate(zip(o0, o1)):
                    if u.shape == v.shape and not torch.equal(u, v):
                        d = u != v
                        det.append({"output": j, "shape": list(u.shape), "dtype": str(u.dtype),
                                    "n_diff": int(d.sum()), "first_idx": d.nonzero()[:6].tolist(),
                                    "max_abs": float((u.double() - v.double()).abs().max())})
                first = {"call": i, "op": n0, "why": "same inputs, different outputs",
                         "outputs": det, "in_shapes": [list(t.shape) for t in i0]}
                break
        print(json.dumps({"run": k, "n_calls": len(runs[k]), "first": first}), flush=True)


if __name__ == "__main__":
    main()
