"""One rank of tests/test_gpu_ddp.py::test_ddp_grad_is_mean_of_shard_grads --
SURVEY.md §8(e)'s data-parallel contract on the HIP path:

* each rank's forward on its B=8 shard equals the one-process forward on that
  shard (the losses, bit for bit: same parameters, same injected draws);
* after the backward, every rank's gradient (DDP's all-reduce, train.py:240-244)
  equals the mean of the two one-process per-shard gradients.

The one-process reference is a plain (non-DDP) Trainer holding the same
parameters, run once per shard in this process.  BatchNorm uses each shard's
batch statistics in both, as the reference's broadcast_buffers=False DDP does.
Writes {rank, losses, ref_losses, max_rel, bit_equal, grad_sums} to argv[1].rank."""
import json
import os
import sys

if os.environ.get("PCFM_DDP_CU_SPLIT") == "1":
    # diagnosis: each rank's queues on its own half of the GPU's 256 CUs, set
    # before the HIP runtime starts (ROCr reads HSA_CU_MASK at initialisation)
    _lr = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ["HSA_CU_MASK"] = "0:0-127" if _lr == 0 else "0:128-255"

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pcfm.train import TrainConfig, Trainer, init_distributed, synthetic_batch  # noqa: E402

B, N = 8, 4096
EPOCH = 201  # full 6-D loss, CFG drop at its final rate


def shard(cfg, s, dev):
    """Batch and injected random draws of shard s (CPU generator, then moved)."""
    g = torch.Generator().manual_seed(1000 + s)
    batch = {k: v.to(dev) for k, v in synthetic_batch(cfg, "cpu", generator=g).items()}
    z_pts = torch.cat([torch.randn(B, N, 3, generator=g), torch.rand(B, N, 3, generator=g)], -1)
    beta = torch.distributions.Beta(torch.tensor(cfg.t_beta_a), torch.tensor(1.0))
    torch.manual_seed(2000 + s)
    draws = {"z_pts": z_pts, "t_pts": beta.sample((B,)), "drop_u": torch.rand(B, generator=g),
             "eps_z": torch.randn(B, cfg.latent_dim, generator=g), "t_z": beta.sample((B,))}
    return batch, draws


TRACE = None  # PCFM_DDP_TRACE=1: per pcfm.ops call, checksums of its float outputs
KEEP = []  # ... and full copies of the devoxelization's inputs / outputs per call


def _trace_ops():
    """Wrap every pcfm.ops function so each call appends (name, [sum, abs-sum of
    every float output]) to TRACE (a diagnostic: where two runs of the same
    shard first part)."""
    import functools
    import types
    from pcfm import ops

    def outs(x):
        if isinstance(x, torch.Tensor):
            return [x]
        if isinstance(x, (list, tuple)):
            return [t for e in x for t in outs(e)]
        return []

    def sums(ts):
        return [(float(t.double().sum()), float(t.double().abs().sum()))
                for t in ts if t.is_floating_point() and t.numel()
                and not (0 in t.stride() and t.numel() > 1)]

    def wrap(name, fn):
        @functools.wraps(fn)
        def inner(*a, **k):
            out = fn(*a, **k)
            if TRACE is not None:
                TRACE.append((name, sums(outs(out))))
                if name == "trilinear_devoxelize_scale_add":  # full copies, after the call
                    KEEP.append([t.detach().clone() for t in outs(list(a)) + outs(out)])
            return out
        return inner
    for name in dir(ops):
        f = getattr(ops, name)
        if (isinstance(f, types.FunctionType) and not name.startswith("_")
                and f.__module__ == ops.__name__):
            setattr(ops, name, wrap(name, f))


def _first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return {"call": i, "op": x[0], "other_op": y[0], "a": x[1], "b": y[1]}
    return None if len(a) == len(b) else {"call": min(len(a), len(b)), "why": "lengths differ"}


def grads(tr):
    return [p.grad.detach().clone() if p.grad is not None else None for p in tr._clip_params]


def main():
    _, rank, world, local = init_distributed("gloo")
    assert world == 2
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    cfg = TrainConfig(batch_size=B, num_points=N, steps_per_epoch=4, epochs=1,
                      tunableop=False, miopen_find=False)
    tr = Trainer(cfg, dev, rank=rank, world_size=world, ddp=True)
    tr.train_mode()
    global TRACE
    tracing = os.environ.get("PCFM_DDP_TRACE") == "1"
    if tracing:
        _trace_ops()
    runs, kept = {}, {}
    TRACE = [] if tracing else None
    KEEP.clear()
    batch, draws = shard(cfg, rank, dev)
    out = tr.forward_backward(batch, EPOCH, draws)
    g_ddp = grads(tr)
    torch.cuda.synchronize(dev)
    runs["ddp"] = TRACE
    kept["ddp"] = list(KEEP)

    # one-process reference on the same (broadcast) parameters
    ref = Trainer(cfg, dev, rank=0, world_size=1, ddp=False)
    for a, b in ((ref.enc, tr.enc), (ref.pf, tr.pf), (ref.lf, tr.lf)):
        a.load_state_dict(b.state_dict())
    ref.train_mode()
    torch.cuda.synchronize(dev)
    per, ref_losses = [], []
    for s in range(world):
        ref.opt.zero_grad(set_to_none=True)
        bs, ds = shard(cfg, s, dev)
        TRACE = [] if tracing else None
        KEEP.clear()
        o = ref.forward_backward(bs, EPOCH, ds)
        ref_losses.append([float(o["loss_point"]), float(o["loss_latent"])])
        per.append(grads(ref))
        runs[f"ref{s}"] = TRACE
        kept[f"ref{s}"] = list(KEEP)
    # the reference once more on shard `rank`: names of gradients that are not
    # reproducible inside one process (diagnostic)
    ref.opt.zero_grad(set_to_none=True)
    bs, ds = shard(cfg, rank, dev)
    TRACE = [] if tracing else None
    KEEP.clear()
    ref.forward_backward(bs, EPOCH, ds)
    again = grads(ref)
    torch.cuda.synchronize(dev)
    runs["again"] = TRACE
    kept["again"] = list(KEEP)
    TRACE = None
    trace_diff = None
    if tracing:
        # the forward differs only where an op is not reproducible (the backward
        # of the DDP run sees all-reduced gradients, so compare up to its first
        # parameter-gradient op only through the ref runs)
        mine = runs[f"ref{rank}"]
        trace_diff = {"ddp_vs_ref": _first_diff(runs["ddp"], mine),
                      "ref_vs_again": _first_diff(mine, runs["again"]), "n_calls": len(mine),
                      "devox": {}}
        # element-level view of the devoxelization calls that differ
        for pair in (("ddp", f"ref{rank}"), (f"ref{rank}", "again")):
            for ci, (ta, tb) in enumerate(zip(kept[pair[0]], kept[pair[1]])):
                rep = []
                for ti, (u, v) in enumerate(zip(ta, tb)):
                    if u.shape == v.shape and not torch.equal(u, v):
                        d = (u != v)
                        idx = d.nonzero()
                        rep.append({"tensor": ti, "shape": list(u.shape), "n_diff": int(d.sum()),
                                    "first_idx": idx[:8].tolist(),
                                    "a": u[d][:8].tolist(), "b": v[d][:8].tolist()})
                if rep:
                    trace_diff["devox"][f"{pair[0]}-{pair[1]}#{ci}"] = rep
                    break

    names = ([f"enc.{n}" for n, _ in tr.enc.named_parameters()]
             + [f"pf.{n}" for n, _ in tr.pf.named_parameters()]
             + [f"lf.{n}" for n, _ in tr.lf.named_parameters()])
    max_rel, bit_equal, n_grads, differ = 0.0, 0, 0, {}
    for name, gd, g0, g1 in zip(names, g_ddp, per[0], per[1]):
        if gd is None:
            assert g0 is None and g1 is None
            continue
        n_grads += 1
        want = (g0 + g1) / world
        scale = want.abs().max().item()
        err = (gd - want).abs().max().item()
        rel = err / scale if scale > 0 else err
        max_rel = max(max_rel, rel)
        bit_equal += int(torch.equal(gd, want))
        if not torch.equal(gd, want):
            differ[name] = rel
    unrepro = [nm for nm, a, b_ in zip(names, per[rank], again)
               if a is not None and not torch.equal(a, b_)]
    sums = torch.tensor([g.double().sum().item() for g in g_ddp if g is not None],
                        dtype=torch.float64)
    gathered = [torch.zeros_like(sums) for _ in range(world)]
    dist.all_gather(gathered, sums)
    res = {"rank": rank, "world": world, "backend": dist.get_backend(),
           "losses": [float(out["loss_point"]), float(out["loss_latent"])],
           "ref_losses": ref_losses, "max_rel": max_rel, "bit_equal": bit_equal,
           "n_grads": n_grads, "differ": differ, "unreproducible": unrepro, "trace": trace_diff,
           "grad_sums_equal_across_ranks":
           all(torch.equal(gathered[0], g) for g in gathered),
           "cu_mask": os.environ.get("HSA_CU_MASK")}
    from pcfm import ops
    if ops.devox_verify.enabled:
        res["devox_verify"] = ops.devox_verify.report()
    with open(f"{sys.argv[1]}.{rank}", "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
