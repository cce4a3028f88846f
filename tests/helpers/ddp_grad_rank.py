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
    batch, draws = shard(cfg, rank, dev)
    out = tr.forward_backward(batch, EPOCH, draws)
    g_ddp = grads(tr)
    torch.cuda.synchronize(dev)

    # one-process reference on the same (broadcast) parameters
    ref = Trainer(cfg, dev, rank=0, world_size=1, ddp=False)
    for a, b in ((ref.enc, tr.enc), (ref.pf, tr.pf), (ref.lf, tr.lf)):
        a.load_state_dict(b.state_dict())
    ref.train_mode()
    per, ref_losses = [], []
    for s in range(world):
        ref.opt.zero_grad(set_to_none=True)
        bs, ds = shard(cfg, s, dev)
        o = ref.forward_backward(bs, EPOCH, ds)
        ref_losses.append([float(o["loss_point"]), float(o["loss_latent"])])
        per.append(grads(ref))
    # the reference once more on shard `rank`: names of gradients that are not
    # reproducible inside one process (diagnostic)
    ref.opt.zero_grad(set_to_none=True)
    bs, ds = shard(cfg, rank, dev)
    ref.forward_backward(bs, EPOCH, ds)
    again = grads(ref)
    torch.cuda.synchronize(dev)

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
           "n_grads": n_grads, "differ": differ, "unreproducible": unrepro, "grad_sums_equal_across_ranks":
           all(torch.equal(gathered[0], g) for g in gathered)}
    with open(f"{sys.argv[1]}.{rank}", "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
