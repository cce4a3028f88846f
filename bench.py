#!/usr/bin/env python
"""Benchmark: the reference's headline workload -- one flow-matching train step
of the hybrid PVConv backbone at B=8, N=20000 points, xyz+rgb (README.md:153,
BASELINE.json configs[1]) -- on N MI355X GPUs, data parallel.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Prints ONE JSON line on rank 0.  value = points/s of the whole job
(world * B * N * K / max-over-ranks wall time of K steps); inputs are resident
in HBM before the timed region.  Besides the contract fields it carries:
  roofline      the dominant hot-path kernel (by time inside the step), its
                algorithmic bytes / its HIP-event time, vs 8 TB/s
  cpu_baseline  the same train step on the host CPU (torch CPU + the C oracle
                behind modules.functional), on a bounded sample
  chamfer       Chamfer-3D fwd+bwd ms at the reference's published shape
                (32x2000 / 32x1000, 1.4 ms) and at the C2 shape
Progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "point-cloud-flow-matching_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "train-step points/sec (B=8, N=20000, xyz+rgb) at 1/2/4/8 MI355X; Chamfer ms"
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_DENSE_TF = 2500.0          # MI355X dense bf16 MFMA peak (no sparsity)
VOXEL_OPS = ("avg_voxelize_fwd", "avg_voxelize_bwd", "trilinear_devoxelize_fwd",
             "trilinear_devoxelize_bwd")  # the PVConv scatter/gather
BF16X3_PEAK_TF = BF16_DENSE_TF / 3  # fp32-equivalent peak of the 3-product split
H100_DERIVED_PTS = 1.88e6       # 25 s/epoch at <= 293 steps/epoch (derived)
# HBM bytes per launch of the voxel ops from rocprofv3 PMC passes (tools/op_traffic.py)
TRAFFIC_FILE = os.path.join(REPO, "profiles", "r01_traffic.json")


def measured_traffic(op):
    """Mean PMC traffic per launch of `op` over the bench's three stage shapes
    (each runs twice per step), or None when no PMC summary is committed."""
    try:
        data = json.load(open(TRAFFIC_FILE))["ops"]
    except (OSError, ValueError, KeyError):
        return None
    vals = [v["traffic_bytes"] for k, v in data.items() if k.split("@")[0] == op]
    return sum(vals) / len(vals) if len(vals) == 3 else None


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--points", type=int, default=20000)
    p.add_argument("--backbone", default="hybrid", choices=["hybrid", "mlp"])
    p.add_argument("--surface", action="store_true", help="points near the unit sphere")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-batch", type=int, default=2, help="CPU baseline sample batch")
    p.add_argument("--no-chamfer", action="store_true")
    p.add_argument("--no-event-timing", action="store_true")
    p.add_argument("--profile-steps", type=int, default=2,
                   help="untimed steps with HIP events around every op (per-kernel table)")
    return p.parse_args()


def chamfer_ms(dev, b, n, m, iters=20):
    from chamfer3D.dist_chamfer_3D import chamfer_3DDist
    cham = chamfer_3DDist()
    g = torch.Generator(device=dev).manual_seed(0)
    p1 = torch.rand(b, n, 3, device=dev, generator=g)
    p2 = torch.rand(b, m, 3, device=dev, generator=g)

    def once(fwd_only):
        x = p1.detach().requires_grad_(not fwd_only)
        d1, d2, _, _ = cham(x, p2)
        if not fwd_only:
            d1.sum().backward()  # unit_test.py:38-61 timings(): loss = sum(dist1)

    res = {}
    for fwd_only in (True, False):
        for _ in range(3):
            once(fwd_only)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(iters):
            once(fwd_only)
        torch.cuda.synchronize(dev)
        res["fwd" if fwd_only else "fwd_bwd"] = (time.perf_counter() - t0) * 1e3 / iters
    return res


def cpu_baseline(args, cfg_kwargs):
    """The reference's CPU-capable path (torch CPU, PVCNN ops through the C
    oracle), one train step on a bounded sample after one warm-up step."""
    from oracle.oracle import TorchBackend
    import modules.functional.backend as be
    from pcfm.train import TrainConfig, Trainer, synthetic_batch

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    saved = be._backend
    be._backend = TorchBackend()
    try:
        cfg = TrainConfig(**{**cfg_kwargs, "batch_size": args.cpu_batch})
        tr = Trainer(cfg, "cpu")
        tr.train_mode()
        batch = synthetic_batch(cfg, "cpu", surface=args.surface)
        tr.step(batch, epoch=201)
        t0 = time.perf_counter()
        tr.step(batch, epoch=201)
        dt = time.perf_counter() - t0
    finally:
        be._backend = saved
    pts = cfg.batch_size * cfg.num_points
    return {"value": pts / dt, "unit": "points/s", "cores": threads, "kind": "port",
            "sample": f"1 timed train step (after 1 warm-up) at B={cfg.batch_size}, "
                      f"N={cfg.num_points}, {cfg.pf_backbone} backbone, fp32 torch CPU + C "
                      f"oracle voxel ops; {dt:.2f} s/step",
            "seconds_per_step": dt}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ddp = world > 1
    if ddp:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from pcfm import _lib, ops
    from pcfm.train import TrainConfig, Trainer, synthetic_batch
    _lib.load()

    cfg_kwargs = dict(batch_size=args.batch, num_points=args.points, pf_backbone=args.backbone)
    cfg = TrainConfig(**cfg_kwargs)
    tr = Trainer(cfg, dev, rank=rank, world_size=world, ddp=ddp)
    tr.train_mode()
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    batch = synthetic_batch(cfg, dev, generator=gen, surface=args.surface)
    epoch = cfg.geom_warmup_epochs + 1  # full 6-D loss, CFG drop at its final rate

    t_w = time.perf_counter()
    for i in range(args.warmup):
        tr.step(batch, epoch)
        torch.cuda.synchronize(dev)
        if rank == 0:
            log(f"warmup step {i + 1}/{args.warmup} done ({time.perf_counter() - t_w:.1f} s)")

    # Per-op HIP-event profile over a few untimed steps: the per-kernel table, and
    # the choice of the roofline kernels.  Events around every op cost ~1.3 ms of
    # host time per step, so the timed region below records only those kernels.
    full, prof_steps = {}, 0
    roof_ops = set()
    if not args.no_event_timing:
        prof_steps = max(1, args.profile_steps)
        ops.timer.reset()
        ops.timer.only = None
        ops.timer.enabled = True
        for i in range(prof_steps):
            tr.step(batch, epoch)
        torch.cuda.synchronize(dev)
        ops.timer.enabled = False
        full = ops.timer.summary()
        if full:
            roof_ops.add(max(full, key=lambda k: full[k]["ms"]))
            hbm = [k for k in full if k in VOXEL_OPS]
            if hbm:
                roof_ops.add(max(hbm, key=lambda k: full[k]["ms"]))
    ops.timer.reset()
    ops.timer.only = roof_ops
    ops.timer.enabled = bool(roof_ops)
    if ddp:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        last = tr.step(batch, epoch)
        if rank == 0 and (i + 1) % max(1, args.steps // 4) == 0:
            log(f"timed step {i + 1}/{args.steps} issued")
    torch.cuda.synchronize(dev)
    if ddp:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ops.timer.enabled = False
    if ddp:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss_p, loss_z = float(last["loss_point"]), float(last["loss_latent"])

    if rank == 0:
        points = world * cfg.batch_size * cfg.num_points * args.steps
        value = points / elapsed
        ms = elapsed * 1e3 / args.steps
        summary = ops.timer.summary()  # the roofline kernels, live over the timed region
        rate_key = {"hbm": "GBps", "mfma": "TFLOPs_fp32_equiv", "mfma_bf16": "TFLOPs_bf16"}
        kernels = {k: {"launches_per_step": v["launches"] / prof_steps,
                       "ms_per_step": v["ms"] / prof_steps,
                       rate_key[v["kind"]]:
                       (v["amount"] / (v["ms"] * 1e-3) / (1e9 if v["kind"] == "hbm" else 1e12))
                       if v["ms"] > 0 else None}
                   for k, v in full.items()}

        def roof(op):
            d = summary[op]
            sec = d["ms"] * 1e-3
            if d["kind"] == "hbm":
                achieved = d["amount"] / sec / 1e9
                traffic = measured_traffic(op)
                return {"kernel": op, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                        "traffic_unit": "bytes per launch (PMC, profiles/r01_traffic.json)"
                        if traffic else None,
                        "algorithmic_bytes_per_launch": d["amount"] / d["launches"],
                        "avg_launch_ms": d["ms"] / d["launches"]}
            achieved = d["amount"] / sec / 1e12
            if d["kind"] == "mfma_bf16":
                return {"kernel": op, "bound": "mfma", "achieved": achieved,
                        "peak": BF16_DENSE_TF, "unit": "TFLOP/s",
                        "frac": achieved / BF16_DENSE_TF, "traffic": None,
                        "algorithmic_flops_per_launch": d["amount"] / d["launches"],
                        "avg_launch_ms": d["ms"] / d["launches"]}
            traffic = measured_traffic(op)
            return {"kernel": op, "bound": "mfma", "achieved": achieved, "peak": BF16X3_PEAK_TF,
                    "unit": "TFLOP/s", "frac": achieved / BF16X3_PEAK_TF, "traffic": traffic,
                    "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE + WRITE_SIZE, "
                                    "profiles/r01_traffic.json)" if traffic else None,
                    "note": "achieved = algorithmic fp32 conv FLOPs / time; each is 3 bf16 "
                            "MFMA products, so peak = dense bf16 2500 TF / 3; raw bf16 MFMA "
                            f"utilisation = {3 * achieved / BF16_DENSE_TF:.3f}",
                    "algorithmic_flops_per_launch": d["amount"] / d["launches"],
                    "avg_launch_ms": d["ms"] / d["launches"]}

        roofline = roof(max(summary, key=lambda k: summary[k]["ms"])) if summary else None
        hbm_ops = [k for k in summary if k in VOXEL_OPS]
        roofline_scatter = roof(max(hbm_ops, key=lambda k: summary[k]["ms"])) if hbm_ops else None
        log(f"{ms:.2f} ms/step, {value / 1e6:.3f} M points/s; losses {loss_p:.4f} {loss_z:.4f}")
        cham = None
        if not args.no_chamfer:
            cham = {"published_shape_32x2000x1000": chamfer_ms(dev, 32, 2000, 1000),
                    "published_fwd_bwd_ms": 1.4,
                    "c2_shape_8x20000x20000": chamfer_ms(dev, 8, 20000, 20000, iters=5),
                    "c5_shape_4x100000x100000": chamfer_ms(dev, 4, 100000, 100000, iters=2)}
            log(f"chamfer: {cham}")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline: running one warm-up + one timed CPU step ...")
            cpu = cpu_baseline(args, cfg_kwargs)
            log(f"cpu baseline: {cpu['seconds_per_step']:.2f} s/step")
        line = {
            "metric": METRIC, "value": value, "unit": "points/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "vs_h100_derived_upper_bound": value / H100_DERIVED_PTS,
            "dtype": "fp32 ContextNet (scatter/gather ops fp32; Conv3d + 1x1 convs as bf16x3 "
                     "split-operand matrix-core products, fp32 accumulate, ~2^-16 per product vs "
                     "the reference's default cuDNN TF32 2^-11) + bf16 autocast MLP head "
                     "(reference AMP config)",
            "data": "synthetic (randn xyz, U[0,1] rgb, U[0,1] cond; no dataset on the box)",
            "config": {"workload": f"{cfg.pf_backbone} flow-matching train step, "
                                   f"B={cfg.batch_size}/GPU, N={cfg.num_points} xyz+rgb, "
                                   "latent 128, 1 joint, stages (128,256,256)@(32,16,8)",
                       "global_batch": world * cfg.batch_size, "points_per_cloud": cfg.num_points,
                       "backbone": cfg.pf_backbone, "parallelism": f"dp{world}"},
            "roofline": roofline, "roofline_voxel_scatter_gather": roofline_scatter,
            "kernels": kernels, "cpu_baseline": cpu, "chamfer": cham,
            "loss_point": loss_p, "loss_latent": loss_z,
        }
        print(json.dumps(line), flush=True)
    if ddp:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
