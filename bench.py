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
                algorithmic FLOPs / its HIP-event time
  roofline_step the whole step: sum_k FLOP_k / peak_k / t_step, against
                the bf16x3 and the fp32 peaks for the fp32 convs
  cpu_baseline  the same train step on the host CPU -- the reference's model
                math (per-point FiLM as models.py:135/594 computes it, fp32
                torch CPU convolutions) on this build's pure-PyTorch CPU
                backend (pcfm.cpu_ops) -- plus the reference's CPU Chamfer
                (train.py:80-84 cdist form), on bounded samples; the host CPU
                model, cores and threads are stated
  chamfer       Chamfer-3D fwd / fwd+bwd ms at the reference's published shape
                (32x2000 / 32x1000, 1.4 ms), at C2 and at C5, with the VALU
                roofline of the forward (8 FLOP per pair)
  emd, ball_query   EMD (approxmatch + matchcost, and backward) at N = 2048 / 4096
                and ball query at the C2 / C5 cloud sizes
  distributed   torch.distributed backend and world size as the run saw them
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

from pcfm.dist_env import pin_rccl_env  # noqa: E402

METRIC = "train-step points/sec (B=8, N=20000, xyz+rgb) at 1/2/4/8 MI355X; Chamfer ms"
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_VALU_TF = 157.3            # MI355X fp32 vector peak (Chamfer / ball query: VALU-bound)
BF16_DENSE_TF = 2500.0          # MI355X dense bf16 MFMA peak (no sparsity)
VOXEL_OPS = ("avg_voxelize_fwd", "avg_voxelize_bwd", "trilinear_devoxelize_fwd",
             "trilinear_devoxelize_bwd")  # the PVConv scatter/gather
BF16X3_PEAK_TF = BF16_DENSE_TF / 3  # fp32-equivalent peak of the 3-product split
H100_DERIVED_PTS = 1.88e6       # 25 s/epoch at <= 293 steps/epoch (derived)
# HBM bytes per launch of the voxel ops from rocprofv3 PMC passes (tools/op_traffic.py)
TRAFFIC_FILE = os.path.join(REPO, "profiles", "r06_traffic.json")


def measured_traffic(op, batch, points):
    """Mean PMC traffic per launch of `op` over the bench's three stage shapes
    (each runs twice per step), or None when no PMC summary is committed for
    this run's (B, N) -- the committed counters are per shape."""
    try:
        blob = json.load(open(TRAFFIC_FILE))
        data = blob["ops"]
    except (OSError, ValueError, KeyError):
        return None
    if (blob.get("batch", 8), blob.get("points", 20000)) != (batch, points):
        return None
    ops_ = op.split("+")  # several ops of one kernel: the mean over all their shapes
    vals = [v["traffic_bytes"] for k, v in data.items() if k.split("@")[0] in ops_]
    return sum(vals) / len(vals) if len(vals) == 3 * len(ops_) else None


# MFMA-pipe busy fractions of the conv kernels (rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES
# over GRBM_GUI_ACTIVE, tools/kernel_pmc.py at the C2 stage shapes)
KERNEL_PMC_FILE = os.path.join(REPO, "profiles", "r06_kernel_pmc.json")
# dense fwd / bwd-data: the slab form at r = 32 / 16, the LDS-DMA form at r = 8
CONV_KERNEL = {"conv3d_fwd": ("conv3_igemm_slab_kernel", "conv3_igemm_glds_kernel"),
               "conv3d_bwd_data": ("conv3_igemm_slab_kernel", "conv3_igemm_glds_kernel"),
               "conv3d_wgrad": ("conv3_wgrad3_kernel",)}
# launches that skip empty-voxel work (PVConv's first conv: chunk lists / tile
# masks) are timed under "<op>_sparse" with the DENSE algorithmic FLOPs as their
# amount, so they never stand for a roofline (their rate would overstate it)
SPARSE_SUFFIX = "_sparse"
# the dominant kernel of the step, conv3_igemm_glds, runs as two ops (forward and
# backward-data): its roofline is taken over both ops' dense launches together
IGEMM_OPS = ("conv3d_fwd", "conv3d_bwd_data")


# every kernel of the PVConv voxel scatter/gather machinery: the four ops and the
# segment plans (sort + work units) they run on
SCATTER_GATHER_OPS = VOXEL_OPS + ("avg_voxelize_plan", "trilinear_devoxelize_bwd_plan")


def scatter_gather_bytes(batch, points, stages=((128, 32), (256, 16), (256, 8)), blocks=2):
    """algorithmic bytes of every PVConv voxelize / devoxelize call of
    one train step, forward and backward (each distinct tensor read or written once):
    4.81 GB at C2 (B=8, N=20000)."""
    b, n, tot = batch, points, 0
    for c, r in stages:
        v = r ** 3
        vf = b * (3 * n * 4 + c * n * 4 + n * 4 + v * 4 + c * v * 4)
        vb = b * (c * v * 4 + n * 4 + v * 4 + c * n * 4)
        df = b * (3 * n * 4 + c * v * 4 + c * n * 4 + 16 * n * 4)
        db = b * (c * n * 4 + 16 * n * 4 + c * v * 4)
        tot += blocks * (vf + vb + df + db)
    return tot


# the train step's FLOPs as the reference executes them at C2
# (B=8, N=20000, hybrid): 1x1 convs 928.8 GFLOP (fp32), per-point head GEMMs
# 2679.8 (bf16 autocast), encoder + latent net 32 (bf16); the Conv3d FLOPs
# (4348.5 at C2) follow from the stage config.  Per-point terms scale with B*N,
# the Conv3d term with B (the grids are fixed-size).
SURVEY_C2_POINTS = 8 * 20000
SURVEY_STEP_GFLOP = {"pointwise_fp32": 928.8, "head_bf16": 2679.8, "enc_lf_bf16": 32.0}


def conv3d_step_flops(cfg):
    """fwd + bwd-data + wgrad of every 3x3x3 conv of the PVConv pyramid:
    3 x 2 B R^3 27 C^2 per conv, two convs per PVConv block."""
    tot = 0.0
    for c, nb, r in zip(cfg.ctx_stage_channels, cfg.ctx_stage_blocks, cfg.ctx_stage_res):
        tot += nb * 2 * 3 * 2.0 * cfg.batch_size * r ** 3 * 27 * c * c
    return tot


def step_roofline(cfg, ms):
    """SURVEY 8(d)'s train-step rate: sum_k FLOP_k / peak_k over t_step, against
    the fp32 convs' two candidate peaks: the bf16x3 matrix-core rate this build
    runs them at (2500 TF / 3) and the fp32 vector peak SURVEY priced them at
    (157.3 TF); the bf16 GEMMs at 2500 TF either way."""
    if cfg.pf_backbone != "hybrid":
        return None
    scale = cfg.batch_size * cfg.num_points / SURVEY_C2_POINTS
    conv = conv3d_step_flops(cfg)
    pw = SURVEY_STEP_GFLOP["pointwise_fp32"] * 1e9 * scale
    bf16 = (SURVEY_STEP_GFLOP["head_bf16"] + SURVEY_STEP_GFLOP["enc_lf_bf16"]) * 1e9 * scale
    out = {"definition": "sum_k FLOP_k / peak_k / t_step (SURVEY.md 8d, reference-as-executed "
                         "FLOPs: Conv3d and 1x1 convs fp32, head / encoder GEMMs bf16)",
           "gflop": {"conv3d_fp32": conv / 1e9, "pointwise_fp32": pw / 1e9,
                     "gemm_bf16": bf16 / 1e9}, "t_step_ms": ms}
    for key, fp32_peak in (("vs_bf16x3_peak", BF16X3_PEAK_TF), ("vs_fp32_peak", FP32_VALU_TF)):
        floor = ((conv + pw) / (fp32_peak * 1e12) + bf16 / (BF16_DENSE_TF * 1e12)) * 1e3
        out[key] = {"fp32_conv_peak_TF": fp32_peak, "bf16_peak_TF": BF16_DENSE_TF,
                    "floor_ms": floor, "frac": floor / ms}
    return out


def committed_mfma_busy(op):
    try:
        kern = json.load(open(KERNEL_PMC_FILE))["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    names = CONV_KERNEL.get(op.split("+")[0], ())
    # time-weighted (GRBM_GUI_ACTIVE) over the op's kernels in the committed pass
    num = den = 0.0
    for k, v in kern.items():
        if any(n in k for n in names) and "mfma_busy_frac" in v:
            t = v["mean_per_dispatch"].get("GRBM_GUI_ACTIVE", 0.0) * v.get("dispatches", 1)
            num += v["mfma_busy_frac"] * t
            den += t
    return num / den if den > 0 else None


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
    p.add_argument("--cpu-batch", type=int, default=8, help="CPU baseline sample batch")
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


def host_cpu():
    """lscpu's model name, sockets, cores and threads of the host."""
    info = {}
    try:
        import subprocess
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in txt.splitlines():
            k, _, v = line.partition(":")
            info[k.strip()] = v.strip()
    except Exception:  # noqa: BLE001 -- informational only
        pass
    out = {"model": info.get("Model name"), "logical_cpus": os.cpu_count()}
    try:
        out["physical_cores"] = int(info["Core(s) per socket"]) * int(info["Socket(s)"])
        out["threads_per_core"] = int(info["Thread(s) per core"])
    except (KeyError, ValueError):
        pass
    return out


def cpu_baseline(args, cfg_kwargs):
    """The reference's CPU-capable path: one train step of the same model on the
    host (fp32 torch CPU, the reference's per-point FiLM form, PVCNN ops on the
    pure-PyTorch CPU backend pcfm.cpu_ops -- the reference itself has no CPU
    backend), timed after one small warm-up step; and the reference's CPU
    Chamfer (train.py:80-84: cdist, squared, min both ways) on one cloud pair."""
    from pcfm.train import TrainConfig, Trainer, synthetic_batch

    # the host's physical cores (lscpu); the box caps OMP_NUM_THREADS at
    # its CPU share, so the count used is stated next to the host's core count
    host = host_cpu()
    want = host.get("physical_cores") or os.cpu_count() or 1
    torch.set_num_threads(int(want))
    threads = torch.get_num_threads()
    cfg = TrainConfig(**{**cfg_kwargs, "batch_size": args.cpu_batch, "film_per_point": True})
    tr = Trainer(cfg, "cpu")
    tr.train_mode()
    warm = TrainConfig(**{**cfg_kwargs, "batch_size": 1, "num_points": 2048})
    tr.step(synthetic_batch(warm, "cpu", surface=args.surface), epoch=201)
    batch = synthetic_batch(cfg, "cpu", surface=args.surface)
    t0 = time.perf_counter()
    tr.step(batch, epoch=201)
    dt = time.perf_counter() - t0
    pts = cfg.batch_size * cfg.num_points
    # the same step at the box's CPU share (16 threads: OMP_NUM_THREADS there), which
    # ran faster than the full core count in rounds 4-5; the FASTER of the two thread
    # counts is the headline baseline, the other is stated beside it
    runs = [{"cores": threads, "value": pts / dt, "seconds_per_step": dt}]
    if threads > 16:
        torch.set_num_threads(16)
        t0 = time.perf_counter()
        tr.step(batch, epoch=201)
        dt16 = time.perf_counter() - t0
        torch.set_num_threads(threads)
        runs.append({"cores": 16, "value": pts / dt16, "seconds_per_step": dt16})
    best = max(runs, key=lambda d: d["value"])
    other = [d for d in runs if d is not best]
    n = cfg.num_points
    g = torch.Generator().manual_seed(0)
    a, b = torch.rand(1, n, 3, generator=g), torch.rand(1, n, 3, generator=g)
    t1 = time.perf_counter()
    d2 = torch.cdist(a, b, p=2).pow(2)
    _ = d2.min(dim=2).values.mean(dim=1) + d2.min(dim=1).values.mean(dim=1)
    cd = time.perf_counter() - t1
    del d2
    return {"value": best["value"], "unit": "points/s", "cores": best["cores"], "kind": "port",
            "host_cpu": host,
            "sample": f"1 timed train step (after a B=1, N=2048 warm-up) at B={cfg.batch_size}, "
                      f"N={n}, {cfg.pf_backbone} backbone, fp32 torch CPU, per-point FiLM, "
                      f"pcfm.cpu_ops voxel ops, the faster of "
                      f"{' / '.join(str(d['cores']) for d in runs)} threads: {best['cores']} "
                      f"({best['seconds_per_step']:.2f} s/step)",
            "seconds_per_step": best["seconds_per_step"],
            "other_thread_counts": other,
            "chamfer_cdist_fwd_ms": {"shape": f"1x{n}x{n}", "ms": cd * 1e3,
                                     "c2_equivalent_ms": cd * 1e3 * cfg_kwargs["batch_size"]}}


def emd_ms(dev, b, n, iters=3):
    """EMD (PyTorchEMD/emd.py: approxmatch + matchcost) forward and fwd+bwd ms."""
    from PyTorchEMD.emd import earth_mover_distance
    g = torch.Generator(device=dev).manual_seed(0)
    p1 = torch.rand(b, n, 3, device=dev, generator=g)
    p2 = torch.rand(b, n, 3, device=dev, generator=g)
    res = {}
    # fwd_ms: inputs need no gradient (cost only, match not materialised);
    # fwd_with_match_ms: the forward a backward will follow (match written and kept)
    for key, grad, bwd in (("fwd_ms", False, False), ("fwd_with_match_ms", True, False),
                           ("fwd_bwd_ms", True, True)):
        for i in range(iters + 1):
            if i == 1:
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
            x = p1.detach().requires_grad_(grad)
            d = earth_mover_distance(x, p2, transpose=False)
            if bwd:
                d.sum().backward()
        torch.cuda.synchronize(dev)
        res[key] = (time.perf_counter() - t0) * 1e3 / iters
    # 10 levels x 3 passes over the B*N*M pairs, one exp each (emd_kernel.cu:44-154)
    res["exps_per_s_fwd"] = 30.0 * b * n * n / (res["fwd_ms"] * 1e-3)
    return res


def ball_query_ms(dev, b, n, m, radius, u, iters=5):
    from pcfm import ops
    g = torch.Generator(device=dev).manual_seed(0)
    pts = torch.rand(b, 3, n, device=dev, generator=g)
    ctr = torch.rand(b, 3, m, device=dev, generator=g)
    ops.ball_query(ctr, pts, radius, u)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(iters):
        ops.ball_query(ctr, pts, radius, u)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3 / iters
    return {"shape": f"B={b} N={n} M={m} radius={radius} U={u}", "ms": ms,
            "distance_tests_per_s_upper": b * m * n / (ms * 1e-3)}


def launch_ranks(args, backend):
    """`bench.py --gpus N` run directly (no WORLD_SIZE in the env): start N ranks
    as a `torch.distributed.run` child -- the reference's `torchrun --standalone
    --nproc_per_node=N` recipe (train.py:810-826) -- and exit with its code.
    Runs before anything touches the GPU (device_count() does not, on ROCm)."""
    import socket
    import subprocess
    ndev = torch.cuda.device_count()
    if backend == "nccl" and args.gpus > ndev:
        log(f"--gpus {args.gpus} but only {ndev} GPU(s) visible: one rank per GPU over RCCL")
        sys.exit(2)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    if backend == "nccl":
        pin_rccl_env(env)  # every rank's RCCL on the ring kernels (pcfm/dist_env.py)
    log("launching:", " ".join(cmd))
    sys.exit(subprocess.call(cmd, env=env))


def main():
    args = parse()
    # one process per GPU; PCFM_DIST_BACKEND=gloo rehearses the N > 1 path with
    # several ranks sharing the GPUs there are (dev knob; the product path is RCCL)
    backend = os.environ.get("PCFM_DIST_BACKEND", "nccl")
    if args.gpus < 1:
        log("--gpus must be >= 1")
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        launch_ranks(args, backend)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU")
        sys.exit(2)
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > ndev:
        log(f"{world} ranks but only {ndev} GPU(s) visible: one rank per GPU over RCCL")
        sys.exit(2)
    ddp = world > 1
    local = local % max(1, ndev)
    if ddp:
        if backend == "nccl":
            pin_rccl_env()  # ranks started by the driver's torch.distributed.run too
        torch.cuda.set_device(local)
        dist.init_process_group(backend, init_method="env://")
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
        if all(k in full for k in IGEMM_OPS):
            roof_ops.update(IGEMM_OPS)
        else:
            dense = [k for k in full if not k.endswith(SPARSE_SUFFIX)]
            if dense:
                roof_ops.add(max(dense, key=lambda k: full[k]["ms"]))
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
                       # sparse launches: the dense op's FLOPs / time (not a rate of work done)
                       rate_key[v["kind"]] + ("_dense_equivalent" if k.endswith(SPARSE_SUFFIX)
                                              else ""):
                       (v["amount"] / (v["ms"] * 1e-3) / (1e9 if v["kind"] == "hbm" else 1e12))
                       if v["ms"] > 0 else None}
                   for k, v in full.items()}

        def roof(op):
            if isinstance(op, tuple):  # one kernel over several ops: their launches together
                parts = [summary[o] for o in op]
                d = {"ms": sum(p["ms"] for p in parts), "amount": sum(p["amount"] for p in parts),
                     "launches": sum(p["launches"] for p in parts), "kind": parts[0]["kind"]}
                op = "+".join(op)
            else:
                d = summary[op]
            sec = d["ms"] * 1e-3
            if d["kind"] == "hbm":
                achieved = d["amount"] / sec / 1e9
                traffic = measured_traffic(op, cfg.batch_size, cfg.num_points)
                return {"kernel": op, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                        "traffic_unit": "bytes per launch (PMC, profiles/r06_traffic.json)"
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
            traffic = measured_traffic(op, cfg.batch_size, cfg.num_points)
            return {"kernel": op, "bound": "mfma", "achieved": achieved, "peak": BF16X3_PEAK_TF,
                    "unit": "TFLOP/s", "frac": achieved / BF16X3_PEAK_TF, "traffic": traffic,
                    "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE + WRITE_SIZE, "
                                    "profiles/r06_traffic.json)" if traffic else None,
                    "note": "achieved = algorithmic fp32 conv FLOPs / time; each is 3 bf16 "
                            "MFMA products, so peak = dense bf16 2500 TF / 3; raw bf16 MFMA "
                            f"utilisation = {3 * achieved / BF16_DENSE_TF:.3f}",
                    "mfma_busy_frac": committed_mfma_busy(op),
                    "mfma_busy_source": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8), "
                                        "profiles/r06_kernel_pmc.json (time-weighted "
                                        "over the slab and LDS-DMA forms)",
                    "algorithmic_flops_per_launch": d["amount"] / d["launches"],
                    "avg_launch_ms": d["ms"] / d["launches"]}

        dense = [k for k in summary if not k.endswith(SPARSE_SUFFIX) and k not in VOXEL_OPS]
        if all(k in summary for k in IGEMM_OPS):
            roofline = roof(IGEMM_OPS)
            roofline["kernel"] = "conv3_igemm_glds (conv3d_fwd + conv3d_bwd_data, dense launches)"
        else:
            roofline = roof(max(dense, key=lambda k: summary[k]["ms"])) if dense else None
        hbm_ops = [k for k in summary if k in VOXEL_OPS]
        roofline_scatter = roof(max(hbm_ops, key=lambda k: summary[k]["ms"])) if hbm_ops else None
        # the whole voxel scatter/gather chain of a step: SURVEY 8(d)'s bytes over the
        # summed time of all its kernels (the profiled steps' HIP events)
        sg_ms = sum(full[k]["ms"] for k in full if k in SCATTER_GATHER_OPS) / max(1, prof_steps)
        sg_bytes = scatter_gather_bytes(cfg.batch_size, cfg.num_points) \
            if args.backbone == "hybrid" else None
        roofline_sg_all = None
        if sg_ms > 0 and sg_bytes:
            ach = sg_bytes / (sg_ms * 1e-3) / 1e9
            roofline_sg_all = {
                "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": ach / HBM_PEAK_GBS, "algorithmic_bytes_per_step": sg_bytes,
                "ms_per_step": sg_ms, "ops": [k for k in SCATTER_GATHER_OPS if k in full],
                "note": "SURVEY 8d bytes of all 6 PVConv voxelize/devoxelize calls, fwd + bwd, "
                        "over the summed HIP-event time of every scatter/gather kernel incl. "
                        "the segment plans"}
        log(f"{ms:.2f} ms/step, {value / 1e6:.3f} M points/s; losses {loss_p:.4f} {loss_z:.4f}")
        cham = None
        extra = {}
        if not args.no_chamfer:
            cham = {"published_shape_32x2000x1000": chamfer_ms(dev, 32, 2000, 1000),
                    "published_fwd_bwd_ms": 1.4,
                    "c2_shape_8x20000x20000": chamfer_ms(dev, 8, 20000, 20000, iters=5),
                    "c5_shape_4x100000x100000": chamfer_ms(dev, 4, 100000, 100000, iters=2)}
            for key, (b_, n_) in (("c2_shape_8x20000x20000", (8, 20000)),
                                  ("c5_shape_4x100000x100000", (4, 100000))):
                fwd = cham[key]["fwd"] * 1e-3
                flops = 8.0 * 2 * b_ * n_ * n_  # 2*B*N*M pairs x 8 FLOP
                culled = n_ * n_ >= 2 ** 31  # ops.chamfer switches to the culled search
                cham[key]["roofline_fwd"] = {
                    "bound": "valu", "achieved": flops / fwd / 1e12, "peak": FP32_VALU_TF,
                    "unit": "TFLOP/s",
                    "frac": None if culled else flops / fwd / 1e12 / FP32_VALU_TF,
                    "pairs_per_s": 2 * b_ * n_ * n_ / fwd,
                    "note": ("culled tile search: most pairs are never evaluated, so the rate is "
                             "the brute-force-equivalent one and no roofline fraction applies"
                             if culled else
                             "wall clock of the op incl. launch; 8 FLOP per pair (SURVEY 8d)")}
            log(f"chamfer: {cham}")
            extra["emd"] = {f"B8_N{n_}": emd_ms(dev, 8, n_) for n_ in (2048, 4096)}
            extra["ball_query"] = {"c2": ball_query_ms(dev, 8, 20000, 2048, 0.1, 32),
                                   "c5": ball_query_ms(dev, 4, 100000, 4096, 0.05, 32)}
            log(f"emd / ball query: {extra}")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline: running one warm-up + one timed CPU step ...")
            cpu = cpu_baseline(args, cfg_kwargs)
            log(f"cpu baseline: {cpu['seconds_per_step']:.2f} s/step")
        metric = METRIC if (cfg.batch_size, cfg.num_points) == (8, 20000) else METRIC.replace(
            "B=8, N=20000", f"B={cfg.batch_size}, N={cfg.num_points}")
        line = {
            "metric": metric, "value": value, "unit": "points/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "vs_h100_derived_upper_bound": value / H100_DERIVED_PTS,
            "dtype": "fp32 ContextNet (scatter/gather ops fp32; Conv3d + 1x1 convs as bf16x3 "
                     "split-operand matrix-core products, fp32 accumulate, ~2^-16 per product vs "
                     "the reference's default cuDNN TF32 2^-11) + bf16 autocast per-point MLP "
                     "head (reference AMP config; its per-cloud B-row layers -- embeddings, "
                     "FiLM affines, latent net, encoder head -- in fp32)",
            "data": "synthetic (randn xyz, U[0,1] rgb, U[0,1] cond; no dataset on the box)",
            "config": {"workload": f"{cfg.pf_backbone} flow-matching train step, "
                                   f"B={cfg.batch_size}/GPU, N={cfg.num_points} xyz+rgb, "
                                   "latent 128, 1 joint, stages (128,256,256)@(32,16,8)",
                       "global_batch": world * cfg.batch_size, "points_per_cloud": cfg.num_points,
                       "backbone": cfg.pf_backbone, "parallelism": f"dp{world}"},
            "roofline": roofline, "roofline_step": step_roofline(cfg, ms),
            "roofline_voxel_scatter_gather": roofline_scatter,
            "roofline_voxel_scatter_gather_all": roofline_sg_all,
            "kernels": kernels, "cpu_baseline": cpu, "chamfer": cham, **extra,
            "loss_point": loss_p, "loss_latent": loss_z,
            "distributed": {"backend": dist.get_backend() if ddp else None,
                            "world_size": dist.get_world_size() if ddp else 1,
                            "NCCL_ALGO": os.environ.get("NCCL_ALGO") if ddp else None},
        }
        print(json.dumps(line), flush=True)
    if ddp:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
