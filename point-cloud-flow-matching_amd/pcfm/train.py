"""Flow-matching train step of the reference (train.py:553-673), data-parallel.

`Trainer.step(batch, epoch)` is one iteration of the reference's inner loop:
encoder -> point-flow FM loss (hybrid PVConv backbone) -> latent FM loss ->
scaled backward (DDP gradient all-reduce over RCCL when world_size > 1) ->
unscale + clip -> AdamW -> EMA -> cosine LR.  Model construction order, loss
terms, mixed-precision regions and optimizer groups follow the reference.

Deliberate, result-preserving differences (all switchable in TrainConfig):
  * `ema_foreach`: the EMA update runs as two torch._foreach ops over the
    state dict instead of a Python loop of ~500 tiny kernels (util.py:16-21);
    per element it is the same mul_ then add_(alpha=1-d).
  * `fused_adamw`: AdamW(fused=True) takes GradScaler's inf check on the
    device instead of the host round trip of GradScaler.step; same update rule.
  * `fused_step` (HIP devices): unscale + clip + AdamW + the parameters' EMA
    update run as three HIP launches (pcfm.optim.FusedAdamWEMA, csrc/optim.hip)
    instead of ~40 multi-tensor launches; same arithmetic, inf check on the
    device as with `fused_adamw`.  The EMA of buffers stays a foreach update.
  * `device_rng`: t ~ Beta(a, 1) is sampled on the device (the reference
    samples on the CPU and copies, train.py:604-605, :639-640); same law.
  * `tunableop`: the autocast Linears use library GEMM algorithms measured on
    MI355X for this step (PyTorch TunableOp, pcfm/data/tunableop_gfx950.csv);
  * `miopen_find`: torch.backends.cudnn.benchmark = True, i.e. MIOpen picks
    each convolution's solver by timing the candidates once per shape.
"""
from __future__ import annotations

import math
import os
import random
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import distributed as dist

from pcfm.dist_env import pin_rccl_env
from pcfm.models import (ConditionalLatentVelocityNet, HybridMLP, ShapeEncoder, VelocityNet)


@dataclass
class TrainConfig:
    # data (README.md:156-170 Scissors run: 20000 pts, bs 8, latent 128, 1 joint)
    batch_size: int = 8
    num_points: int = 20000
    cond_dim: int = 1
    has_rgb: bool = True
    # backbone
    pf_backbone: str = "hybrid"
    latent_dim: int = 128
    enc_width: int = 128
    enc_depth: int = 4
    pf_width: int = 512
    pf_depth: int = 6
    # runtime: MI355X-measured library GEMM choices (pcfm/data/tunableop_gfx950.csv)
    tunableop: bool = True
    pf_emb_dim: int = 256
    cfg_drop_p: float = 0.1
    lf_width: int = 512
    lf_depth: int = 6
    lf_emb_dim: int = 256
    ctx_dim: int = 64
    ctx_emb_dim: int = 256
    ctx_stage_channels: List[int] = field(default_factory=lambda: [128, 256, 256])
    ctx_stage_blocks: List[int] = field(default_factory=lambda: [2, 2, 2])
    ctx_stage_res: List[int] = field(default_factory=lambda: [32, 16, 8])
    ctx_with_se: bool = True
    ctx_norm: str = "group"
    ctx_gn_groups: int = 32
    ctx_with_global: bool = True
    ctx_voxel_normalize: bool = True
    ctx_t_gate_tau: float = 0.8
    ctx_t_gate_k: float = 10.0
    use_rgb_in_latent: bool = True
    pointflow_rgb: bool = True
    # optimisation
    epochs: int = 3000
    steps_per_epoch: int = 293
    lr_enc: float = 3e-4
    lr_pf: float = 3e-4
    lr_lf: float = 3e-4
    min_lr: float = 1e-6
    use_cosine_lr: bool = True
    warmup_steps: int = 1000
    weight_decay: float = 1e-4
    grad_clip_norm: float = 1.0
    t_beta_a: float = 2.0
    geom_warmup_epochs: int = 200
    cfg_drop_warmup_epochs: int = 100
    point_prior_std: float = 1.0
    latent_prior_std: float = 1.0
    color_prior: str = "uniform"
    color_prior_std: float = 1.0
    ema_decay: float = 0.999
    lambda_point: float = 1.0
    lambda_latent: float = 1.0
    lambda_color: float = 1.0
    seed: int = 123
    amp: bool = True
    use_bf16: bool = True
    # result-preserving implementation switches (module docstring)
    ema_foreach: bool = True
    fused_adamw: bool = True
    fused_step: bool = True
    device_rng: bool = True
    film_per_point: bool = False
    # MIOpen exhaustive solver search for every conv shape (cudnn.benchmark):
    # ~94-113 TFLOP/s fp32 on the PVConv Conv3d shapes vs 12-68 TFLOP/s with
    # the default heuristic pick (tools/conv3d_probe.py on MI355X); same math.
    miopen_find: bool = True
    # parity mode: fp32 convolutions on exact fp32 arithmetic instead of the
    # bf16x3 matrix-core kernels (pcfm.precision); process-wide when set
    exact_fp32: bool = False

    @property
    def enc_in_ch(self) -> int:
        return 6 if (self.use_rgb_in_latent and self.has_rgb) else 3

    @property
    def pf_point_dim(self) -> int:
        return 6 if (self.pointflow_rgb and self.has_rgb) else 3


# ---------------------------------------------------------------------------
# util.py equivalents
# ---------------------------------------------------------------------------
def seed_all(seed: int) -> None:
    """util.py:27-32."""
    import numpy as np
    random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)


def cosine_lr(step: int, total: int, base_lr: float, min_lr: float = 1e-6, warmup: int = 0):
    """util.py:113-117: linear warm-up, then cosine decay to min_lr."""
    if step < warmup:
        return min_lr + (base_lr - min_lr) * step / max(1, warmup)
    frac = (step - warmup) / max(1, total - warmup)
    return min_lr + 0.5 * (base_lr - min_lr) * (1 + math.cos(math.pi * frac))


def init_distributed(backend: Optional[str] = None):
    """util.py:71-84: torchrun env -> process group ("nccl" = RCCL on ROCm)."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        rank = int(os.environ["RANK"])
        world = int(os.environ["WORLD_SIZE"])
        local = int(os.environ.get("LOCAL_RANK", 0))
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            pin_rccl_env()  # the all-reduce on RCCL's ring kernels (pcfm/dist_env.py)
            torch.cuda.set_device(local)
        if not dist.is_initialized():
            dist.init_process_group(backend=backend, init_method="env://")
        return True, rank, world, local
    return False, 0, 1, 0


def cleanup_distributed() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


class EMA:
    """Exponential moving average of a state dict (util.py:11-24)."""

    def __init__(self, model: nn.Module, decay: float = 0.999, foreach: bool = True):
        self.decay = float(decay)
        self.foreach = bool(foreach)
        self.shadow = {k: v.detach().clone() for k, v in model.state_dict().items()}
        self._keys = None
        self._lists = None  # (model id, shadow list, live tensor list), built once
        # keys whose update another component performs (the fused parameter
        # update, pcfm.optim): update() leaves them alone
        self.external = frozenset()

    def param_shadows(self, model: nn.Module) -> Dict[torch.Tensor, torch.Tensor]:
        """{parameter: its shadow tensor} for model's parameters."""
        return {p: self.shadow[k] for k, p in model.named_parameters()}

    @torch.no_grad()
    def update(self, model: nn.Module) -> None:
        d = self.decay
        if self.foreach:
            # model.state_dict() per step costs ~1 ms of host time, during which the
            # GPU drains its queue; the live parameter / buffer tensors do not change
            # identity across steps (in-place optimizer updates), so list them once
            if self._lists is None or self._lists[0] != id(model):
                sd = model.state_dict()
                keys = [k for k, v in sd.items()
                        if v.dtype.is_floating_point and k not in self.external]
                self._lists = (id(model), [self.shadow[k] for k in keys],
                               [sd[k].detach() for k in keys])
            _, shadow, cur = self._lists
            if not shadow:
                return
            torch._foreach_mul_(shadow, d)
            torch._foreach_add_(shadow, cur, alpha=1.0 - d)
            return
        sd = model.state_dict()
        if self._keys is None:
            self._keys = [k for k, v in sd.items()
                          if v.dtype.is_floating_point and k not in self.external]
        for k in self._keys:
            self.shadow[k].mul_(d).add_(sd[k].detach(), alpha=1.0 - d)

    def copy_to(self, model: nn.Module) -> None:
        model.load_state_dict(self.shadow, strict=True)


def count_parameters(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


# ---------------------------------------------------------------------------
# models (train.py:201-233)
# ---------------------------------------------------------------------------
def build_models(cfg: TrainConfig, device):
    enc = ShapeEncoder(cfg.latent_dim, width=cfg.enc_width, depth=cfg.enc_depth,
                       in_channels=cfg.enc_in_ch).to(device)
    pf_cond_dim = cfg.latent_dim + cfg.cond_dim
    if cfg.pf_backbone == "mlp":
        pf = VelocityNet(cond_dim=pf_cond_dim, width=cfg.pf_width, depth=cfg.pf_depth,
                         emb_dim=cfg.pf_emb_dim, cfg_dropout_p=cfg.cfg_drop_p,
                         point_dim=cfg.pf_point_dim, film_per_point=cfg.film_per_point)
    else:
        pf = HybridMLP(
            cond_dim=pf_cond_dim, point_dim=cfg.pf_point_dim, ctx_dim=cfg.ctx_dim,
            ctx_emb_dim=cfg.ctx_emb_dim, stage_channels=cfg.ctx_stage_channels,
            stage_blocks=cfg.ctx_stage_blocks, stage_res=cfg.ctx_stage_res,
            with_se=cfg.ctx_with_se, norm_type=cfg.ctx_norm, gn_groups=cfg.ctx_gn_groups,
            with_global=cfg.ctx_with_global, voxel_normalize=cfg.ctx_voxel_normalize,
            use_t_gate=True, t_gate_k=cfg.ctx_t_gate_k, t_gate_tau=cfg.ctx_t_gate_tau,
            pf_width=cfg.pf_width, pf_depth=cfg.pf_depth, pf_emb_dim=cfg.pf_emb_dim,
            cfg_dropout_p=cfg.cfg_drop_p, film_per_point=cfg.film_per_point)
    pf = pf.to(device)
    lf = ConditionalLatentVelocityNet(cfg.latent_dim, cond_dim=0, width=cfg.lf_width,
                                      depth=cfg.lf_depth, emb_dim=cfg.lf_emb_dim).to(device)
    return enc, pf, lf


def synthetic_batch(cfg: TrainConfig, device, generator: Optional[torch.Generator] = None,
                    surface: bool = False) -> Dict[str, torch.Tensor]:
    """A batch in the schema of the PartNet-H5 loader (datasets.py:374-621):
    train_points (B,N,3), train_rgb (B,N,3) in [0,1], cond (B,J).  `surface`
    draws points near the unit sphere (dense voxels) instead of N(0, I)."""
    b, n = cfg.batch_size, cfg.num_points
    kw = dict(device=device, generator=generator)
    pts = torch.randn(b, n, 3, **kw)
    if surface:
        pts = pts / pts.norm(dim=-1, keepdim=True).clamp_min(1e-6)
        pts = pts + 0.01 * torch.randn(b, n, 3, **kw)
    batch = {"train_points": pts, "train_rgb": torch.rand(b, n, 3, **kw)}
    if cfg.cond_dim > 0:
        batch["cond"] = torch.rand(b, cfg.cond_dim, **kw)
    return batch


TUNABLEOP_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data",
                              "tunableop_gfx950.csv")


def enable_tunableop(path: str = TUNABLEOP_FILE, tune: bool = False) -> bool:
    """Library GEMM choice for the autocast Linears (hipBLASLt / rocBLAS) from
    PyTorch TunableOp results measured on MI355X for this train step
    (tools/tune_gemms.sh writes them; tune=True measures unseen shapes).  Shapes
    not in the file, or a file from another library version, keep the default
    algorithm.  Returns False if the file is absent."""
    from torch.cuda import tunable
    if not tune and not os.path.exists(path):
        return False
    tunable.enable(True)
    tunable.tuning_enable(bool(tune))
    tunable.set_filename(path, insert_device_ordinal=False)
    if os.path.exists(path):
        tunable.read_file(path)
    return True


class Trainer:
    """Models + optimizer + one FM training iteration (train.py:553-673)."""

    def __init__(self, cfg: TrainConfig, device, rank: int = 0, world_size: int = 1,
                 ddp: bool = False):
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.type == "cuda" and cfg.miopen_find:
            torch.backends.cudnn.benchmark = True
        if self.device.type == "cuda" and cfg.tunableop:
            out = os.environ.get("PCFM_TUNE_GEMMS")  # tools/tune_gemms.sh: measure, write here
            enable_tunableop(out, tune=True) if out else enable_tunableop()
        if cfg.exact_fp32:
            from pcfm.precision import set_exact_fp32
            set_exact_fp32(True)
        self.rank, self.world_size = rank, world_size
        seed_all(cfg.seed + rank)
        self.enc, self.pf, self.lf = build_models(cfg, self.device)
        self.ema_pf = EMA(self.pf, cfg.ema_decay, foreach=cfg.ema_foreach)
        self.ema_lf = EMA(self.lf, cfg.ema_decay, foreach=cfg.ema_foreach)
        self.model_enc, self.model_pf, self.model_lf = self.enc, self.pf, self.lf
        if ddp:
            from torch.nn.parallel import DistributedDataParallel as DDP
            ids = [self.device.index] if self.device.type == "cuda" else None
            kw = dict(device_ids=ids, output_device=ids[0] if ids else None,
                      broadcast_buffers=False, find_unused_parameters=False)
            self.model_enc = DDP(self.enc, **kw)
            self.model_pf = DDP(self.pf, **kw)
            self.model_lf = DDP(self.lf, **kw)
        groups = [
            {"params": list(self.enc.parameters()), "lr": cfg.lr_enc},
            {"params": list(self.pf.parameters()), "lr": cfg.lr_pf},
            {"params": list(self.lf.parameters()), "lr": cfg.lr_lf},
        ]
        self.fused_step = bool(cfg.fused_step and self.device.type == "cuda")
        if self.fused_step:
            from pcfm.optim import FusedAdamWEMA
            for g in groups:
                g["weight_decay"] = cfg.weight_decay
            shadows = {**self.ema_pf.param_shadows(self.pf), **self.ema_lf.param_shadows(self.lf)}
            self.opt = FusedAdamWEMA(groups, ema_shadows=shadows, ema_decay=cfg.ema_decay)
            self.ema_pf.external = frozenset(k for k, _ in self.pf.named_parameters())
            self.ema_lf.external = frozenset(k for k, _ in self.lf.named_parameters())
        else:
            fused = bool(cfg.fused_adamw and self.device.type == "cuda")
            self.opt = torch.optim.AdamW(groups, weight_decay=cfg.weight_decay, fused=fused)
        self.scaler = torch.amp.GradScaler(self.device.type, enabled=cfg.amp)
        self.total_steps = cfg.epochs * max(1, cfg.steps_per_epoch)
        self.global_step = 0
        self._clip_params = (list(self.enc.parameters()) + list(self.pf.parameters())
                             + list(self.lf.parameters()))
        self._beta = None
        self.last_grad_norm = None  # clip_grad_norm_'s value of the last step

    # -- helpers ------------------------------------------------------------
    def _autocast(self):
        dtype = torch.bfloat16 if self.cfg.use_bf16 else torch.float16
        return torch.amp.autocast(self.device.type if self.device.type == "cuda" else "cpu",
                                  enabled=self.cfg.amp and self.device.type == "cuda", dtype=dtype)

    def _sample_t(self, b: int, dtype) -> torch.Tensor:
        a = self.cfg.t_beta_a
        if self.cfg.device_rng and self.device.type == "cuda":
            if self._beta is None:
                one = torch.ones((), device=self.device)
                self._beta = torch.distributions.Beta(one * a, one)
            return self._beta.sample((b,)).to(dtype=dtype)
        beta = torch.distributions.Beta(concentration1=a, concentration0=1.0)
        return beta.sample((b,)).to(device=self.device, dtype=dtype)

    def _pf_prior(self, data_pf: torch.Tensor) -> torch.Tensor:
        """make_pf_prior_like (train.py:266-279)."""
        b, n, d = data_pf.shape
        cfg = self.cfg
        if d == 3:
            return torch.randn_like(data_pf) * cfg.point_prior_std
        z = data_pf.new_empty(b, n, 6)
        z[..., :3] = torch.randn(b, n, 3, device=data_pf.device,
                                 dtype=data_pf.dtype) * cfg.point_prior_std
        if cfg.color_prior == "gauss":
            z[..., 3:] = torch.randn(b, n, 3, device=data_pf.device,
                                     dtype=data_pf.dtype) * cfg.color_prior_std
        elif cfg.color_prior == "uniform":
            z[..., 3:] = torch.rand(b, n, 3, device=data_pf.device, dtype=data_pf.dtype)
        else:
            z[..., 3:] = 0.0
        return z

    def _pf_prior_from(self, raw: torch.Tensor) -> torch.Tensor:
        """make_pf_prior_like (train.py:266-279) on injected raw draws."""
        cfg = self.cfg
        if raw.shape[-1] == 3:
            return raw * cfg.point_prior_std
        z = torch.empty_like(raw)
        z[..., :3] = raw[..., :3] * cfg.point_prior_std
        if cfg.color_prior == "gauss":
            z[..., 3:] = raw[..., 3:] * cfg.color_prior_std
        elif cfg.color_prior == "uniform":
            z[..., 3:] = raw[..., 3:]
        else:
            z[..., 3:] = 0.0
        return z

    def train_mode(self):
        self.enc.train()
        self.pf.train()
        self.lf.train()

    def _update_params(self) -> None:
        """unscale + clip + AdamW step + scale update + zero_grad (train.py:652-657);
        with `fused_step` also the parameters' EMA update (pcfm.optim)."""
        cfg = self.cfg
        clip = float(cfg.grad_clip_norm) if cfg.grad_clip_norm and cfg.grad_clip_norm > 0 else 0.0
        if self.fused_step:
            self.last_grad_norm = self.opt.step(clip, self.scaler)
        else:
            if clip > 0:
                self.scaler.unscale_(self.opt)
                self.last_grad_norm = torch.nn.utils.clip_grad_norm_(self._clip_params, clip)
            self.scaler.step(self.opt)
            self.scaler.update()
        self.opt.zero_grad(set_to_none=True)

    # -- checkpoint / resume (train.py:681-699 save, :470-520 resume) ---------
    def checkpoint(self, epoch: int) -> Dict:
        """The reference's checkpoint dict: epoch, the three models' state dicts,
        the EMA shadows, args, cond_dim, optimizer (torch AdamW layout) and AMP
        scaler state, global step.  torch.save-able with weights_only loads."""
        cfg = self.cfg
        args = {k: (list(v) if isinstance(v, tuple) else v) for k, v in asdict(cfg).items()}
        args.update(enc_in_channels=cfg.enc_in_ch, pf_point_dim=cfg.pf_point_dim)
        return {
            "epoch": int(epoch),
            "encoder": self.enc.state_dict(),
            "pf": self.pf.state_dict(),
            "lf": self.lf.state_dict(),
            "ema_pf": {k: v.detach().clone() for k, v in self.ema_pf.shadow.items()},
            "ema_lf": {k: v.detach().clone() for k, v in self.ema_lf.shadow.items()},
            "args": args,
            "cond_dim": cfg.cond_dim,
            "opt": self.opt.state_dict(),
            "scaler": self.scaler.state_dict() if cfg.amp else None,
            "global_step": int(self.global_step),
        }

    def load_checkpoint(self, ckpt: Dict) -> int:
        """Resume from a `checkpoint()` dict (or the reference's): encoder strict,
        pf (or the old key "model") and lf non-strict, EMA shadow entries present
        in the file copied in place (the fused update holds these tensors), the
        optimizer and AMP scaler state when present and loadable (otherwise a
        warning, as the reference's auto-resume).  Returns the epoch to run
        next (the saved epoch + 1), as the reference's auto-resume does."""
        if "encoder" in ckpt:
            self.enc.load_state_dict(ckpt["encoder"], strict=True)
        if "pf" in ckpt:
            self.pf.load_state_dict(ckpt["pf"], strict=False)
        elif "model" in ckpt:
            self.pf.load_state_dict(ckpt["model"], strict=False)
        if "lf" in ckpt:
            self.lf.load_state_dict(ckpt["lf"], strict=False)
        with torch.no_grad():
            for ema, key in ((self.ema_pf, "ema_pf"), (self.ema_lf, "ema_lf")):
                src = ckpt.get(key)
                if not isinstance(src, dict):
                    continue
                for k, cur in ema.shadow.items():
                    v = src.get(k)
                    if torch.is_tensor(v) and v.dtype.is_floating_point:
                        if tuple(v.shape) != tuple(cur.shape):
                            raise ValueError(f"load_checkpoint: {key}[{k}] shape "
                                             f"{tuple(v.shape)} != {tuple(cur.shape)}")
                        cur.copy_(v.to(device=cur.device, dtype=cur.dtype))
        # optimizer / AMP scaler: a state that does not fit (groups, betas,
        # shapes) is reported and skipped, the weights, EMA and epoch still
        # resume -- the reference's auto-resume (train.py:498-516)
        key = "opt" if "opt" in ckpt else ("opt_main" if "opt_main" in ckpt else None)
        if key is not None:
            try:
                self.opt.load_state_dict(ckpt[key])
            except Exception as e:  # noqa: BLE001 -- the reference's catch-all
                if self.rank == 0:
                    print(f"[Auto-Resume][WARN] {key} state load failed: {e}")
        if self.cfg.amp and ckpt.get("scaler") is not None:
            try:
                self.scaler.load_state_dict(ckpt["scaler"])
            except Exception as e:  # noqa: BLE001
                if self.rank == 0:
                    print(f"[Auto-Resume][WARN] scaler state load failed: {e}")
        self.global_step = int(ckpt.get("global_step", self.global_step))
        return int(ckpt.get("epoch", 0)) + 1

    # -- one iteration ------------------------------------------------------
    def step(self, batch: Dict[str, torch.Tensor], epoch: int,
             draws: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
        """One iteration.  `draws` injects the step's random numbers instead of
        sampling them (parity tests replay a recorded reference step,
        tests/golden/make_train_golden.py): z_pts (B, N, D) raw prior draws (xyz
        randn | rgb rand), t_pts (B,), drop_u (B,) CFG-drop uniforms, eps_z
        (B, latent) randn, t_z (B,) -- scaled by the configured stds here as the
        reference scales its own draws (train.py:271-276, :595, :617, :637)."""
        out = self.forward_backward(batch, epoch, draws)
        self._update_params()

        self.ema_pf.update(self.pf)
        self.ema_lf.update(self.lf)

        if self.cfg.use_cosine_lr:
            cfg = self.cfg
            for group, base in zip(self.opt.param_groups, (cfg.lr_enc, cfg.lr_pf, cfg.lr_lf)):
                group["lr"] = cosine_lr(self.global_step, self.total_steps, base, cfg.min_lr,
                                        cfg.warmup_steps)
        self.global_step += 1
        return out

    def forward_backward(self, batch: Dict[str, torch.Tensor], epoch: int,
                         draws: Optional[Dict[str, torch.Tensor]] = None
                         ) -> Dict[str, torch.Tensor]:
        """The step up to and including the scaled backward (train.py:553-652):
        afterwards every parameter's .grad holds the loss-scaled gradient -- under
        DDP the all-reduced mean over the ranks -- and nothing is updated yet."""
        cfg = self.cfg
        dev = self.device
        dr = None if draws is None else {k: v.to(dev) for k, v in draws.items()}
        pts = batch["train_points"].to(dev).float()
        rgb = batch.get("train_rgb")
        rgb = rgb.to(dev).float() if rgb is not None else None
        cond_j = batch.get("cond")
        cond_j = cond_j.to(dev).float() if cond_j is not None else None
        use_rgb = (epoch > cfg.geom_warmup_epochs) and cfg.pointflow_rgb and cfg.has_rgb

        # encoder input (train.py:566-578)
        if cfg.enc_in_ch == 6:
            colour = rgb if (rgb is not None and use_rgb) else torch.zeros_like(pts)
            enc_in = torch.cat([pts, colour], dim=-1)
        else:
            enc_in = pts
        with self._autocast():
            z, _ = self.model_enc(enc_in)

        # point-flow FM target (train.py:585-607)
        if cfg.pf_point_dim == 6:
            if rgb is not None and use_rgb:
                data_pf = torch.cat([pts, rgb], dim=-1)
                z_pts = self._pf_prior(data_pf) if dr is None else self._pf_prior_from(dr["z_pts"])
            else:
                data_pf = torch.cat([pts, torch.zeros_like(pts)], dim=-1)
                z_pts = torch.empty_like(data_pf)
                xyz = torch.randn_like(pts) if dr is None else dr["z_pts"][..., :3]
                z_pts[..., :3] = xyz * cfg.point_prior_std
                z_pts[..., 3:] = 0.0
        else:
            data_pf = pts
            z = torch.randn_like(data_pf) if dr is None else dr["z_pts"]
            z_pts = z * cfg.point_prior_std
        b, n, d = data_pf.shape
        t_pts = self._sample_t(b, data_pf.dtype) if dr is None else dr["t_pts"].to(data_pf.dtype)
        x_t = (1.0 - t_pts)[:, None, None] * z_pts + t_pts[:, None, None] * data_pf
        target_v = data_pf - z_pts

        cond_full = z if cond_j is None else torch.cat([z, cond_j], dim=1)
        cond_drop_mask = None
        if cfg.cfg_drop_p > 0.0:
            p_now = cfg.cfg_drop_p * min(1.0, max(0.0, epoch / max(1, cfg.cfg_drop_warmup_epochs)))
            if p_now > 0.0:
                u = torch.rand(b, device=dev) if dr is None else dr["drop_u"]
                cond_drop_mask = (u < p_now).to(data_pf.dtype)[:, None]

        with self._autocast():
            pred_v = self.model_pf(x_t, t_pts, cond_full, cond_drop_mask=cond_drop_mask)
            if d == 6 and not (rgb is not None and use_rgb):
                loss_point = F.mse_loss(pred_v[..., :3], target_v[..., :3])
            elif d == 6:
                loss_point = (F.mse_loss(pred_v[..., :3], target_v[..., :3])
                              + cfg.lambda_color * F.mse_loss(pred_v[..., 3:], target_v[..., 3:]))
            else:
                loss_point = F.mse_loss(pred_v, target_v)

        # latent FM (train.py:636-645)
        z_det = z.detach()
        eps_z = (torch.randn_like(z_det) if dr is None else dr["eps_z"]) * cfg.latent_prior_std
        t_z = self._sample_t(b, z_det.dtype) if dr is None else dr["t_z"].to(z_det.dtype)
        y_t = (1.0 - t_z)[:, None] * eps_z + t_z[:, None] * z_det
        target_v_z = z_det - eps_z
        with self._autocast():
            pred_v_z = self.model_lf(y_t, t_z, cond=None)
            loss_latent = F.mse_loss(pred_v_z, target_v_z)

        loss = cfg.lambda_point * loss_point + cfg.lambda_latent * loss_latent
        self.scaler.scale(loss).backward()
        return {"loss_point": loss_point.detach(), "loss_latent": loss_latent.detach()}
