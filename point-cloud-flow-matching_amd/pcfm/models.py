"""Flow-matching networks of the reference (models.py), on top of the gfx950
PVConv path (modules.PVConv / modules.SharedMLP from this package).

Every class keeps the reference's constructor arguments, parameter names (so
reference checkpoints load with strict=True), module creation order (so a torch
seed gives the same initial weights) and forward arithmetic.  One documented
deviation, switchable per instance: VelocityNetWithContext / VelocityNet apply
each FiLM affine to the per-batch embedding (B, E) and broadcast over points,
where the reference feeds the expanded (B*N, E) copy through the same Linear
(models.py:135, :594).  Row for row it is the same
product; set ``film_per_point=True`` to run the reference's form.

Reference line numbers refer to /root/reference/models.py.
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from modules.norm_act import bn_act, gn_silu, post_gn_film_residual
from modules.pvconv import PVConv
from modules.shared_mlp import PointwiseConv1d, SharedMLP
from pcfm.layers import RowsLinear, fused_trunk, fused_trunk_supported, max_over_points

__all__ = [
    "timestep_embedding", "FiLMBlock", "VelocityNet", "ShapeEncoder",
    "ConditionalLatentVelocityNet", "ContextNet", "VelocityNetWithContext", "HybridMLP",
]


def timestep_embedding(t: torch.Tensor, dim: int, max_period: float = 10000.0) -> torch.Tensor:
    """[cos(t*f_i), sin(t*f_i)], f_i = exp(-ln(max_period) * i / half)  (models.py:22-37)."""
    if dim % 2:
        raise AssertionError("timestep_embedding dim must be even")
    half = dim // 2
    steps = torch.arange(0, half, device=t.device, dtype=t.dtype)
    freqs = torch.exp(-math.log(max_period) * steps / half)
    phase = t.reshape(*t.shape, 1) * freqs
    return torch.cat([torch.cos(phase), torch.sin(phase)], dim=-1)


# Per-cloud layers (B rows: time / condition embeddings, FiLM affines, the latent
# velocity net, the shape encoder's pooled head) in fp32 under bf16 autocast
# instead of bf16: the same results to >= the reference's precision, without
# the ~100 tiny cast launches per train step autocast spends on them.
# PCFM_BATCH_FP32=0 restores autocast's bf16 for them.
_BATCH_FP32 = os.environ.get("PCFM_BATCH_FP32", "1") != "0"
# ContextNet's PV-block FiLM affines as batched products (A/B knob, dev)
_FILM_GROUPS = os.environ.get("PCFM_FILM_GROUPS", "1") != "0"


def _batch_fp32(ref: torch.Tensor):
    """autocast off for a per-cloud layer when it would run in bf16 on the GPU."""
    on = (_BATCH_FP32 and ref.is_cuda and torch.is_autocast_enabled("cuda")
          and torch.get_autocast_dtype("cuda") == torch.bfloat16)
    return torch.autocast("cuda", enabled=False) if on else contextlib.nullcontext(), on


def _kaiming_relu_(linear: nn.Module) -> None:
    nn.init.kaiming_normal_(linear.weight, nonlinearity="relu")
    if linear.bias is not None:
        nn.init.zeros_(linear.bias)


def _small_normal_(linear: nn.Linear) -> None:
    nn.init.normal_(linear.weight, std=0.02)
    nn.init.zeros_(linear.bias)


class _TimeCondEmbed(nn.Module):
    """emb = SiLU(t_proj(sinusoid(t))) + SiLU(c_proj(cond)), shared by the nets."""

    def _embed_t(self, t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
        if t.dim() == 1:
            t = t[:, None]
        ctx, fp32 = _batch_fp32(t)
        with ctx:
            e = timestep_embedding(t.squeeze(-1), self.emb_dim).to(torch.float32 if fp32 else dtype)
            return F.silu(self.t_proj(e))


class FiLMBlock(nn.Module):
    """LayerNorm then (1 + gamma) * h + beta, gamma/beta from the embedding (models.py:62-79)."""

    def __init__(self, width: int, emb_dim: int):
        super().__init__()
        self.norm = nn.LayerNorm(width)
        self.affine = nn.Linear(emb_dim, width * 2)
        nn.init.zeros_(self.affine.bias)

    def forward(self, h: torch.Tensor, emb: torch.Tensor) -> torch.Tensor:
        """h (R, W); emb (R, E) -- or (B, E) with R = B*N, broadcast per batch."""
        y = self.norm(h)
        scale, shift = self.affine(emb).chunk(2, dim=-1)
        if emb.shape[0] != h.shape[0]:
            b = emb.shape[0]
            y = y.view(b, -1, y.shape[-1])
            out = y * (1.0 + scale[:, None, :]) + shift[:, None, :]
            return out.view(h.shape[0], -1)
        return y * (1.0 + scale) + shift


class _PointTrunk(_TimeCondEmbed):
    """input Linear -> (FiLM, residual SiLU+Linear) x (depth-1) -> SiLU+Linear."""

    def _build_trunk(self, in_dim: int, width: int, depth: int, emb_dim: int, out_dim: int):
        self.input = RowsLinear(in_dim, width)
        self.blocks = nn.ModuleList([nn.Sequential(nn.SiLU(), RowsLinear(width, width))
                                     for _ in range(depth - 1)])
        self.films = nn.ModuleList([FiLMBlock(width, emb_dim) for _ in range(depth - 1)])
        self.out = nn.Sequential(nn.SiLU(), RowsLinear(width, out_dim))
        _kaiming_relu_(self.input)
        for seq in self.blocks:
            _kaiming_relu_(seq[1])
        nn.init.zeros_(self.out[1].bias)

    def _cond_embed(self, ref: torch.Tensor, cond: Optional[torch.Tensor],
                    cond_drop_mask: Optional[torch.Tensor]) -> torch.Tensor:
        if self.cond_dim > 0 and cond is not None:
            c_in = cond if cond_drop_mask is None else cond * (1.0 - cond_drop_mask)
        else:
            c_in = ref.new_zeros((ref.shape[0], self.cond_dim if self.cond_dim > 0 else 1))
        ctx, fp32 = _batch_fp32(ref)
        with ctx:
            return F.silu(self.c_proj(c_in.float() if fp32 else c_in))

    # the gfx950 fused trunk (pcfm/layers.py) under bf16 autocast; False = torch ops
    fused = True

    def _run_trunk(self, h: torch.Tensor, emb: torch.Tensor, n: int) -> torch.Tensor:
        """The trunk on input cat([h, emb broadcast over the n points]); h is the
        (B*n, k) per-point part (models.py:135, 594 build the concat)."""
        if self.fused and fused_trunk_supported(self, h, emb, n):
            return fused_trunk(self, h, emb, n)
        b = emb.shape[0]
        h = torch.cat([h.reshape(b, n, -1), emb[:, None, :].expand(b, n, -1).to(h.dtype)],
                      dim=-1).reshape(b * n, -1)
        if self.film_per_point:
            film_emb = emb[:, None, :].expand(emb.shape[0], n, -1).reshape(-1, emb.shape[-1])
        else:
            film_emb = emb
        h = self.input(h)
        for blk, film in zip(self.blocks, self.films):
            h = film(h, film_emb)
            h = h + blk(h)
        return self.out(h)


class VelocityNet(_PointTrunk):
    """Per-point MLP velocity v(x, t, cond) -- the `mlp` backbone (models.py:82-153)."""

    def __init__(self, cond_dim: int, width: int = 512, depth: int = 6, emb_dim: int = 256,
                 cfg_dropout_p: float = 0.1, point_dim: int = 3, film_per_point: bool = False):
        super().__init__()
        self.cond_dim = int(cond_dim)
        self.emb_dim = int(emb_dim)
        self.cfg_dropout_p = float(cfg_dropout_p)
        self.point_dim = int(point_dim)
        self.film_per_point = bool(film_per_point)
        self.t_proj = nn.Linear(emb_dim, emb_dim)
        self.c_proj = nn.Linear(cond_dim if cond_dim > 0 else 1, emb_dim)
        _small_normal_(self.t_proj)
        _small_normal_(self.c_proj)
        self._build_trunk(self.point_dim + emb_dim, width, depth, emb_dim, self.point_dim)

    def forward(self, x, t, cond, cond_drop_mask=None):
        b, n, d = x.shape
        assert d == self.point_dim, f"VelocityNet expected point_dim={self.point_dim}, got {d}"
        emb = self._embed_t(t, x.dtype) + self._cond_embed(x, cond, cond_drop_mask)
        return self._run_trunk(x.reshape(b * n, -1), emb, n).reshape(b, n, self.point_dim)

    @torch.no_grad()
    def guided_velocity(self, x, t, cond, guidance_scale: float = 0.0):
        if guidance_scale <= 0.0 or cond is None or self.cond_dim == 0:
            return self.forward(x, t, cond, cond_drop_mask=None)
        v_c = self.forward(x, t, cond, cond_drop_mask=None)
        drop_all = torch.ones((x.shape[0], 1), device=x.device, dtype=x.dtype)
        v_u = self.forward(x, t, cond, cond_drop_mask=drop_all)
        return v_c + guidance_scale * (v_c - v_u)


class ShapeEncoder(nn.Module):
    """PointNet-lite: per-point MLP, max-pool, head -> z (models.py:156-187)."""

    def __init__(self, latent_dim: int = 256, width: int = 128, depth: int = 4,
                 in_channels: int = 3):
        super().__init__()
        self.latent_dim = int(latent_dim)
        self.in_channels = int(in_channels)
        w = width
        self.mlp = nn.Sequential(RowsLinear(self.in_channels, w), nn.SiLU(), RowsLinear(w, w),
                                 nn.SiLU(), RowsLinear(w, w), nn.SiLU())
        head: List[nn.Module] = []
        for _ in range(max(1, depth - 3)):
            head += [nn.Linear(w, w), nn.SiLU()]
        head.append(nn.Linear(w, latent_dim))
        self.head = nn.Sequential(*head)
        for mod in list(self.mlp) + list(self.head):
            if isinstance(mod, nn.Linear):
                _kaiming_relu_(mod)

    def forward(self, pts_or_feats: torch.Tensor):
        h = self.mlp(pts_or_feats)
        pooled = max_over_points(h)
        ctx, fp32 = _batch_fp32(pooled)
        with ctx:
            z = self.head(pooled.float() if fp32 else pooled)
        # z leaves in autocast's dtype, as the reference's autocast Linear returns
        # it: the latent FM draws, interpolants and targets (train.py:636-641) and
        # the point flow's condition then carry the reference's bf16 rounding
        return (z.to(torch.bfloat16) if fp32 else z), h


class ConditionalLatentVelocityNet(_TimeCondEmbed):
    """v(y, t, cond) in latent space (models.py:224-290)."""

    def __init__(self, latent_dim: int, cond_dim: int, width: int = 512, depth: int = 6,
                 emb_dim: int = 256):
        super().__init__()
        self.latent_dim = int(latent_dim)
        self.cond_dim = int(cond_dim)
        self.emb_dim = int(emb_dim)
        self.t_proj = nn.Linear(emb_dim, emb_dim)
        self.c_proj = nn.Linear(cond_dim if cond_dim > 0 else 1, emb_dim)
        _small_normal_(self.t_proj)
        _small_normal_(self.c_proj)
        self.input = nn.Linear(latent_dim + emb_dim, width)
        self.blocks = nn.ModuleList([nn.Sequential(nn.SiLU(), nn.Linear(width, width))
                                     for _ in range(depth - 1)])
        self.out = nn.Sequential(nn.SiLU(), nn.Linear(width, latent_dim))
        _kaiming_relu_(self.input)
        for seq in self.blocks:
            _kaiming_relu_(seq[1])
        nn.init.zeros_(self.out[1].bias)

    def forward(self, y, t, cond, cond_drop_p: float = 0.0):
        ctx, fp32 = _batch_fp32(y)
        if fp32:  # the whole net acts on B rows; its output in autocast's dtype
            with ctx:
                v = self._forward(y.float(), t, None if cond is None else cond.float(),
                                  cond_drop_p)
            return v.to(torch.bfloat16)
        return self._forward(y, t, cond, cond_drop_p)

    def _forward(self, y, t, cond, cond_drop_p: float = 0.0):
        t_emb = self._embed_t(t, y.dtype)
        if self.cond_dim > 0 and cond is not None:
            if cond_drop_p > 0.0:
                keep = (torch.rand(y.shape[0], 1, device=y.device, dtype=y.dtype)
                        < cond_drop_p).to(y.dtype)
                cond = cond * (1.0 - keep)
            c_in = cond
        else:
            c_in = y.new_zeros((y.shape[0], self.cond_dim if self.cond_dim > 0 else 1))
        emb = t_emb + F.silu(self.c_proj(c_in))
        h = self.input(torch.cat([y, emb], dim=-1))
        for blk in self.blocks:
            h = h + blk(h)
        return self.out(h)

    @torch.no_grad()
    def euler_sample(self, y0, cond, steps: int = 50, guidance_scale: float = 0.0):
        y, dt = y0, 1.0 / steps
        for i in range(steps):
            t = y.new_full((y.shape[0],), (i + 0.5) * dt)
            v = self.forward(y, t, cond, cond_drop_p=0.0)
            if guidance_scale > 0.0 and self.cond_dim > 0 and cond is not None:
                v_u = self.forward(y, t, None, cond_drop_p=1.0)
                v = v + guidance_scale * (v - v_u)
            y = y + v * dt
        return y


# ---------------------------------------------------------------------------
# Hybrid backbone: PVConv context pyramid + per-point head (models.py:297-694)
# ---------------------------------------------------------------------------
def _choose_gn_groups(channels: int, prefer: int = 32) -> int:
    g = math.gcd(channels, min(prefer, channels)) or 1
    if g == 1 and channels >= 16:
        for cand in (32, 16, 8, 4, 2):
            if channels % cand == 0:
                return cand
    return max(g, 1)


def _make_norm(norm_type: str, channels: int, gn_groups: int) -> nn.Module:
    if norm_type == "group":
        return nn.GroupNorm(_choose_gn_groups(channels, gn_groups), channels)
    if norm_type in ("batch", "syncbn"):  # the reference maps syncbn to plain BN (models.py:316)
        return nn.BatchNorm1d(channels)
    return nn.Identity()


class _FiLM1d(nn.Module):
    """Norm over (B, C, N) then (1 + gamma) * y + beta, zero-initialised (models.py:322-346)."""

    def __init__(self, channels: int, emb_dim: int, norm_type: str = "group",
                 gn_groups: int = 32, one_plus: bool = True):
        super().__init__()
        self.norm = _make_norm(norm_type, channels, gn_groups)
        self.affine = nn.Linear(emb_dim, channels * 2)
        self.one_plus = bool(one_plus)
        nn.init.zeros_(self.affine.weight)
        nn.init.zeros_(self.affine.bias)

    def forward(self, x: torch.Tensor, emb: torch.Tensor) -> torch.Tensor:
        b, c, _ = x.shape
        y = self.norm(x)
        gamma, beta = self.affine(emb.to(y.dtype)).chunk(2, dim=-1)
        gamma, beta = gamma.view(b, c, 1), beta.view(b, c, 1)
        return y * (1.0 + gamma) + beta if self.one_plus else y * gamma + beta


class _PVBlock(nn.Module):
    """PVConv -> SharedMLP -> residual FiLM (models.py:349-368)."""

    def __init__(self, channels: int, resolution: int, emb_dim: int, with_se: bool,
                 norm_type: str = "group", gn_groups: int = 32, voxel_normalize: bool = True,
                 eps: float = 1e-6):
        super().__init__()
        self.pvconv = PVConv(channels, channels, kernel_size=3, resolution=int(resolution),
                             with_se=bool(with_se), normalize=bool(voxel_normalize), eps=eps)
        self.post = SharedMLP(channels, [channels])
        self.film = _FiLM1d(channels, emb_dim, norm_type=norm_type, gn_groups=gn_groups,
                            one_plus=True)

    def forward(self, feat_coords: Tuple[torch.Tensor, torch.Tensor], emb: torch.Tensor,
                gb: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
        """gb: this block's (gamma, beta) = film.affine(emb) precomputed by
        ContextNet with the other blocks' in one batched product."""
        f, c = self.pvconv(feat_coords)
        film = self.film
        if film.one_plus and isinstance(film.norm, nn.GroupNorm):
            # f + GroupNorm(f) * (1 + gamma) + beta with f = post(.) as one fused op
            # (modules/norm_act.py: the post activation is never written)
            gamma, beta = gb if gb is not None else film.affine(emb.to(f.dtype)).chunk(2, dim=-1)
            return post_gn_film_residual(self.post, film.norm, f, gamma, beta), c
        f = self.post(f)
        return f + film(f, emb), c


class _PVStage(nn.Module):
    """1x1 channel lift, then k PV blocks at one voxel resolution (models.py:371-389)."""

    def __init__(self, in_c: int, out_c: int, num_blocks: int, resolution: int, emb_dim: int,
                 with_se: bool, norm_type: str = "group", gn_groups: int = 32,
                 voxel_normalize: bool = True):
        super().__init__()
        self.proj = SharedMLP(in_c, [out_c])
        self.blocks = nn.ModuleList([
            _PVBlock(out_c, resolution, emb_dim, with_se, norm_type=norm_type,
                     gn_groups=gn_groups, voxel_normalize=voxel_normalize)
            for _ in range(int(num_blocks))])

    def forward(self, feat: torch.Tensor, coords: torch.Tensor, emb: torch.Tensor, gbs=None):
        f, c = self.proj((feat, coords))
        return self.run_blocks(f, c, emb, gbs)

    def run_blocks(self, f: torch.Tensor, c: torch.Tensor, emb: torch.Tensor, gbs=None):
        for i, blk in enumerate(self.blocks):
            f, c = blk((f, c), emb, None if gbs is None else gbs[i])
        return f, c


class _PointwiseParts(torch.autograd.Function):
    """y = W cat(xs, 1) + bias[b] on the segmented bf16x3 GEMMs (ops.pointwise_*_parts)."""

    @staticmethod
    def forward(ctx, weight, bias_b, *xs):
        from pcfm import ops
        ctx.save_for_backward(weight, *xs)
        return ops.pointwise_forward_parts(xs, weight, bias_b.contiguous(), bias_per_batch=True)

    @staticmethod
    def backward(ctx, gy):
        from pcfm import ops
        weight, *xs = ctx.saved_tensors
        gy = gy.contiguous()
        gw = gb = None
        gxs = [None] * len(xs)
        if any(ctx.needs_input_grad[2:]):
            gxs = ops.pointwise_backward_data_parts(gy, weight, [int(x.shape[1]) for x in xs])
        if ctx.needs_input_grad[0]:
            gw = ops.pointwise_backward_weight_parts(xs, gy)
        if ctx.needs_input_grad[1]:
            bb, cc, nn_ = gy.shape
            gb = ops.rows_dot(gy.view(bb * cc, nn_), None, 1.0).view(bb, cc)
        return (gw, gb, *gxs)


class _MaxTee(torch.autograd.Function):
    """(f, max of f over the points) with f passed through: f's gradient from
    its other consumer gets the max's gradient added at the argmax in place, a
    (B, C) scatter, instead of torch's dense zero-filled max gradient and the
    autograd add of two (B, C, N) gradients (models.py:523-524 global_mlp).

    The add is in place only when the caller passes `exclusive_grad=True`,
    asserting that f's other consumer returns a freshly allocated gradient
    that nothing else holds (`_PointwiseParts`, whose backward allocates every
    input gradient); otherwise the incoming gradient is cloned first."""

    @staticmethod
    def forward(ctx, f, exclusive_grad=False):
        m, idx = f.max(dim=-1)
        ctx.save_for_backward(idx)
        ctx.shape = f.shape
        ctx.exclusive = bool(exclusive_grad)
        return f.view_as(f), m

    @staticmethod
    def backward(ctx, df, dm):
        (idx,) = ctx.saved_tensors
        if dm is None:
            return df, None
        if df is None:
            df = dm.new_zeros(ctx.shape)
        elif ctx.exclusive and df.is_contiguous():
            pass  # the consumer's own fresh tensor: add in place
        else:
            df = df.clone(memory_format=torch.contiguous_format)
        return df.scatter_add_(2, idx.unsqueeze(-1), dm.unsqueeze(-1)), None


class _TGate(torch.autograd.Function):
    """ctx (B, N, C) = a[b] * head (B, C, N)^T + (1 - a[b]) * glb[b] (models.py:533-541);
    the gate a depends on t only (no gradient)."""

    @staticmethod
    def forward(ctx, head, glb, alpha):
        from pcfm import ops
        alpha = alpha.contiguous()
        ctx.save_for_backward(alpha)
        return ops.tgate_forward(head.contiguous(), glb.contiguous(), alpha)

    @staticmethod
    def backward(ctx, dout):
        from pcfm import ops
        (alpha,) = ctx.saved_tensors
        dout = dout.contiguous()
        dhead = ops.tgate_backward(dout, alpha) if ctx.needs_input_grad[0] else None
        dglb = None
        if ctx.needs_input_grad[1]:
            s = ops.rows_colsum(dout) if ops.colsum_ok(dout) else dout.sum(dim=1)
            dglb = (1.0 - alpha)[:, None] * s
        return dhead, dglb, None


class ContextNet(_TimeCondEmbed):
    """Multi-resolution PVConv pyramid -> per-point context (B, N, ctx_dim), blended with a
    (t, cond)-only context by a sigmoid gate in t (models.py:392-543)."""

    def __init__(self, in_point_dim: int, cond_dim: int, emb_dim: int = 256, ctx_dim: int = 64,
                 stage_channels: Sequence[int] = (128, 256, 256),
                 stage_blocks: Sequence[int] = (2, 2, 2),
                 stage_res: Sequence[int] = (32, 16, 8), with_se: bool = True,
                 norm_type: str = "group", gn_groups: int = 32, with_global: bool = True,
                 voxel_normalize: bool = True, use_t_gate: bool = True, t_gate_k: float = 10.0,
                 t_gate_tau: float = 0.4):
        super().__init__()
        assert len(stage_channels) == len(stage_blocks) == len(stage_res)
        self.in_point_dim = int(in_point_dim)
        self.emb_dim = int(emb_dim)
        self.ctx_dim = int(ctx_dim)
        self.with_global = bool(with_global)
        self.use_t_gate = bool(use_t_gate)
        self.t_gate_k = float(t_gate_k)
        self.t_gate_tau = float(t_gate_tau)
        self.use_xyz = True
        self.use_rgb = self.in_point_dim == 6

        self.t_proj = nn.Linear(emb_dim, emb_dim)
        self.c_proj = nn.Linear(cond_dim if cond_dim > 0 else 1, emb_dim)
        _small_normal_(self.t_proj)
        _small_normal_(self.c_proj)

        widths = [emb_dim + (3 if self.use_xyz else 0) + (3 if self.use_rgb else 0)]
        widths += list(stage_channels)
        self.stages = nn.ModuleList([
            _PVStage(widths[i], widths[i + 1], nb, rs, emb_dim, with_se, norm_type=norm_type,
                     gn_groups=gn_groups, voxel_normalize=voxel_normalize)
            for i, (nb, rs) in enumerate(zip(stage_blocks, stage_res))])

        c_last = stage_channels[-1]
        if self.with_global:
            self.global_mlp = nn.Sequential(nn.Linear(c_last, c_last), nn.SiLU(),
                                            nn.Linear(c_last, c_last))
            _kaiming_relu_(self.global_mlp[0])
            _kaiming_relu_(self.global_mlp[2])

        self.stage_channels = list(stage_channels)
        head_in = sum(self.stage_channels) + (c_last if self.with_global else 0)
        self.head_pre = PointwiseConv1d(head_in, c_last, 1, bias=True)
        self.head_norm = _make_norm(norm_type, c_last, gn_groups)
        self.head_act = nn.SiLU()
        self.head_out = PointwiseConv1d(c_last, ctx_dim, 1, bias=True)
        _kaiming_relu_(self.head_pre)
        nn.init.zeros_(self.head_out.weight)
        nn.init.zeros_(self.head_out.bias)
        self.norm_type = norm_type
        self.gn_groups = int(gn_groups)
        self.ctx_from_emb = nn.Sequential(nn.Linear(self.emb_dim, self.ctx_dim))
        _kaiming_relu_(self.ctx_from_emb[0])

    def _c_emb(self, x: torch.Tensor, cond: Optional[torch.Tensor]) -> torch.Tensor:
        c_in = x.new_zeros((x.shape[0], 1)) if cond is None or cond.numel() == 0 else cond
        ctx, fp32 = _batch_fp32(x)
        with ctx:
            return F.silu(self.c_proj(c_in.float() if fp32 else c_in))

    def _stem_proj(self, pts: List[torch.Tensor], emb32: torch.Tensor, coords: torch.Tensor):
        """Stage 1's 1x1 lift of the stem cat([emb broadcast, xyz, rgb]) (models.py:
        431-441) without building the stem: the embedding columns of the conv act on
        a per-cloud constant, so W_emb emb + b is a per-cloud bias and the GEMM runs
        over the 3 or 6 point channels only; then its BatchNorm + ReLU.  None when
        the layer is not on the bf16x3 path (the caller builds the stem)."""
        proj = self.stages[0].proj
        conv, bn = proj.layers[0], proj.layers[1]
        if not (pts and isinstance(conv, PointwiseConv1d) and conv.bias is not None
                and conv.x3_ok(coords) and isinstance(proj.layers[2], nn.ReLU)):
            return None
        e = self.emb_dim
        w = conv.weight[:, :, 0]
        bias_b = torch.addmm(conv.bias, emb32, w[:, :e].t())
        pts = torch.cat(pts, dim=1).float() if len(pts) > 1 else pts[0].float().contiguous()
        pre = _PointwiseParts.apply(w[:, e:], bias_b, pts)
        return bn_act(pre, bn, 0.0)

    def _block_films(self, emb32: torch.Tensor):
        """Every PV block's FiLM (gamma, beta) = affine(emb) (models.py:322-346),
        the blocks of equal width as one batched product (nb*2, B, C) -- each
        gamma / beta a contiguous (B, C) slice -- instead of one Linear, two
        copies and their backward per block.  None per stage when a block's FiLM
        is not the fused GroupNorm form (the block then runs its own affine)."""
        if not (emb32.is_cuda and _FILM_GROUPS):
            return [None] * len(self.stages)
        films = [(si, bi, blk.film) for si, st in enumerate(self.stages)
                 for bi, blk in enumerate(st.blocks)]
        if not all(f.one_plus and isinstance(f.norm, nn.GroupNorm) for _, _, f in films):
            return [None] * len(self.stages)
        out = [[None] * len(st.blocks) for st in self.stages]
        by_c: dict = {}
        for si, bi, f in films:
            by_c.setdefault(f.affine.out_features, []).append((si, bi, f))
        for oc, group in by_c.items():
            c = oc // 2
            aw = torch.stack([f.affine.weight for _, _, f in group])  # (g, 2C, E)
            ab = torch.stack([f.affine.bias for _, _, f in group])    # (g, 2C)
            ng = len(group)
            wt = aw.view(ng * 2, c, -1).transpose(1, 2)                 # (2g, E, C)
            gb = torch.baddbmm(ab.view(ng * 2, 1, c), emb32.expand(ng * 2, -1, -1), wt)
            parts = gb.unbind(0)  # one autograd node: its backward stacks the grads
            for j, (si, bi, _) in enumerate(group):
                out[si][bi] = (parts[2 * j], parts[2 * j + 1])
        return out

    def _head_pre_segmented(self, scales: List[torch.Tensor]) -> bool:
        """Whether _head_pre runs as one _PointwiseParts node over the scales."""
        widths = [int(s.shape[1]) for s in scales]
        return bool(self.head_pre.x3_ok(scales[-1]) and len(scales) <= 4
                    and self.head_pre.bias is not None
                    and all(w % 128 == 0 for w in widths[:-1]))

    def _head_pre(self, scales: List[torch.Tensor], g: Optional[torch.Tensor]) -> torch.Tensor:
        """head_pre(cat(scales | g broadcast over points)) (models.py:460-466).

        On the bf16x3 path the concat is never built: the segmented GEMM reads
        the stage outputs in place, and the global feature's columns of the
        weight collapse to a per-cloud bias W_g g + b (the broadcast columns
        are constant along the points)."""
        pre = self.head_pre
        if self._head_pre_segmented(scales):
            widths = [int(s.shape[1]) for s in scales]
            w = pre.weight[:, :, 0]
            cs = sum(widths)
            if g is not None:
                bias_b = torch.addmm(pre.bias, g, w[:, cs:].t())
            else:
                bias_b = pre.bias.expand(scales[0].shape[0], -1)
            return _PointwiseParts.apply(w[:, :cs], bias_b, *scales)
        if g is not None:
            scales = scales + [g[:, :, None].expand_as(scales[-1])]
        return pre(torch.cat(scales, dim=1))

    def forward(self, x: torch.Tensor, t: torch.Tensor, cond: Optional[torch.Tensor]):
        b, n, d = x.shape
        coords = x[..., :3].permute(0, 2, 1).contiguous()
        emb = self._embed_t(t, x.dtype) + self._c_emb(x, cond)
        pts = []
        if self.use_xyz:
            pts.append(coords)
        if self.use_rgb and d == 6:
            pts.append(x[..., 3:].permute(0, 2, 1).contiguous())

        with torch.amp.autocast("cuda", enabled=False):  # the pyramid runs in fp32
            c = coords.float()
            emb32 = emb.float()
            scales = []
            gbs = self._block_films(emb32)
            f = self._stem_proj(pts, emb32, c)
            if f is None:  # stem = cat([emb broadcast over the points, xyz, rgb])
                stem = torch.cat([emb[:, :, None].expand(b, self.emb_dim, n)] + pts, dim=1)
                f, c = self.stages[0](stem.float(), c, emb32, gbs[0])
            else:
                f, c = self.stages[0].run_blocks(f, c, emb32, gbs[0])
            scales.append(f)
            for stage, gb in zip(self.stages[1:], gbs[1:]):
                f, c = stage(f, c, emb32, gb)
                scales.append(f)
            g = None
            if self.with_global:
                if f.is_cuda and f.requires_grad:
                    # in place only when f's other consumer is _head_pre's
                    # _PointwiseParts, whose backward returns fresh gradients
                    f, fmax = _MaxTee.apply(f, self._head_pre_segmented(scales))
                    scales[-1] = f
                else:
                    fmax = f.max(dim=-1).values
                g = self.global_mlp(fmax)
            pre = self._head_pre(scales, g)
            if isinstance(self.head_norm, nn.GroupNorm) and isinstance(self.head_act, nn.SiLU):
                h = gn_silu(pre, self.head_norm)  # one fused pass pair on the GPU
            else:
                h = self.head_act(self.head_norm(pre))
            ctx = self.head_out(h)
            if self.use_t_gate:
                glb = self.ctx_from_emb(emb32)
                alpha = torch.sigmoid(self.t_gate_k * (t.view(b, 1, 1).float() - self.t_gate_tau))
                if ctx.is_cuda and ctx.dtype == torch.float32 and glb.dtype == torch.float32:
                    # blend + permute in one pass (csrc/head.hip tgate)
                    ctx = _TGate.apply(ctx, glb, alpha.reshape(b).detach())
                else:
                    ctx = alpha * ctx.permute(0, 2, 1) + (1.0 - alpha) * glb[:, None, :].expand(
                        b, n, -1)
            else:
                ctx = ctx.permute(0, 2, 1)
        return ctx.to(x.dtype)


class VelocityNetWithContext(_PointTrunk):
    """[x | ctx | emb] -> v per point, FiLM-modulated (models.py:546-601)."""

    def __init__(self, cond_dim: int, point_dim: int = 3, ctx_dim: int = 64, width: int = 512,
                 depth: int = 6, emb_dim: int = 256, cfg_dropout_p: float = 0.1,
                 film_per_point: bool = False):
        super().__init__()
        self.cond_dim, self.point_dim = int(cond_dim), int(point_dim)
        self.emb_dim, self.ctx_dim = int(emb_dim), int(ctx_dim)
        self.cfg_dropout_p = float(cfg_dropout_p)
        self.film_per_point = bool(film_per_point)
        self.t_proj = nn.Linear(emb_dim, emb_dim)
        self.c_proj = nn.Linear(cond_dim if cond_dim > 0 else 1, emb_dim)
        _small_normal_(self.t_proj)
        _small_normal_(self.c_proj)
        self._build_trunk(self.point_dim + self.ctx_dim + emb_dim, width, depth, emb_dim,
                          self.point_dim)

    def forward(self, x, t, cond, ctx, cond_drop_mask=None):
        b, n, _ = x.shape
        assert ctx.shape[:2] == (b, n), f"ctx shape mismatch: {tuple(ctx.shape)} vs {(b, n, '*')}"
        emb = self._embed_t(t, x.dtype) + self._cond_embed(x, cond, cond_drop_mask)
        h = torch.cat([x, ctx.to(x.dtype)], dim=-1).reshape(b * n, -1)
        return self._run_trunk(h, emb, n).reshape(b, n, self.point_dim)


class HybridMLP(nn.Module):
    """ContextNet + VelocityNetWithContext: the `hybrid` point-flow backbone (models.py:604-694)."""

    def __init__(self, cond_dim: int, point_dim: int = 3, ctx_dim: int = 64,
                 ctx_emb_dim: int = 256, stage_channels: Sequence[int] = (128, 256, 256),
                 stage_blocks: Sequence[int] = (2, 2, 2), stage_res: Sequence[int] = (32, 16, 8),
                 with_se: bool = True, norm_type: str = "group", gn_groups: int = 32,
                 with_global: bool = True, voxel_normalize: bool = True, use_t_gate: bool = True,
                 t_gate_k: float = 10.0, t_gate_tau: float = 0.8, pf_width: int = 512,
                 pf_depth: int = 6, pf_emb_dim: int = 256, cfg_dropout_p: float = 0.1,
                 film_per_point: bool = False):
        super().__init__()
        self.cond_dim = int(cond_dim)
        self.point_dim = int(point_dim)
        self.ctx_net = ContextNet(
            in_point_dim=point_dim, cond_dim=cond_dim, emb_dim=ctx_emb_dim, ctx_dim=ctx_dim,
            stage_channels=list(stage_channels), stage_blocks=list(stage_blocks),
            stage_res=list(stage_res), with_se=with_se, norm_type=norm_type,
            gn_groups=gn_groups, with_global=with_global, voxel_normalize=voxel_normalize,
            use_t_gate=use_t_gate, t_gate_k=t_gate_k, t_gate_tau=t_gate_tau)
        self.head = VelocityNetWithContext(
            cond_dim=cond_dim, point_dim=point_dim, ctx_dim=ctx_dim, width=pf_width,
            depth=pf_depth, emb_dim=pf_emb_dim, cfg_dropout_p=cfg_dropout_p,
            film_per_point=film_per_point)

    @staticmethod
    def _cond_eff(cond, mask, x):
        if cond is None:
            return x.new_zeros((x.shape[0], 1))
        return cond if mask is None else cond * (1.0 - mask.to(cond.dtype))

    def set_bn_eval(self, freeze: bool = True):
        """Freeze / unfreeze every BatchNorm (models.py:663-673)."""
        for mod in self.modules():
            if isinstance(mod, (nn.BatchNorm1d, nn.BatchNorm2d, nn.SyncBatchNorm)):
                mod.train(not freeze)
                mod.track_running_stats = True
                mod.momentum = 0.0 if freeze else 0.1

    def forward(self, x, t, cond, cond_drop_mask=None):
        ctx_cond = self._cond_eff(cond, cond_drop_mask, x) if self.cond_dim > 0 else None
        ctx = self.ctx_net(x, t, ctx_cond)
        return self.head(x, t, cond, ctx, cond_drop_mask=cond_drop_mask)

    @torch.no_grad()
    def guided_velocity(self, x, t, cond, guidance_scale: float = 0.0):
        if guidance_scale <= 0.0 or self.cond_dim == 0 or cond is None:
            return self.forward(x, t, cond, cond_drop_mask=None)
        v_c = self.forward(x, t, cond, cond_drop_mask=None)
        v_u = self.forward(x, t, torch.zeros_like(cond), cond_drop_mask=None)
        return v_c + guidance_scale * (v_c - v_u)
