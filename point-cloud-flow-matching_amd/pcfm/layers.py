"""Per-point layers of the flow model's head on the gfx950 path.

`RowsLinear` is nn.Linear (same parameters, state_dict, init) whose bf16
autocast backward computes the weight gradient with pcfm's split-row MFMA
kernel (csrc/head.hip, `pcfm_rows_wgrad_bf16`) instead of the library GEMM,
which runs the (out, B*N) x (B*N, in) product with the long axis as its
reduction on a handful of tiles.  Semantics are autocast's: inputs and weight
cast to bf16, y = x W^T + b in bf16, grads dx = dy W, dW = dy^T x, db = sum dy,
all bf16 results of fp32 accumulation.  Outside bf16 autocast on a HIP device
it is exactly nn.Linear.forward.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ["RowsLinear"]


class _RowsLinearBF16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        from pcfm import ops
        x, w = ctx.saved_tensors
        lead = gy.shape[:-1]
        g2 = gy.reshape(-1, gy.shape[-1])
        if g2.stride(1) != 1:
            g2 = g2.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.mm(g2, w).view(*lead, w.shape[1])
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1])
            if x2.stride(1) != 1:
                x2 = x2.contiguous()
            gw = ops.rows_wgrad_bf16(g2, x2)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = ops.rows_colsum(g2).to(g2.dtype) if ops.colsum_ok(g2) else g2.sum(0)
        return gx, gw, gb


class RowsLinear(nn.Linear):
    """nn.Linear with the split-row MFMA weight gradient under bf16 autocast."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if (x.is_cuda and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16
                and x.numel() // max(1, x.shape[-1]) >= 4096):
            dt = torch.bfloat16
            b = self.bias.to(dt) if self.bias is not None else None
            with torch.autocast("cuda", enabled=False):
                return _RowsLinearBF16.apply(x.to(dt), self.weight.to(dt), b)
        return super().forward(x)


# ---------------------------------------------------------------------------
# Fused trunk of VelocityNetWithContext / VelocityNet (models.py:82-153,
# 546-601): input Linear -> (depth-1) x [FiLM(LayerNorm) -> h + Linear(SiLU(h))]
# -> Linear(SiLU(h)), under bf16 autocast, with the per-batch FiLM vectors.
# The row passes run as csrc/head_film.hip kernels (one pass per block forward,
# one backward), the Linears as library GEMMs (forward, backward-data) and the
# split-row MFMA weight gradient.  Saved per block: u (f32), g and a (bf16),
# row mean/rstd; the residual sum h = u_prev + g_prev is recomputed.
# ---------------------------------------------------------------------------
_PER_BLOCK = 6  # ln_weight, ln_bias, sp1, shift, weight16, bias16


class _HeadTrunkBF16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, n, eps, x16, w_in, hb, w_out, b_out, *blk):
        # hb (B, W) fp32: the input Linear's bias plus its embedding columns applied
        # to the per-batch embedding, added to h1 inside the first FiLM kernel
        from pcfm import ops
        nb = len(blk) // _PER_BLOCK
        h1 = F.linear(x16, w_in)
        hb = hb.contiguous()
        us, gs, as_, stats = [], [], [], []
        u = g = None
        for k in range(nb):
            lw, lb, sp1, sh, wk, bk = blk[_PER_BLOCK * k:_PER_BLOCK * (k + 1)]
            u, a, mean, rstd = ops.head_film_fwd(h1 if k == 0 else None, u, g, lw, lb, sp1, sh,
                                                 n, eps, hbias=hb if k == 0 else None)
            g = F.linear(a, wk, bk)
            us.append(u)
            gs.append(g)
            as_.append(a)
            stats += [mean, rstd]
        a_out = ops.head_silu_fwd(u, g, n)
        out = F.linear(a_out, w_out, b_out)
        ctx.n, ctx.eps, ctx.nb = n, eps, nb
        ctx.save_for_backward(x16, w_in, h1, hb, w_out, a_out, *us, *gs, *as_, *stats, *blk)
        return out

    @staticmethod
    def backward(ctx, gout):
        from pcfm import ops
        n, nb = ctx.n, ctx.nb
        sv = ctx.saved_tensors
        x16, w_in, h1, hb, w_out, a_out = sv[:6]
        us, gs, as_ = sv[6:6 + nb], sv[6 + nb:6 + 2 * nb], sv[6 + 2 * nb:6 + 3 * nb]
        stats = sv[6 + 3 * nb:6 + 5 * nb]
        blk = sv[6 + 5 * nb:]
        gout = gout.contiguous()
        d_w_out = ops.rows_wgrad_bf16(gout, a_out)
        d_b_out = ops.rows_colsum(gout).to(gout.dtype) if ops.colsum_ok(gout) else gout.sum(0)
        da = torch.mm(gout, w_out)
        dh, dh16, dbias = ops.head_silu_bwd(da, us[-1], gs[-1], n)
        d_blk = [None] * len(blk)
        for k in range(nb - 1, -1, -1):
            lw, lb, sp1, sh, wk, _ = blk[_PER_BLOCK * k:_PER_BLOCK * (k + 1)]
            # dh16 is dL/dg_k (the bf16 operand of h_{k+1} = u_k + g_k)
            d_blk[_PER_BLOCK * k + 4] = ops.rows_wgrad_bf16(dh16, as_[k])
            d_blk[_PER_BLOCK * k + 5] = dbias.to(torch.bfloat16)
            da = torch.mm(dh16, wk)
            first = k == 0
            # u_k recomputed in the kernel from h_k and the row statistics (not read back)
            res = ops.head_film_bwd(
                dh, da, None, h1 if first else None, None if first else us[k - 1],
                None if first else gs[k - 1], stats[2 * k], stats[2 * k + 1], lw, lb, sp1, n,
                want_dh=not first, hbias=hb if first else None, shift=sh)
            dh, dh16, dsp1, dshift, dgamma, dbeta, dbias = res[:7]
            if first:
                d_hb = res[7]
            d_blk[_PER_BLOCK * k] = dgamma
            d_blk[_PER_BLOCK * k + 1] = dbeta
            d_blk[_PER_BLOCK * k + 2] = dsp1.to(torch.bfloat16)
            d_blk[_PER_BLOCK * k + 3] = dshift.to(torch.bfloat16)
        # dh16 = dL/dh_1 (bf16 output of the input Linear); d hb per batch
        d_w_in = ops.rows_wgrad_bf16(dh16, x16)
        dx = torch.mm(dh16, w_in)
        return (None, None, dx, d_w_in, d_hb, d_w_out, d_b_out, *d_blk)


def fused_trunk_supported(trunk, h: torch.Tensor, emb: torch.Tensor, n: int) -> bool:
    """The fused trunk covers the reference configuration: bf16 autocast on a HIP
    device, per-batch FiLM, LayerNorm widths 256/512, biased Linears."""
    if not (h.is_cuda and h.dim() == 2 and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    if getattr(trunk, "film_per_point", False) or emb.dim() != 2 or emb.shape[0] * n != h.shape[0]:
        return False
    width = trunk.input.out_features
    if len(trunk.films) == 0 or width not in (256, 512) or trunk.input.bias is None or trunk.out[1].bias is None:
        return False
    for seq, film in zip(trunk.blocks, trunk.films):
        norm = film.norm
        if not (isinstance(norm, nn.LayerNorm) and norm.elementwise_affine
                and norm.weight is not None and norm.bias is not None
                and tuple(norm.normalized_shape) == (width,)) or seq[1].bias is None:
            return False
    eps = {film.norm.eps for film in trunk.films}
    return len(eps) <= 1


_FILM_BATCH = os.environ.get("PCFM_FILM_BATCH", "1") != "0"  # A/B knob (dev)


def fused_trunk(trunk, h: torch.Tensor, emb: torch.Tensor, n: int) -> torch.Tensor:
    """trunk._run_trunk(h, emb, n) through _HeadTrunkBF16 (same math, autocast casts).

    h holds the per-point input columns only; the trunk input of the reference is
    cat([h, emb broadcast over the points]) (models.py:135, 594).  The embedding
    columns of the input Linear are constant along the points, so they and the
    bias become one per-batch row hb = W_emb bf16(emb) + b (fp32 accumulation of
    the same bf16 products), added to h1 in the first FiLM kernel: the input GEMM
    runs over the point columns only (K = 70 instead of 326)."""
    dt = torch.bfloat16
    blk = []
    from pcfm.models import _batch_fp32
    ctx, fp32 = _batch_fp32(emb)
    nb = len(trunk.films)
    if fp32 and nb > 1 and _FILM_BATCH:
        # all blocks at once: the FiLM affines as one batched fp32 product
        # (nb*2, B, W) and the blocks' Linear weights / biases cast to bf16 as one
        # stacked tensor each -- a handful of launches instead of ~6 per block
        with ctx:
            aw = torch.stack([f.affine.weight for f in trunk.films])  # (nb, 2W, E)
            ab = torch.stack([f.affine.bias for f in trunk.films])    # (nb, 2W)
            w2 = aw.shape[1] // 2
            wt = aw.view(nb * 2, w2, -1).transpose(1, 2)                # (nb*2, E, W)
            ss = torch.baddbmm(ab.view(nb * 2, 1, w2), emb.float().expand(nb * 2, -1, -1), wt)
            ss = ss.view(nb, 2, emb.shape[0], w2)
            # (nb, B, W) contiguous, so each block's slice is a contiguous (B, W)
            sp1s = (1.0 + ss[:, 0]).to(dt, memory_format=torch.contiguous_format)
            shifts = ss[:, 1].to(dt, memory_format=torch.contiguous_format)
        ws = torch.stack([seq[1].weight for seq in trunk.blocks]).to(dt)
        bs = torch.stack([seq[1].bias for seq in trunk.blocks]).to(dt)
        # unbind: one autograd node per stack, whose backward stacks the slices'
        # gradients in one launch (per-slice indexing would zero-fill and add)
        per = zip(sp1s.unbind(0), shifts.unbind(0), ws.unbind(0), bs.unbind(0))
        for film, (sp1, shift, wk, bk) in zip(trunk.films, per):
            blk += [film.norm.weight, film.norm.bias, sp1, shift, wk, bk]
    else:
        for seq, film in zip(trunk.blocks, trunk.films):
            with ctx:  # per-cloud FiLM vectors: fp32 (PCFM_BATCH_FP32=0: autocast bf16)
                scale, shift = film.affine(emb.float() if fp32 else emb).chunk(2, dim=-1)
            sp1 = 1.0 + scale
            blk += [film.norm.weight, film.norm.bias, sp1.to(dt).contiguous(),
                    shift.to(dt).contiguous(), seq[1].weight.to(dt), seq[1].bias.to(dt)]
    eps = trunk.films[0].norm.eps if len(trunk.films) else 1e-5
    lin_in, lin_out = trunk.input, trunk.out[1]
    k = h.shape[1]
    kp = (k + 7) // 8 * 8  # 16-B rows for the GEMM operands
    x16 = F.pad(h.to(dt), (0, kp - k))
    w_pts = F.pad(lin_in.weight[:, :k].to(dt), (0, kp - k))
    with torch.autocast("cuda", enabled=False):
        hb = F.linear(emb.to(dt).float(), lin_in.weight[:, k:].to(dt).float(),
                      lin_in.bias.to(dt).float())
        return _HeadTrunkBF16.apply(n, float(eps), x16, w_pts, hb, lin_out.weight.to(dt),
                                    lin_out.bias.to(dt), *blk)


class _RowsMax(torch.autograd.Function):
    """h.max(dim=1).values for (B, N, C) bf16 with torch.max's backward (the
    gradient goes to the argmax row, zeros elsewhere)."""

    @staticmethod
    def forward(ctx, h):
        from pcfm import ops
        val, idx = ops.rows_max_bf16(h)
        ctx.save_for_backward(idx)
        ctx.shape = h.shape
        return val

    @staticmethod
    def backward(ctx, gv):
        (idx,) = ctx.saved_tensors
        g = torch.zeros(ctx.shape, dtype=gv.dtype, device=gv.device)
        g.scatter_(1, idx.long().unsqueeze(1), gv.unsqueeze(1))
        return g


def max_over_points(h: torch.Tensor) -> torch.Tensor:
    """h.max(dim=1).values; the gfx950 kernel for contiguous (B, N, C) bf16 on a HIP device."""
    if (h.is_cuda and h.dtype == torch.bfloat16 and h.dim() == 3 and h.is_contiguous()
            and h.shape[1] > 0 and h.shape[2] % 2 == 0):
        return _RowsMax.apply(h)
    return h.max(dim=1).values
