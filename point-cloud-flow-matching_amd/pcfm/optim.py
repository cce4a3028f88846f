"""The train step's parameter update as three HIP launches (include/pcfm.h,
csrc/optim.hip): GradScaler.unscale_ + clip_grad_norm_ + AdamW.step + the EMA
update of the new parameters, i.e. reference train.py:652-661 with
torch.optim.AdamW (train.py:249-253) and util.EMA (util.py:17-21).

torch runs this tail as ~40 multi-tensor launches, several passes over every
parameter list (~0.8 ms per step at the C2 configuration); here one pass reads
the gradients (norm), one reads g, p, m, v, shadow and writes p, m, v, shadow.

Semantics kept: per-group lr / weight decay (the cosine schedule writes
`param_groups[i]["lr"]` as it does for torch's optimizer), the gradient norm
over the UNSCALED gradients with clip coefficient min(1, max / (norm + 1e-6)),
the GradScaler inf check (a non-finite gradient skips the update and the step
count, like AdamW(fused=True), and the scale backs off through
torch._amp_update_scale_), AdamW's foreach arithmetic, and the EMA's
shadow.mul_(d).add_(p, alpha=1 - d) on the updated parameters.  Parameters
without a gradient are left alone (torch skips them too).  `p.grad` is not
modified (it is freed by zero_grad anyway).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib

__all__ = ["FusedAdamWEMA"]

_TAB = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"), ("ema", "<u8"),
                 ("n", "<i8"), ("group", "<i4"), ("flags", "<i4")])
_VEC4, _SKIP, _EMA = 1, 2, 4


class FusedAdamWEMA:
    """AdamW over parameter groups + clip + GradScaler unscale + EMA, fused.

    groups: [{"params": [...], "lr": lr, "weight_decay": wd}, ...] (as
    torch.optim.AdamW); ema_shadows: {parameter: shadow tensor} for the
    parameters whose EMA is updated in the same pass."""

    def __init__(self, groups: Sequence[Dict], betas=(0.9, 0.999), eps: float = 1e-8,
                 ema_shadows: Optional[Dict[torch.Tensor, torch.Tensor]] = None,
                 ema_decay: float = 0.999):
        self.param_groups: List[Dict] = []
        params: List[torch.Tensor] = []
        group_of: List[int] = []
        for gi, g in enumerate(groups):
            ps = [p for p in g["params"]]
            self.param_groups.append({"params": ps, "lr": float(g["lr"]),
                                      "weight_decay": float(g.get("weight_decay", 1e-2))})
            params += ps
            group_of += [gi] * len(ps)
        if not 1 <= len(self.param_groups) <= 8:
            raise ValueError("FusedAdamWEMA: 1..8 parameter groups")
        dev = params[0].device
        if dev.type != "cuda" or any(p.dtype != torch.float32 or not p.is_contiguous()
                                     or p.device != dev for p in params):
            raise ValueError("FusedAdamWEMA: contiguous fp32 parameters on one HIP device")
        self.params = params
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.ema_decay = float(ema_decay)
        shadows = ema_shadows or {}
        # exp_avg / exp_avg_sq: one buffer each, every tensor 64-element aligned
        offs, tot = [], 0
        for p in params:
            offs.append(tot)
            tot += (p.numel() + 63) // 64 * 64
        self.exp_avg = torch.zeros(max(tot, 1), device=dev)
        self.exp_avg_sq = torch.zeros(max(tot, 1), device=dev)
        self.state_dev = torch.zeros(4, device=dev)  # norm, multiplier, found_inf
        self.steps = torch.zeros(len(params), device=dev)  # per-parameter step counts
        tab = np.zeros(len(params), dtype=_TAB)
        chunk = _lib.query("pcfm_adamw_chunk_elems")
        chunks = []
        base = self.exp_avg.data_ptr()
        vbase = self.exp_avg_sq.data_ptr()
        self._ema_ptr = []
        for i, p in enumerate(params):
            sh = shadows.get(p)
            if sh is not None and (sh.shape != p.shape or sh.dtype != p.dtype
                                   or not sh.is_contiguous() or sh.device != dev):
                raise ValueError("FusedAdamWEMA: EMA shadow must match its parameter")
            tab[i]["p"] = p.data_ptr()
            tab[i]["m"] = base + 4 * offs[i]
            tab[i]["v"] = vbase + 4 * offs[i]
            tab[i]["ema"] = sh.data_ptr() if sh is not None else 0
            tab[i]["n"] = p.numel()
            tab[i]["group"] = group_of[i]
            self._ema_ptr.append(sh)
            for s in range(0, p.numel(), chunk):
                chunks.append((i, s))
        self._tab = tab
        self._static_vec4 = np.array([
            p.numel() % 4 == 0 and p.data_ptr() % 16 == 0
            and (sh is None or sh.data_ptr() % 16 == 0)
            for p, sh in zip(params, self._ema_ptr)])
        self._has_ema = np.array([sh is not None for sh in self._ema_ptr])
        self.nchunks = len(chunks)
        self.chunks = torch.tensor(np.array(chunks, dtype=np.int32).reshape(-1), device=dev)
        self.ws = torch.empty(_lib.query("pcfm_adamw_workspace_bytes", self.nchunks),
                              dtype=torch.uint8, device=dev)
        # the per-step table (gradient pointers change every step) goes through two
        # pinned staging buffers, each reused only after its previous copy finished
        nb = tab.nbytes
        self._pinned = [torch.empty(nb, dtype=torch.uint8).pin_memory() for _ in range(2)]
        self._events = [None, None]
        self._tab_dev = torch.empty(nb, dtype=torch.uint8, device=dev)
        self._turn = 0

    # torch.optim API pieces the Trainer uses
    def zero_grad(self, set_to_none: bool = True) -> None:
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    # checkpoint layout of torch.optim.AdamW (the reference saves opt.state_dict()
    # with every checkpoint and restores it on resume, train.py:501, :701)
    def _moments(self, i: int):
        off = int(self._tab[i]["m"] - self.exp_avg.data_ptr()) // 4
        p = self.params[i]
        n = p.numel()
        return (self.exp_avg[off:off + n].view_as(p), self.exp_avg_sq[off:off + n].view_as(p))

    def state_dict(self) -> Dict:
        """{'state': {index: {'step', 'exp_avg', 'exp_avg_sq'}}, 'param_groups':
        [...]} as torch.optim.AdamW.state_dict() lays it out: parameters numbered
        in group order, an entry only for parameters that have taken a step,
        `step` a float32 scalar tensor on the CPU."""
        steps = self.steps.cpu()
        state = {}
        for i in range(len(self.params)):
            if float(steps[i]) > 0:
                m, v = self._moments(i)
                state[i] = {"step": steps[i].clone(), "exp_avg": m.clone(),
                            "exp_avg_sq": v.clone()}
        groups, k = [], 0
        for g in self.param_groups:
            n = len(g["params"])
            groups.append({"lr": g["lr"], "betas": self.betas, "eps": self.eps,
                           "weight_decay": g["weight_decay"], "amsgrad": False,
                           "maximize": False, "foreach": None, "capturable": False,
                           "differentiable": False, "fused": None,
                           "params": list(range(k, k + n))})
            k += n
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd: Dict) -> None:
        """Accepts torch.optim.AdamW's (or this class's) state_dict: moments and
        step counts per parameter, lr / weight decay per group."""
        groups = sd["param_groups"]
        if len(groups) != len(self.param_groups) or any(
                len(a["params"]) != len(b["params"]) for a, b in zip(groups, self.param_groups)):
            raise ValueError("FusedAdamWEMA.load_state_dict: parameter groups do not match")
        if any(g.get("amsgrad") or g.get("maximize") for g in groups):
            raise ValueError("FusedAdamWEMA.load_state_dict: amsgrad / maximize unsupported")
        if any(tuple(g.get("betas", self.betas)) != self.betas
               or float(g.get("eps", self.eps)) != self.eps for g in groups):
            raise ValueError("FusedAdamWEMA.load_state_dict: betas / eps differ")
        index = [i for g in groups for i in g["params"]]
        steps = torch.zeros(len(self.params))
        with torch.no_grad():
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            for pos, key in enumerate(index):
                st = sd["state"].get(key)
                if st is None:
                    continue
                m, v = self._moments(pos)
                for name, dst in (("exp_avg", m), ("exp_avg_sq", v)):
                    if tuple(st[name].shape) != tuple(dst.shape):  # copy_ would broadcast
                        raise ValueError(f"FusedAdamWEMA.load_state_dict: state {key} {name} "
                                         f"shape {tuple(st[name].shape)} != parameter shape "
                                         f"{tuple(dst.shape)}")
                m.copy_(st["exp_avg"])
                v.copy_(st["exp_avg_sq"])
                steps[pos] = float(st["step"])
            self.steps.copy_(steps)
        for mine, g in zip(self.param_groups, groups):
            mine["lr"] = float(g["lr"])
            mine["weight_decay"] = float(g["weight_decay"])

    @property
    def last_grad_norm(self) -> torch.Tensor:
        """clip_grad_norm_'s return value of the last step (device scalar)."""
        return self.state_dev[0]

    @property
    def found_inf(self) -> torch.Tensor:
        return self.state_dev[2:3]

    def _upload_table(self, stream) -> None:
        tab = self._tab
        grads = [p.grad for p in self.params]
        gp = np.array([0 if g is None else g.data_ptr() for g in grads], dtype=np.uint64)
        for g in grads:
            if g is not None and (g.dtype != torch.float32 or not g.is_contiguous()):
                raise ValueError("FusedAdamWEMA: gradients must be contiguous fp32")
        tab["g"] = gp
        skip = gp == 0
        vec4 = self._static_vec4 & (gp % 16 == 0)
        tab["flags"] = (np.where(vec4, _VEC4, 0) | np.where(skip, _SKIP, 0)
                        | np.where(self._has_ema, _EMA, 0))
        k = self._turn
        self._turn ^= 1
        if self._events[k] is not None:
            self._events[k].synchronize()
        buf = self._pinned[k]
        buf.numpy()[:] = tab.view(np.uint8)
        with torch.cuda.stream(stream):
            self._tab_dev.copy_(buf, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        self._events[k] = ev

    @torch.no_grad()
    def step(self, max_norm: float = 0.0, scaler=None) -> torch.Tensor:
        """Unscale (scaler enabled) + clip (max_norm > 0) + AdamW + EMA; then the
        scaler's scale update.  Returns the total gradient norm (device scalar)."""
        dev = self.params[0].device
        stream = torch.cuda.current_stream(dev)
        self._upload_table(stream)
        scale = None
        if scaler is not None and scaler.is_enabled():
            scale = scaler._scale  # set by scaler.scale(loss) (lazy init)
            if scale is None:
                raise RuntimeError("FusedAdamWEMA.step: scaler.scale(loss) was not called")
        _lib.call("pcfm_adamw_grad_norm", self._tab_dev.data_ptr(), len(self.params),
                  self.chunks.data_ptr(), self.nchunks,
                  scale.data_ptr() if scale is not None else None, float(max_norm),
                  self.steps.data_ptr(), self.state_dev.data_ptr(), self.ws.data_ptr(),
                  self.ws.numel(), stream.cuda_stream)
        ng = len(self.param_groups)
        lr = (ctypes.c_double * ng)(*[g["lr"] for g in self.param_groups])
        wd = (ctypes.c_double * ng)(*[g["weight_decay"] for g in self.param_groups])
        _lib.call("pcfm_adamw_ema_step", self._tab_dev.data_ptr(), self.chunks.data_ptr(),
                  self.nchunks, self.steps.data_ptr(), self.state_dev.data_ptr(), ng, lr, wd,
                  self.betas[0],
                  self.betas[1], self.eps, self.ema_decay, stream.cuda_stream)
        if scale is not None:
            torch._amp_update_scale_(scaler._scale, scaler._growth_tracker, self.found_inf,
                                     scaler._growth_factor, scaler._backoff_factor,
                                     scaler._growth_interval)
        return self.last_grad_norm
