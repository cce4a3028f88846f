"""Tensor-level operators with the reference's native-module signatures.

``backend`` mirrors the pybind module ``_pvcnn_backend``
(third_party/pvcnn/modules/functional/src/bindings.cpp:10-37): same function
names, argument order and meaning, return values, and the same argument checks
(utils.hpp:7-18 -> RuntimeError).  ``chamfer_3D`` mirrors the Chamfer module
(chamfer3D/chamfer_cuda.cpp:17-32) and ``emd_cuda`` the EMD module
(PyTorchEMD/cuda/emd.cpp:8-27).

Every op runs on the current HIP stream of the tensors' device through the C ABI
(include/pcfm.h); outputs are allocated with torch.empty (the kernels write
every element, so the reference's torch::zeros pre-fill is not needed).  The
reference-named entry points also accept CPU tensors, which run the pure-PyTorch
backend in pcfm.cpu_ops (BASELINE configs[0]); HIP tensors never fall back.
"""
from __future__ import annotations

import ctypes
import types

import torch

from . import _lib, cpu_ops


# --------------------------------------------------------------------------
# argument checks (utils.hpp:7-18)
# --------------------------------------------------------------------------
def _check_cuda(x: torch.Tensor, name: str) -> None:
    if not (isinstance(x, torch.Tensor) and x.is_cuda):
        raise RuntimeError(f"{name} must be a CUDA tensor")


def _check_contig(x: torch.Tensor, name: str) -> None:
    if not x.is_contiguous():
        raise RuntimeError(f"{name} must be a contiguous tensor")


def _check_float(x: torch.Tensor, name: str) -> None:
    if x.dtype != torch.float32:
        raise RuntimeError(f"{name} must be a float tensor")


def _check_int(x: torch.Tensor, name: str) -> None:
    if x.dtype != torch.int32:
        raise RuntimeError(f"{name} must be an int tensor")


def _check(x, name, kind):
    _check_cuda(x, name)
    _check_contig(x, name)
    (_check_float if kind == "f" else _check_int)(x, name)


def _host(*ts) -> bool:
    """True when every tensor is a CPU tensor: the call then runs the pure-PyTorch
    backend (pcfm.cpu_ops, BASELINE configs[0]); a mix of CPU and HIP tensors is an
    error, as in the reference (utils.hpp:7-18)."""
    cpu = [not t.is_cuda for t in ts if isinstance(t, torch.Tensor)]
    if all(cpu):
        return True
    if any(cpu):
        raise RuntimeError("all tensors must be on the same device (CUDA or CPU)")
    return False


def _check_host(x, name, kind):
    _check_contig(x, name)
    (_check_float if kind == "f" else _check_int)(x, name)


def _ptr(x: torch.Tensor) -> int:
    return x.data_ptr()


def _stream(x: torch.Tensor) -> int:
    return torch.cuda.current_stream(x.device).cuda_stream


def _workspace(nbytes: int, like: torch.Tensor) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=like.device)


# --------------------------------------------------------------------------
# optional live timing: HIP events around each C-ABI call, on the stream the
# kernels are launched on (bench.py turns this on for its timed region)
# --------------------------------------------------------------------------
class _OpTimer:
    def __init__(self):
        self.enabled = False
        self.only = None  # None: every op; else the set of op names to time
        self.records = []  # (op, start_event, end_event, amount, kind)

    def on(self, op):
        return self.enabled and (self.only is None or op in self.only)

    def reset(self):
        self.records = []

    def summary(self):
        """{op: {"launches", "ms", "amount", "kind"}} -- synchronize() first.
        kind "hbm": amount = algorithmic bytes; kind "mfma":
        amount = algorithmic fp32 FLOPs of the convolution."""
        out = {}
        for op, e0, e1, amount, kind in self.records:
            d = out.setdefault(op, {"launches": 0, "ms": 0.0, "amount": 0, "kind": kind})
            d["launches"] += 1
            d["ms"] += e0.elapsed_time(e1)
            d["amount"] += amount
        return out


timer = _OpTimer()


class _timed:
    __slots__ = ("op", "amount", "kind", "dev", "e0")

    def __init__(self, op, amount, like, kind="hbm"):
        self.op, self.amount, self.kind, self.dev = op, int(amount), kind, like.device

    def __enter__(self):
        self.e0 = None
        if timer.on(self.op):
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record(torch.cuda.current_stream(self.dev))

    def __exit__(self, *exc):
        if self.e0 is not None and exc[0] is None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(torch.cuda.current_stream(self.dev))
            timer.records.append((self.op, self.e0, e1, self.amount, self.kind))
        return False


# --------------------------------------------------------------------------
# _pvcnn_backend
# --------------------------------------------------------------------------
def avg_voxelize_forward(features: torch.Tensor, coords: torch.Tensor, resolution: int):
    """vox.cpp:17-43: -> [out f32 (b,c,r^3), ind i32 (b,n), cnt i32 (b,r^3)]"""
    if _host(features, coords):
        _check_host(features, "features", "f")
        _check_host(coords, "coords", "i")
        return cpu_ops.avg_voxelize_forward(features, coords, resolution)
    _check(features, "features", "f")
    _check(coords, "coords", "i")
    b, c, n = features.shape
    r = int(resolution)
    s = r * r * r
    out = torch.empty((b, c, s), dtype=torch.float32, device=features.device)
    ind = torch.empty((b, n), dtype=torch.int32, device=features.device)
    cnt = torch.empty((b, s), dtype=torch.int32, device=features.device)
    ws = _workspace(_lib.query("pcfm_avg_voxelize_fwd_workspace_bytes", b, c, n, r), features)
    nbytes = 4 * b * (3 * n + c * n + n + s + c * s)  # vox-fwd
    with _timed("avg_voxelize_fwd", nbytes, features):
        _lib.call("pcfm_avg_voxelize_fwd", _ptr(features), _ptr(coords), b, c, n, r, _ptr(out),
                  _ptr(ind), _ptr(cnt), _ptr(ws), ws.numel(), _stream(features))
    return [out, ind, cnt]


def avg_voxelize_backward(grad_y: torch.Tensor, indices: torch.Tensor, cnt: torch.Tensor):
    """vox.cpp:54-76: grad_y (b,c,s) -> grad_x (b,c,n)"""
    if _host(grad_y, indices, cnt):
        _check_host(grad_y, "grad_y", "f")
        _check_host(indices, "indices", "i")
        _check_host(cnt, "cnt", "i")
        return cpu_ops.avg_voxelize_backward(grad_y, indices, cnt)
    _check(grad_y, "grad_y", "f")
    _check(indices, "indices", "i")
    _check(cnt, "cnt", "i")
    b, c, s = grad_y.shape
    n = indices.shape[1]
    grad_x = torch.empty((b, c, n), dtype=torch.float32, device=grad_y.device)
    nbytes = 4 * b * (c * s + n + s + c * n)  # vox-bwd
    with _timed("avg_voxelize_bwd", nbytes, grad_y):
        _lib.call("pcfm_avg_voxelize_bwd", _ptr(grad_y), _ptr(indices), _ptr(cnt), b, c, n, s,
                  _ptr(grad_x), _stream(grad_y))
    return grad_x


def avg_voxelize_backward_add(grad_y: torch.Tensor, indices: torch.Tensor, cnt: torch.Tensor,
                              add: torch.Tensor):
    """avg_voxelize_backward(grad_y) + add, add (b,c,n) fp32, in one gather."""
    _check(grad_y, "grad_y", "f")
    _check(indices, "indices", "i")
    _check(cnt, "cnt", "i")
    add = add.contiguous()
    _check(add, "add", "f")
    b, c, s = grad_y.shape
    n = indices.shape[1]
    if tuple(add.shape) != (b, c, n):
        raise ValueError("avg_voxelize_backward_add: add must be (B, C, N)")
    grad_x = torch.empty((b, c, n), dtype=torch.float32, device=grad_y.device)
    nbytes = 4 * b * (c * s + n + s + 2 * c * n)
    with _timed("avg_voxelize_bwd", nbytes, grad_y):
        _lib.call("pcfm_avg_voxelize_bwd_add", _ptr(grad_y), _ptr(indices), _ptr(cnt), _ptr(add),
                  b, c, n, s, _ptr(grad_x), _stream(grad_y))
    return grad_x


def trilinear_devoxelize_forward(r: int, is_training: bool, coords: torch.Tensor,
                                 features: torch.Tensor):
    """trilinear_devox.cpp:18-55: -> [outs (b,c,n), inds (b,8,n)|(1,), wgts (b,8,n)|(1,)]"""
    if _host(coords, features):
        _check_host(features, "features", "f")
        _check_host(coords, "coords", "f")
        return cpu_ops.trilinear_devoxelize_forward(r, is_training, coords, features)
    _check(features, "features", "f")
    _check(coords, "coords", "f")
    b, c = features.shape[0], features.shape[1]
    n = coords.shape[2]
    r = int(r)
    dev = features.device
    outs = torch.empty((b, c, n), dtype=torch.float32, device=dev)
    if is_training:
        inds = torch.empty((b, 8, n), dtype=torch.int32, device=dev)
        wgts = torch.empty((b, 8, n), dtype=torch.float32, device=dev)
        pi, pw = _ptr(inds), _ptr(wgts)
    else:
        inds = torch.zeros((1,), dtype=torch.int32, device=dev)
        wgts = torch.zeros((1,), dtype=torch.float32, device=dev)
        pi, pw = None, None
    nbytes = 4 * b * (3 * n + c * r ** 3 + c * n + (16 * n if is_training else 0))
    with _timed("trilinear_devoxelize_fwd", nbytes, features):  # devox-fwd
        _lib.call("pcfm_trilinear_devoxelize_fwd", _ptr(coords), _ptr(features), b, c, n, r,
                  1 if is_training else 0, _ptr(outs), pi, pw, _stream(features))
    if devox_verify.enabled:
        devox_verify(coords, features, None, None, outs, inds if is_training else None,
                     wgts if is_training else None, r)
    return [outs, inds, wgts]


def trilinear_devoxelize_scale_add(r: int, is_training: bool, coords: torch.Tensor,
                                   features: torch.Tensor, scale, add):
    """scale[b, c] * devox(features) + add (either None): SE3d and the PVConv
    point-branch sum folded into the devoxelization -> [outs, inds, wgts]."""
    _check(features, "features", "f")
    _check(coords, "coords", "f")
    b, c = features.shape[0], features.shape[1]
    n = coords.shape[2]
    r = int(r)
    dev = features.device
    if scale is not None:
        scale = scale.contiguous()
        _check(scale, "scale", "f")
        if scale.numel() != b * c:
            raise ValueError("trilinear_devoxelize_scale_add: scale must be (B, C)")
    if add is not None:
        add = add.contiguous()
        _check(add, "add", "f")
        if tuple(add.shape) != (b, c, n):
            raise ValueError("trilinear_devoxelize_scale_add: add must be (B, C, N)")
    outs = torch.empty((b, c, n), dtype=torch.float32, device=dev)
    if is_training:
        inds = torch.empty((b, 8, n), dtype=torch.int32, device=dev)
        wgts = torch.empty((b, 8, n), dtype=torch.float32, device=dev)
        pi, pw = _ptr(inds), _ptr(wgts)
    else:
        inds = torch.zeros((1,), dtype=torch.int32, device=dev)
        wgts = torch.zeros((1,), dtype=torch.float32, device=dev)
        pi, pw = None, None
    nbytes = 4 * b * (3 * n + c * r ** 3 + c * n * (2 if add is not None else 1)
                      + (16 * n if is_training else 0))
    with _timed("trilinear_devoxelize_fwd", nbytes, features):
        _lib.call("pcfm_trilinear_devoxelize_scale_add_fwd", _ptr(coords), _ptr(features),
                  _ptr(scale) if scale is not None else None,
                  _ptr(add) if add is not None else None, b, c, n, r, 1 if is_training else 0,
                  _ptr(outs), pi, pw, _stream(features))
    if devox_verify.enabled:
        devox_verify(coords, features, scale, add, outs, inds if is_training else None,
                     wgts if is_training else None, r)
    return [outs, inds, wgts]


class _DevoxVerify:
    """Diagnosis switch (PCFM_DEVOX_VERIFY=1): after every devoxelization gather,
    pcfm_debug_devox_verify recomputes each output in the plainest form on the
    same stream and compares bit for bit; mismatches accumulate on the device
    (report() reads them once, at the end)."""

    def __init__(self):
        import os
        self.enabled = os.environ.get("PCFM_DEVOX_VERIFY") == "1"
        self.rec = None
        self.calls = 0

    def __call__(self, coords, features, scale, add, outs, inds, wgts, r):
        if self.rec is None or self.rec.device != outs.device:
            self.rec = torch.zeros(2 + 16 * 8, dtype=torch.int32, device=outs.device)
        b, c, n = outs.shape
        self.calls += 1
        _lib.call("pcfm_debug_devox_verify", _ptr(coords), _ptr(features),
                  _ptr(scale) if scale is not None else None,
                  _ptr(add) if add is not None else None, _ptr(outs),
                  _ptr(inds) if inds is not None else None,
                  _ptr(wgts) if wgts is not None else None, b, c, n, int(r), _ptr(self.rec),
                  _stream(outs))

    def bn(self, coords, features, bn, scale, add, add_bn, outs, inds, wgts, r):
        """The check for trilinear_devoxelize_bn_scale_add (bn / add_bn: the
        (mean, invstd, weight, bias, slope) transforms of the rows / the add)."""
        if self.rec is None or self.rec.device != outs.device:
            self.rec = torch.zeros(2 + 16 * 8, dtype=torch.int32, device=outs.device)
        b, c, n = outs.shape
        self.calls += 1
        abn = [_ptr(t) for t in add_bn[:4]] if add_bn is not None else [None] * 4
        aslope = float(add_bn[4]) if add_bn is not None else 0.0
        _lib.call("pcfm_debug_devox_verify_bn", _ptr(coords), _ptr(features),
                  *[_ptr(t) for t in bn[:4]], float(bn[4]),
                  _ptr(scale) if scale is not None else None,
                  _ptr(add) if add is not None else None, *abn, aslope, _ptr(outs),
                  _ptr(inds) if inds is not None else None,
                  _ptr(wgts) if wgts is not None else None, b, c, n, int(r), _ptr(self.rec),
                  _stream(outs))

    def report(self):
        if self.rec is None:
            return {"calls": self.calls, "mismatches": 0, "bad_weight_sums": 0, "records": []}
        h = self.rec.cpu().tolist()
        recs = []
        for k in range(min(h[0], 16)):
            e = h[2 + 8 * k: 10 + 8 * k]
            recs.append({"kind": ("out", "ind", "wgt")[e[0]], "b": e[1], "c": e[2], "i": e[3],
                         "got_bits": e[4], "want_bits": e[5], "lane": e[6], "wave_of_i": e[7]})
        return {"calls": self.calls, "mismatches": h[0], "bad_weight_sums": h[1], "records": recs}


devox_verify = _DevoxVerify()


# --------------------------------------------------------------------------
# segment plans (include/pcfm.h): the sort + work units of a scatter, built
# once per (points, resolution) and applied to several feature tensors
# --------------------------------------------------------------------------
class SegPlan:
    """A device-resident segment plan; `ind` / `cnt` for a voxelization plan."""

    __slots__ = ("buf", "b", "n", "r", "taps", "ind", "cnt")

    def __init__(self, buf, b, n, r, taps, ind=None, cnt=None):
        self.buf, self.b, self.n, self.r, self.taps = buf, b, n, r, taps
        self.ind, self.cnt = ind, cnt


def avg_voxelize_plan(coords: torch.Tensor, resolution: int) -> SegPlan:
    """Voxelization plan of integer coords (b, 3, n); plan.ind (b, n) and
    plan.cnt (b, r^3) are avg_voxelize_forward's ind / cnt."""
    _check(coords, "coords", "i")
    b, n = coords.shape[0], coords.shape[2]
    r = int(resolution)
    dev = coords.device
    ind = torch.empty((b, n), dtype=torch.int32, device=dev)
    cnt = torch.empty((b, r ** 3), dtype=torch.int32, device=dev)
    buf = _workspace(_lib.query("pcfm_seg_plan_bytes", b, n, r, 1), coords)
    with _timed("avg_voxelize_plan", 4 * b * (3 * n + 3 * n + 2 * r ** 3), coords):
        _lib.call("pcfm_avg_voxelize_plan", _ptr(coords), b, n, r, _ptr(ind), _ptr(cnt), _ptr(buf),
                  buf.numel(), _stream(coords))
    return SegPlan(buf, b, n, r, 1, ind, cnt)


def avg_voxelize_forward_planned(features: torch.Tensor, plan: SegPlan) -> torch.Tensor:
    """avg_voxelize_forward's `out` (b, c, r^3) on a voxelization plan."""
    _check(features, "features", "f")
    b, c, n = features.shape
    if plan.taps != 1 or (b, n) != (plan.b, plan.n):
        raise ValueError("avg_voxelize_forward_planned: plan does not match the features")
    r = plan.r
    out = torch.empty((b, c, r ** 3), dtype=torch.float32, device=features.device)
    ws = _workspace(_lib.query("pcfm_seg_apply_workspace_bytes", b, c, n, r, 1), features)
    with _timed("avg_voxelize_fwd", 4 * b * (c * n + c * r ** 3), features):
        _lib.call("pcfm_avg_voxelize_fwd_planned", _ptr(features), _ptr(plan.buf), b, c, n, r,
                  _ptr(out), _ptr(ws), ws.numel(), _stream(features))
    return out


def trilinear_devoxelize_backward_plan(indices: torch.Tensor, weights: torch.Tensor,
                                       r: int) -> SegPlan:
    """Devoxelization-backward plan from the forward's inds / wgts (b, 8, n)."""
    _check(indices, "indices", "i")
    _check(weights, "weights", "f")
    b, n = indices.shape[0], indices.shape[2]
    r = int(r)
    buf = _workspace(_lib.query("pcfm_seg_plan_bytes", b, n, r, 8), indices)
    with _timed("trilinear_devoxelize_bwd_plan", 4 * b * 16 * n * 2, indices):
        _lib.call("pcfm_trilinear_devoxelize_bwd_plan", _ptr(indices), _ptr(weights), b, n, r,
                  _ptr(buf), buf.numel(), _stream(indices))
    return SegPlan(buf, b, n, r, 8)


def trilinear_devoxelize_backward_planned(grad_y: torch.Tensor, plan: SegPlan) -> torch.Tensor:
    """trilinear_devoxelize_backward's grad_x (b, c, r^3) on a devoxelization plan."""
    _check(grad_y, "grad_y", "f")
    b, c, n = grad_y.shape
    if plan.taps != 8 or (b, n) != (plan.b, plan.n):
        raise ValueError("trilinear_devoxelize_backward_planned: plan does not match grad_y")
    r = plan.r
    grad_x = torch.empty((b, c, r ** 3), dtype=torch.float32, device=grad_y.device)
    ws = _workspace(_lib.query("pcfm_seg_apply_workspace_bytes", b, c, n, r, 8), grad_y)
    # SURVEY 8d devox-bwd: grad_y in, inds + wgts (16N.4) in, grad_x out
    with _timed("trilinear_devoxelize_bwd", 4 * b * (c * n + 16 * n + c * r ** 3), grad_y):
        _lib.call("pcfm_trilinear_devoxelize_bwd_planned", _ptr(grad_y), _ptr(plan.buf), b, c, n,
                  r, _ptr(grad_x), _ptr(ws), ws.numel(), _stream(grad_y))
    return grad_x


def rows_dot(a: torch.Tensor, b, scale: float = 1.0) -> torch.Tensor:
    """scale * sum over the last axis of a * b (b None: of a) for 2-D (rows, len)."""
    _check(a, "a", "f")
    if b is not None:
        _check(b, "b", "f")
        if b.shape != a.shape:
            raise ValueError("rows_dot: shape mismatch")
    rows, length = a.shape
    out = torch.empty((rows,), dtype=torch.float32, device=a.device)
    nbytes = 4 * rows * length * (2 if b is not None else 1)
    with _timed("rows_dot", nbytes, a):
        _lib.call("pcfm_rows_dot", _ptr(a), _ptr(b) if b is not None else None, rows, length,
                  float(scale), _ptr(out), _stream(a))
    return out


def se_mlp_ok(m: torch.Tensor, w1: torch.Tensor) -> bool:
    b, c = m.shape
    h = w1.shape[0]
    return 2 * (b + h) * c + 2 * b * h <= 32768


def se_mlp_forward(m: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor):
    """SE3d's MLP (se.py:9-19): (s = sigmoid(W2 relu(W1 m)), hid = relu(W1 m))."""
    for t, n in ((m, "m"), (w1, "w1"), (w2, "w2")):
        _check(t, n, "f")
    b, c = m.shape
    h = w1.shape[0]
    if w1.shape != (h, c) or w2.shape != (c, h):
        raise ValueError("se_mlp_forward: weight shapes")
    hid = torch.empty((b, h), dtype=torch.float32, device=m.device)
    s = torch.empty((b, c), dtype=torch.float32, device=m.device)
    _lib.call("pcfm_se_mlp_fwd", _ptr(m), _ptr(w1), _ptr(w2), b, c, h, _ptr(hid), _ptr(s),
              _stream(m))
    return s, hid


def se_mlp_backward(m, hid, s, ds, w1, w2, dm_scale: float = 1.0):
    """-> (dm * dm_scale, dW1, dW2) of se_mlp_forward for the output gradient ds."""
    for t, n in ((m, "m"), (hid, "hid"), (s, "s"), (ds, "ds"), (w1, "w1"), (w2, "w2")):
        _check(t, n, "f")
    b, c = m.shape
    h = w1.shape[0]
    dm = torch.empty_like(m)
    dw1 = torch.empty_like(w1)
    dw2 = torch.empty_like(w2)
    _lib.call("pcfm_se_mlp_bwd", _ptr(m), _ptr(hid), _ptr(s), _ptr(ds), _ptr(w1), _ptr(w2), b, c,
              h, float(dm_scale), _ptr(dm), _ptr(dw1), _ptr(dw2), _stream(m))
    return dm, dw1, dw2


def rows_affine_(x: torch.Tensor, s: torch.Tensor, t) -> torch.Tensor:
    """x[r, :] = s[r] * x[r, :] + t[r] in place, x (rows, len) with len % 4 == 0."""
    _check(x, "x", "f")
    _check(s, "s", "f")
    if t is not None:
        _check(t, "t", "f")
    rows, length = x.shape
    if s.numel() != rows or (t is not None and t.numel() != rows):
        raise ValueError("rows_affine_: per-row parameters must have one value per row")
    with _timed("rows_affine", 8 * rows * length, x):
        _lib.call("pcfm_rows_affine", _ptr(x), _ptr(s), _ptr(t) if t is not None else None, rows,
                  length, _stream(x))
    return x


def trilinear_devoxelize_backward(grad_y: torch.Tensor, indices: torch.Tensor,
                                  weights: torch.Tensor, r: int):
    """trilinear_devox.cpp:67-91: grad_y (b,c,n) -> grad_x (b,c,r^3)"""
    if _host(grad_y, indices, weights):
        _check_host(grad_y, "grad_y", "f")
        _check_host(weights, "weights", "f")
        _check_host(indices, "indices", "i")
        return cpu_ops.trilinear_devoxelize_backward(grad_y, indices, weights, r)
    _check(grad_y, "grad_y", "f")
    _check(weights, "weights", "f")
    _check(indices, "indices", "i")
    b, c, n = grad_y.shape
    r = int(r)
    grad_x = torch.empty((b, c, r * r * r), dtype=torch.float32, device=grad_y.device)
    ws = _workspace(_lib.query("pcfm_trilinear_devoxelize_bwd_workspace_bytes", b, c, n, r),
                    grad_y)
    nbytes = 4 * b * (c * n + 16 * n + c * r ** 3)  # devox-bwd
    with _timed("trilinear_devoxelize_bwd", nbytes, grad_y):
        _lib.call("pcfm_trilinear_devoxelize_bwd", _ptr(grad_y), _ptr(indices), _ptr(weights),
                  b, c, n, r, _ptr(grad_x), _ptr(ws), ws.numel(), _stream(grad_y))
    return grad_x


def ball_query(centers_coords: torch.Tensor, points_coords: torch.Tensor, radius: float,
               num_neighbors: int):
    """ball_query.cpp:6-30: centers (b,3,m), points (b,3,n) -> idx i32 (b,m,u)"""
    if _host(centers_coords, points_coords):
        _check_host(centers_coords, "centers_coords", "f")
        _check_host(points_coords, "points_coords", "f")
        return cpu_ops.ball_query(centers_coords, points_coords, radius, num_neighbors)
    _check(centers_coords, "centers_coords", "f")
    _check(points_coords, "points_coords", "f")
    b, m = centers_coords.shape[0], centers_coords.shape[2]
    n = points_coords.shape[2]
    u = int(num_neighbors)
    idx = torch.zeros((b, m, u), dtype=torch.int32, device=centers_coords.device)
    _lib.call("pcfm_ball_query", _ptr(centers_coords), _ptr(points_coords), b, m, n,
              float(radius), u, _ptr(idx), _stream(centers_coords))
    return idx


def grouping_forward(features: torch.Tensor, indices: torch.Tensor):
    """grouping.cpp:6-22: features (b,c,n), indices (b,m,u) -> (b,c,m,u)"""
    if _host(features, indices):
        _check_host(features, "features", "f")
        _check_host(indices, "indices", "i")
        return cpu_ops.grouping_forward(features, indices)
    _check(features, "features", "f")
    _check(indices, "indices", "i")
    b, c, n = features.shape
    m, u = indices.shape[1], indices.shape[2]
    out = torch.empty((b, c, m, u), dtype=torch.float32, device=features.device)
    _lib.call("pcfm_grouping_fwd", _ptr(features), _ptr(indices), b, c, n, m, u, _ptr(out),
              _stream(features))
    return out


def grouping_backward(grad_y: torch.Tensor, indices: torch.Tensor, n: int):
    """grouping.cpp:24-44: grad_y (b,c,m,u) -> grad_x (b,c,n)"""
    if _host(grad_y, indices):
        _check_host(grad_y, "grad_y", "f")
        _check_host(indices, "indices", "i")
        return cpu_ops.grouping_backward(grad_y, indices, n)
    _check(grad_y, "grad_y", "f")
    _check(indices, "indices", "i")
    b, c = grad_y.shape[0], grad_y.shape[1]
    m, u = indices.shape[1], indices.shape[2]
    n = int(n)
    grad_x = torch.empty((b, c, n), dtype=torch.float32, device=grad_y.device)
    ws = _workspace(_lib.query("pcfm_grouping_bwd_workspace_bytes", b, c, n, m, u), grad_y)
    _lib.call("pcfm_grouping_bwd", _ptr(grad_y), _ptr(indices), b, c, n, m, u, _ptr(grad_x),
              _ptr(ws), ws.numel(), _stream(grad_y))
    return grad_x


def _out_of_scope(name):
    def f(*args, **kwargs):
        raise NotImplementedError(
            f"_pvcnn_backend.{name}: PointNet++ operator outside this build's hot path "
            "(SURVEY.md section 2.2: FPS / gather / 3-NN are used only by PointNet SA/FP "
            "modules, which the flow model never calls)")
    f.__name__ = name
    return f


backend = types.SimpleNamespace(
    avg_voxelize_forward=avg_voxelize_forward,
    avg_voxelize_backward=avg_voxelize_backward,
    trilinear_devoxelize_forward=trilinear_devoxelize_forward,
    trilinear_devoxelize_backward=trilinear_devoxelize_backward,
    ball_query=ball_query,
    grouping_forward=grouping_forward,
    grouping_backward=grouping_backward,
    gather_features_forward=_out_of_scope("gather_features_forward"),
    gather_features_backward=_out_of_scope("gather_features_backward"),
    furthest_point_sampling=_out_of_scope("furthest_point_sampling"),
    three_nearest_neighbors_interpolate_forward=_out_of_scope(
        "three_nearest_neighbors_interpolate_forward"),
    three_nearest_neighbors_interpolate_backward=_out_of_scope(
        "three_nearest_neighbors_interpolate_backward"),
)


# --------------------------------------------------------------------------
# chamfer_3D (chamfer_cuda.cpp:17-32): caller-allocated outputs, int status
# --------------------------------------------------------------------------
def _chamfer_forward(xyz1, xyz2, dist1, dist2, idx1, idx2) -> int:
    try:
        host = _host(xyz1, xyz2, dist1, dist2, idx1, idx2)
        for t, nm, k in ((xyz1, "xyz1", "f"), (xyz2, "xyz2", "f"), (dist1, "dist1", "f"),
                         (dist2, "dist2", "f"), (idx1, "idx1", "i"), (idx2, "idx2", "i")):
            (_check_host if host else _check)(t, nm, k)
        if host:
            cpu_ops.chamfer_forward(xyz1, xyz2, dist1, dist2, idx1, idx2)
            return 1
        b, n, m = xyz1.shape[0], xyz1.shape[1], xyz2.shape[1]
        ws = _workspace(_lib.query("pcfm_chamfer_workspace_bytes", b, n, m), xyz1)
        _lib.call("pcfm_chamfer_fwd", _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(dist1), _ptr(dist2),
                  _ptr(idx1), _ptr(idx2), _ptr(ws), ws.numel(), _stream(xyz1))
    except RuntimeError as e:  # the reference prints and returns 0 (chamfer3D.cu:145-151)
        print(f"error in nnd updateOutput: {e}")
        return 0
    return 1


def _chamfer_backward(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1, idx2) -> int:
    try:
        host = _host(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1, idx2)
        for t, nm, k in ((xyz1, "xyz1", "f"), (xyz2, "xyz2", "f"), (gradxyz1, "gradxyz1", "f"),
                         (gradxyz2, "gradxyz2", "f"), (graddist1, "graddist1", "f"),
                         (graddist2, "graddist2", "f"), (idx1, "idx1", "i"), (idx2, "idx2", "i")):
            (_check_host if host else _check)(t, nm, k)
        if host:
            cpu_ops.chamfer_backward(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1,
                                     idx2)
            return 1
        b, n, m = xyz1.shape[0], xyz1.shape[1], xyz2.shape[1]
        _lib.call("pcfm_chamfer_bwd", _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(graddist1),
                  _ptr(graddist2), _ptr(idx1), _ptr(idx2), _ptr(gradxyz1), _ptr(gradxyz2),
                  _stream(xyz1))
    except RuntimeError as e:
        print(f"error in nnd get grad: {e}")
        return 0
    return 1


chamfer_3D = types.SimpleNamespace(forward=_chamfer_forward, backward=_chamfer_backward)


# --------------------------------------------------------------------------
# emd_cuda (PyTorchEMD/cuda/emd.cpp:8-27): float and double
# --------------------------------------------------------------------------
def _emd_check(xyz1, xyz2):
    if xyz2.shape[0] != xyz1.shape[0] or xyz1.shape[2] != 3 or xyz2.shape[2] != 3:
        raise RuntimeError(f"emd: expected (B,N,3) and (B,M,3), got {tuple(xyz1.shape)} "
                           f"and {tuple(xyz2.shape)}")
    if xyz1.dtype not in (torch.float32, torch.float64) or xyz2.dtype != xyz1.dtype:
        raise RuntimeError("emd: xyz1/xyz2 must both be float32 or both float64")


def _emd_args(xyz1, xyz2):
    _check_cuda(xyz1, "xyz1")
    _check_cuda(xyz2, "xyz2")
    _emd_check(xyz1, xyz2)
    sfx = "f32" if xyz1.dtype == torch.float32 else "f64"
    b, n, m = xyz1.shape[0], xyz1.shape[1], xyz2.shape[1]
    ws = _workspace(_lib.query("pcfm_emd_workspace_bytes", b, n, m, xyz1.element_size()), xyz1)
    return sfx, b, n, m, ws


def approxmatch_forward(xyz1: torch.Tensor, xyz2: torch.Tensor) -> torch.Tensor:
    """emd_kernel.cu:169-191: -> match (B, M, N)"""
    xyz1, xyz2 = xyz1.contiguous(), xyz2.contiguous()
    if _host(xyz1, xyz2):
        _emd_check(xyz1, xyz2)
        return cpu_ops.approxmatch_forward(xyz1, xyz2)
    sfx, b, n, m, ws = _emd_args(xyz1, xyz2)
    match = torch.empty((b, m, n), dtype=xyz1.dtype, device=xyz1.device)
    if n == 0 or m == 0:
        return match.zero_()
    _lib.call(f"pcfm_emd_approxmatch_{sfx}", _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(match),
              _ptr(ws), ws.numel(), _stream(xyz1))
    return match


def matchcost_forward(xyz1: torch.Tensor, xyz2: torch.Tensor, match: torch.Tensor):
    """emd_kernel.cu:255-277: -> cost (B,)"""
    xyz1, xyz2, match = xyz1.contiguous(), xyz2.contiguous(), match.contiguous()
    if _host(xyz1, xyz2, match):
        _emd_check(xyz1, xyz2)
        return cpu_ops.matchcost_forward(xyz1, xyz2, match)
    sfx, b, n, m, ws = _emd_args(xyz1, xyz2)
    cost = torch.empty((b,), dtype=xyz1.dtype, device=xyz1.device)
    _lib.call(f"pcfm_emd_matchcost_{sfx}", _ptr(xyz1), _ptr(xyz2), _ptr(match), b, n, m,
              _ptr(cost), _ptr(ws), ws.numel(), _stream(xyz1))
    return cost


def approxmatch_cost_forward(xyz1: torch.Tensor, xyz2: torch.Tensor, want_match: bool = True):
    """approxmatch_forward + matchcost_forward in one native call (the forward
    of PyTorchEMD/emd.py:14-19): -> (match (B, M, N) or None, cost (B,)).  The
    cost is summed from the match kernel's own values; want_match=False skips
    writing match (a forward whose inputs need no gradient)."""
    xyz1, xyz2 = xyz1.contiguous(), xyz2.contiguous()
    if _host(xyz1, xyz2):
        _emd_check(xyz1, xyz2)
        match = cpu_ops.approxmatch_forward(xyz1, xyz2)
        return (match if want_match else None), cpu_ops.matchcost_forward(xyz1, xyz2, match)
    sfx, b, n, m, ws = _emd_args(xyz1, xyz2)
    match = torch.empty((b, m, n), dtype=xyz1.dtype, device=xyz1.device) if want_match else None
    cost = torch.empty((b,), dtype=xyz1.dtype, device=xyz1.device)
    _lib.call(f"pcfm_emd_approxmatch_cost_{sfx}", _ptr(xyz1), _ptr(xyz2), b, n, m,
              _ptr(match) if match is not None else None, _ptr(cost), _ptr(ws), ws.numel(),
              _stream(xyz1))
    return match, cost


def matchcost_backward(grad_cost: torch.Tensor, xyz1: torch.Tensor, xyz2: torch.Tensor,
                       match: torch.Tensor):
    """emd_kernel.cu:371-396: -> [grad1 (B,N,3), grad2 (B,M,3)]"""
    xyz1, xyz2, match = xyz1.contiguous(), xyz2.contiguous(), match.contiguous()
    grad_cost = grad_cost.contiguous().to(xyz1.dtype)
    if _host(grad_cost, xyz1, xyz2, match):
        _emd_check(xyz1, xyz2)
        return cpu_ops.matchcost_backward(grad_cost, xyz1, xyz2, match)
    sfx, b, n, m, ws = _emd_args(xyz1, xyz2)
    g1 = torch.empty((b, n, 3), dtype=xyz1.dtype, device=xyz1.device)
    g2 = torch.empty((b, m, 3), dtype=xyz1.dtype, device=xyz1.device)
    _lib.call(f"pcfm_emd_matchcost_bwd_{sfx}", _ptr(grad_cost), _ptr(xyz1), _ptr(xyz2),
              _ptr(match), b, n, m, _ptr(g1), _ptr(g2), _ptr(ws), ws.numel(), _stream(xyz1))
    return [g1, g2]


emd_cuda = types.SimpleNamespace(approxmatch_forward=approxmatch_forward,
                                 matchcost_forward=matchcost_forward,
                                 matchcost_backward=matchcost_backward)


def host_routed(ext, host, names):
    """A binding namespace that calls the torch C++ extension `ext` (HIP tensors
    only: csrc/torch_backend.cpp, torch_losses.cpp) and sends a call whose tensor
    arguments are all CPU tensors to `host` (this module's binding, which runs
    them on pcfm.cpu_ops, BASELINE configs[0]) -- so PCFM_TORCH_BACKEND=1 keeps the
    CPU path working.  `.extension` is the extension module itself."""
    def route(name):
        on_dev, on_host = getattr(ext, name), getattr(host, name)

        def call(*args):
            ts = [a for a in args if isinstance(a, torch.Tensor)]
            return (on_host if ts and not any(t.is_cuda for t in ts) else on_dev)(*args)
        call.__name__ = name
        return call
    ns = types.SimpleNamespace(**{n: route(n) for n in names})
    ns.extension = ext
    return ns


# --------------------------------------------------------------------------
# Voxel convolution (PVConv's Conv3d k=3 s=1 p=1) on the bf16x3 matrix-core
# path -- include/pcfm.h "Voxel convolution".
# --------------------------------------------------------------------------
def conv3d_wgrad_supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    b, cin, r = x.shape[0], x.shape[1], x.shape[2]
    return _lib.query("pcfm_conv3d_wgrad_workspace_bytes", b, cin, weight.shape[0], r) > 0


def conv3d_supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    """True if the bf16x3 implicit GEMM handles this (input, weight) pair."""
    if x.dim() != 5 or weight.dim() != 5 or tuple(weight.shape[2:]) != (3, 3, 3):
        return False
    b, cin, d, hh, ww = x.shape
    if not (d == hh == ww) or weight.shape[1] != cin:
        return False
    cout = weight.shape[0]
    return bool(_lib.query("pcfm_conv3d_supported", b, cin, cout, d)) and \
        bool(_lib.query("pcfm_conv3d_supported", b, cout, cin, d))


def conv3d_prep_weight(weight: torch.Tensor, transpose: bool) -> torch.Tensor:
    """Split + rearrange a (Cout, Cin, 3, 3, 3) fp32 kernel into the bf16 hi/lo image."""
    _check(weight, "weight", "f")
    cout, cin = weight.shape[0], weight.shape[1]
    w = weight.contiguous()
    img = torch.empty(_lib.query("pcfm_conv3d_weight_bytes", cout, cin), dtype=torch.uint8,
                      device=weight.device)
    _lib.call("pcfm_conv3d_prep_weight", _ptr(w), cout, cin, int(transpose), _ptr(img),
              _stream(w))
    return img


def conv3d_forward(x: torch.Tensor, weight: torch.Tensor, bias) -> torch.Tensor:
    """y = conv3d(x, weight, bias, stride 1, padding 1) (NCDHW fp32)."""
    _check(x, "input", "f")
    x = x.contiguous()
    b, cin, r = x.shape[0], x.shape[1], x.shape[2]
    cout = weight.shape[0]
    img = conv3d_prep_weight(weight, False)
    y = torch.empty((b, cout, r, r, r), dtype=torch.float32, device=x.device)
    bias_p = _ptr(bias.contiguous()) if bias is not None else None
    ws = _workspace(_lib.query("pcfm_conv3d_igemm_workspace_bytes", b, cin, cout, r), x)
    with _timed("conv3d_fwd", 54 * b * r ** 3 * cin * cout, x, "mfma"):
        _lib.call("pcfm_conv3d_igemm", _ptr(x), _ptr(img), bias_p, b, cin, cout, r, _ptr(y),
                  _ptr(ws), ws.numel(), _stream(x))
    return y


def conv3d_backward_data(grad_y: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """dL/dx of conv3d(x, weight, padding 1) for dL/dy = grad_y."""
    _check(grad_y, "grad_output", "f")
    g = grad_y.contiguous()
    b, cout, r = g.shape[0], g.shape[1], g.shape[2]
    cin = weight.shape[1]
    img = conv3d_prep_weight(weight, True)
    dx = torch.empty((b, cin, r, r, r), dtype=torch.float32, device=g.device)
    ws = _workspace(_lib.query("pcfm_conv3d_igemm_workspace_bytes", b, cout, cin, r), g)
    with _timed("conv3d_bwd_data", 54 * b * r ** 3 * cin * cout, g, "mfma"):
        _lib.call("pcfm_conv3d_igemm", _ptr(g), _ptr(img), None, b, cout, cin, r, _ptr(dx),
                  _ptr(ws), ws.numel(), _stream(g))
    return dx


def conv3d_backward_weight(x: torch.Tensor, grad_y: torch.Tensor) -> torch.Tensor:
    """dL/dW (Cout, Cin, 3, 3, 3) of conv3d(x, W, padding 1) for dL/dy = grad_y."""
    _check(x, "input", "f")
    _check(grad_y, "grad_output", "f")
    x, g = x.contiguous(), grad_y.contiguous()
    b, cin, r = x.shape[0], x.shape[1], x.shape[2]
    cout = g.shape[1]
    ws = _workspace(_lib.query("pcfm_conv3d_wgrad_workspace_bytes", b, cin, cout, r), x)
    dw = torch.empty((cout, cin, 3, 3, 3), dtype=torch.float32, device=x.device)
    with _timed("conv3d_wgrad", 54 * b * r ** 3 * cin * cout, x, "mfma"):
        _lib.call("pcfm_conv3d_wgrad", _ptr(x), _ptr(g), b, cin, cout, r, _ptr(dw), _ptr(ws),
                  ws.numel(), _stream(x))
    return dw


def conv3d_split(x: torch.Tensor) -> torch.Tensor:
    """Channels-last bf16 hi/lo split of a (B, C, R, R, R) fp32 tensor
    (pcfm_conv3d_split); opaque uint8 storage for the split-operand entry points."""
    _check(x, "input", "f")
    b, c, r = x.shape[0], x.shape[1], x.shape[2]
    n = _lib.query("pcfm_conv3d_split_bytes", b, c, r)
    if n == 0:
        raise RuntimeError(f"conv3d_split: unsupported shape {tuple(x.shape)}")
    xs = torch.empty(n, dtype=torch.uint8, device=x.device)
    _lib.call("pcfm_conv3d_split", _ptr(x), b, c, r, _ptr(xs), _stream(x))
    return xs


def conv3d_split_supported(x: torch.Tensor) -> bool:
    return _lib.query("pcfm_conv3d_split_bytes", x.shape[0], x.shape[1], x.shape[2]) > 0


def conv3d_occupancy(cnt: torch.Tensor, r: int):
    """Occupancy masks of a voxelized grid from the voxelization's counts cnt
    (b, r^3) int32 (pcfm_conv3d_occupancy), or None where r^3 % 256 != 0."""
    _check(cnt, "cnt", "i")
    b = cnt.shape[0]
    n = _lib.query("pcfm_conv3d_occupancy_bytes", b, int(r))
    if n == 0:
        return None
    masks = torch.empty(n // 4, dtype=torch.int32, device=cnt.device)
    _lib.call("pcfm_conv3d_occupancy", _ptr(cnt), b, int(r), _ptr(masks), _stream(cnt))
    return masks


def conv3d_vlists(cnt: torch.Tensor, r: int):
    """Voxel lists of a voxelized grid from the voxelization's counts cnt (b, r^3)
    int32 (pcfm_conv3d_vlist: occupied voxels, and voxels with an occupied
    neighbour), or None where r^3 % 256 != 0."""
    _check(cnt, "cnt", "i")
    b = cnt.shape[0]
    n = _lib.query("pcfm_conv3d_vlist_bytes", b, int(r))
    if n == 0:
        return None
    lists = torch.empty(n // 4, dtype=torch.int32, device=cnt.device)
    _lib.call("pcfm_conv3d_vlist", _ptr(cnt), b, int(r), _ptr(lists), _stream(cnt))
    return lists


def conv3d_igemm_split(xs: torch.Tensor, img: torch.Tensor, bias, b: int, cin: int, cout: int,
                       r: int, op: str, occ=None, occ_mode: int = 0, vlists=None,
                       cnt=None) -> torch.Tensor:
    """y (b, cout, r, r, r) from a split input (forward, or backward-data with the
    transposed weight image).  occ (conv3d_occupancy of the voxelized input /
    gradient target) with occ_mode 1 (forward) / 2 (backward-data) skips the
    exact-zero / unread work (pcfm_conv3d_igemm_cl_occ); with the grid's voxel
    lists (conv3d_vlists) and counts the GEMM runs at the listed voxels only
    (pcfm_conv3d_igemm_cl_list: mode 1 -> the neighbourhood-occupied voxels,
    bias elsewhere; mode 2 -> the occupied voxels, 0 elsewhere)."""
    y = torch.empty((b, cout, r, r, r), dtype=torch.float32, device=xs.device)
    bias_p = _ptr(bias.contiguous()) if bias is not None else None
    ws = _workspace(_lib.query("pcfm_conv3d_igemm_cl_workspace_bytes", b, cin, cout, r), xs)
    if occ_mode and (occ is not None or vlists is not None):
        op = op + "_sparse"  # skips work: timed apart from the dense launches (roofline)
    with _timed(op, 54 * b * r ** 3 * cin * cout, xs, "mfma"):
        if vlists is not None and cnt is not None and occ_mode in (1, 2):
            _lib.call("pcfm_conv3d_igemm_cl_list", _ptr(xs), _ptr(img), bias_p, b, cin, cout, r,
                      _ptr(cnt), _ptr(vlists), 1 if occ_mode == 1 else 0, _ptr(y), _ptr(ws),
                      ws.numel(), _stream(xs))
        elif occ is not None and occ_mode:
            _lib.call("pcfm_conv3d_igemm_cl_occ", _ptr(xs), _ptr(img), bias_p, b, cin, cout, r,
                      _ptr(occ), int(occ_mode), _ptr(y), _ptr(ws), ws.numel(), _stream(xs))
        else:
            _lib.call("pcfm_conv3d_igemm_cl", _ptr(xs), _ptr(img), bias_p, b, cin, cout, r,
                      _ptr(y), _ptr(ws), ws.numel(), _stream(xs))
    return y


def conv3d_wgrad_split(xs: torch.Tensor, gys: torch.Tensor, b: int, cin: int, cout: int,
                       r: int, occ=None) -> torch.Tensor:
    """dW (cout, cin, 3, 3, 3) from split(x) and split(grad_y); occ (the
    occupancy masks of a voxelized x) skips the steps whose X rows are empty."""
    q = "pcfm_conv3d_wgrad_occ_workspace_bytes" if occ is not None else \
        "pcfm_conv3d_wgrad_workspace_bytes"
    ws = _workspace(_lib.query(q, b, cin, cout, r), xs)
    dw = torch.empty((cout, cin, 3, 3, 3), dtype=torch.float32, device=xs.device)
    with _timed("conv3d_wgrad_sparse" if occ is not None else "conv3d_wgrad",
                54 * b * r ** 3 * cin * cout, xs, "mfma"):
        if occ is not None:
            _lib.call("pcfm_conv3d_wgrad_cl_occ", _ptr(xs), _ptr(gys), b, cin, cout, r, _ptr(occ),
                      _ptr(dw), _ptr(ws), ws.numel(), _stream(xs))
        else:
            _lib.call("pcfm_conv3d_wgrad_cl", _ptr(xs), _ptr(gys), b, cin, cout, r, _ptr(dw),
                      _ptr(ws), ws.numel(), _stream(xs))
    return dw


# --------------------------------------------------------------------------
# Pointwise (1x1) convolution on the bf16x3 matrix-core path
# (include/pcfm.h "Pointwise convolution").  x, y are (B, C, N) fp32.
# --------------------------------------------------------------------------
def pointwise_prep_weight(weight: torch.Tensor, transpose: bool) -> torch.Tensor:
    _check(weight, "weight", "f")
    w = weight.reshape(weight.shape[0], -1).contiguous()
    cout, cin = w.shape
    img = torch.empty(_lib.query("pcfm_pointwise_weight_bytes", cout, cin), dtype=torch.uint8,
                      device=w.device)
    _lib.call("pcfm_pointwise_prep_weight", _ptr(w), cout, cin, int(transpose), _ptr(img),
              _stream(w))
    return img


def pointwise_forward(x: torch.Tensor, weight: torch.Tensor, bias) -> torch.Tensor:
    """y = Conv1d(x; weight (Cout, Cin[, 1]), bias) for x (B, Cin, N)."""
    _check(x, "input", "f")
    x = x.contiguous()
    b, cin, n = x.shape
    cout = weight.shape[0]
    img = pointwise_prep_weight(weight, False)
    y = torch.empty((b, cout, n), dtype=torch.float32, device=x.device)
    bias_p = _ptr(bias.contiguous()) if bias is not None else None
    with _timed("pointwise_fwd", 2 * b * n * cin * cout, x, "mfma"):
        _lib.call("pcfm_pointwise_gemm", _ptr(x), _ptr(img), bias_p, b, cin, cout, n, _ptr(y),
                  _stream(x))
    return y


def pointwise_forward_bnstats(x: torch.Tensor, weight: torch.Tensor, bias):
    """pointwise_forward with the BatchNorm statistics of y from the GEMM's
    epilogue -> (y, stats f32 (Cout, P, 2)), or None for the shapes without that
    path (pcfm_pointwise_bnstats_groups)."""
    _check(x, "input", "f")
    x = x.contiguous()
    b, cin, n = x.shape
    cout = weight.shape[0]
    groups = _lib.query("pcfm_pointwise_bnstats_groups", b, cin, cout, n)
    if groups <= 0:
        return None
    img = pointwise_prep_weight(weight, False)
    y = torch.empty((b, cout, n), dtype=torch.float32, device=x.device)
    stats = torch.empty((cout, groups, 2), dtype=torch.float32, device=x.device)
    bias_p = _ptr(bias.contiguous()) if bias is not None else None
    with _timed("pointwise_fwd", 2 * b * n * cin * cout, x, "mfma"):
        _lib.call("pcfm_pointwise_gemm_bnstats", _ptr(x), _ptr(img), bias_p, b, cin, cout, n,
                  _ptr(y), _ptr(stats), _stream(x))
    return y, stats


def pointwise_backward_data(grad_y: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    _check(grad_y, "grad_output", "f")
    g = grad_y.contiguous()
    b, cout, n = g.shape
    cin = weight.shape[1]
    img = pointwise_prep_weight(weight, True)
    dx = torch.empty((b, cin, n), dtype=torch.float32, device=g.device)
    with _timed("pointwise_bwd_data", 2 * b * n * cin * cout, g, "mfma"):
        _lib.call("pcfm_pointwise_gemm", _ptr(g), _ptr(img), None, b, cout, cin, n, _ptr(dx),
                  _stream(g))
    return dx


def pointwise_backward_weight(x: torch.Tensor, grad_y: torch.Tensor) -> torch.Tensor:
    """dL/dW (Cout, Cin) of y = W x."""
    _check(x, "input", "f")
    _check(grad_y, "grad_output", "f")
    x, g = x.contiguous(), grad_y.contiguous()
    b, cin, n = x.shape
    cout = g.shape[1]
    ws = _workspace(_lib.query("pcfm_pointwise_wgrad_workspace_bytes", b, cin, cout, n), x)
    dw = torch.empty((cout, cin), dtype=torch.float32, device=x.device)
    with _timed("pointwise_wgrad", 2 * b * n * cin * cout, x, "mfma"):
        _lib.call("pcfm_pointwise_wgrad", _ptr(x), _ptr(g), b, cin, cout, n, _ptr(dw), _ptr(ws),
                  ws.numel(), _stream(x))
    return dw


def _parts(ts):
    """Host pointer / width arrays of a channel-segmented tensor list."""
    ptrs = (ctypes.c_void_p * len(ts))(*[_ptr(t) for t in ts])
    widths = (ctypes.c_int * len(ts))(*[int(t.shape[1]) for t in ts])
    return ptrs, widths


def pointwise_forward_parts(xs, weight: torch.Tensor, bias, bias_per_batch: bool = False):
    """y = W cat(xs, 1) + bias without materialising the concat; xs (B, C_i, N)
    fp32 (every C_i but the last a multiple of 32), bias (Cout,) or, with
    bias_per_batch, (B, Cout)."""
    xs = [x.contiguous() for x in xs]
    for x in xs:
        _check(x, "input", "f")
    b, _, n = xs[0].shape
    cin = sum(int(x.shape[1]) for x in xs)
    cout = weight.shape[0]
    weight = weight.reshape(cout, -1).contiguous()
    if weight.shape[1] != cin:
        raise ValueError("pointwise_forward_parts: weight does not match the parts")
    img = pointwise_prep_weight(weight, False)
    y = torch.empty((b, cout, n), dtype=torch.float32, device=xs[0].device)
    bias_c = bias.contiguous() if bias is not None else None
    xp, xw = _parts(xs)
    yp, yw = _parts([y])
    with _timed("pointwise_fwd", 2 * b * n * cin * cout, xs[0], "mfma"):
        _lib.call("pcfm_pointwise_gemm_parts", len(xs), ctypes.addressof(xp), ctypes.addressof(xw),
                  _ptr(img), _ptr(bias_c) if bias_c is not None else None, int(bias_per_batch),
                  b, n, 1, ctypes.addressof(yp), ctypes.addressof(yw), _stream(xs[0]))
    return y


def pointwise_backward_data_parts(grad_y: torch.Tensor, weight: torch.Tensor, widths):
    """dx parts (B, w_i, N) of y = W cat(parts); every width but the last % 128."""
    _check(grad_y, "grad_output", "f")
    g = grad_y.contiguous()
    b, cout, n = g.shape
    weight = weight.reshape(cout, -1).contiguous()
    cin = weight.shape[1]
    if sum(widths) != cin:
        raise ValueError("pointwise_backward_data_parts: widths do not match the weight")
    img = pointwise_prep_weight(weight, True)
    dxs = [torch.empty((b, w, n), dtype=torch.float32, device=g.device) for w in widths]
    gp, gw = _parts([g])
    dp, dw = _parts(dxs)
    with _timed("pointwise_bwd_data", 2 * b * n * cin * cout, g, "mfma"):
        _lib.call("pcfm_pointwise_gemm_parts", 1, ctypes.addressof(gp), ctypes.addressof(gw),
                  _ptr(img), None, 0, b, n, len(dxs), ctypes.addressof(dp), ctypes.addressof(dw),
                  _stream(g))
    return dxs


def pointwise_backward_weight_parts(xs, grad_y: torch.Tensor) -> torch.Tensor:
    """dL/dW (Cout, sum C_i) of y = W cat(xs, 1)."""
    xs = [x.contiguous() for x in xs]
    for x in xs:
        _check(x, "input", "f")
    _check(grad_y, "grad_output", "f")
    g = grad_y.contiguous()
    b, _, n = xs[0].shape
    cin = sum(int(x.shape[1]) for x in xs)
    cout = g.shape[1]
    ws = _workspace(_lib.query("pcfm_pointwise_wgrad_workspace_bytes", b, cin, cout, n), g)
    dw = torch.empty((cout, cin), dtype=torch.float32, device=g.device)
    xp, xw = _parts(xs)
    with _timed("pointwise_wgrad", 2 * b * n * cin * cout, g, "mfma"):
        _lib.call("pcfm_pointwise_wgrad_parts", len(xs), ctypes.addressof(xp),
                  ctypes.addressof(xw), _ptr(g), b, cout, n, _ptr(dw), _ptr(ws), ws.numel(),
                  _stream(g))
    return dw


# --------------------------------------------------------------------------
# Per-point head: bf16 Linear weight gradient over B*N rows
# (include/pcfm.h "Per-point head").
# --------------------------------------------------------------------------
def rows_wgrad_bf16(grad_y: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW (M, N) bf16 = grad_y^T @ x for grad_y (R, M), x (R, N) bf16 row-major
    (unit column stride; row strides may exceed the width)."""
    for t, name in ((grad_y, "grad_y"), (x, "x")):
        _check_cuda(t, name)
        if t.dtype != torch.bfloat16 or t.dim() != 2 or t.stride(1) != 1:
            raise RuntimeError(f"rows_wgrad_bf16: {name} must be a 2-D bf16 row-major tensor")
    rows, m = grad_y.shape
    n = x.shape[1]
    if x.shape[0] != rows:
        raise RuntimeError(f"rows_wgrad_bf16: row mismatch {rows} vs {x.shape[0]}")
    out = torch.empty((m, n), dtype=torch.bfloat16, device=x.device)
    ws = _workspace(_lib.query("pcfm_rows_wgrad_workspace_bytes", rows, m, n), x)
    with _timed("rows_wgrad_bf16", 2 * rows * m * n, x, "mfma_bf16"):
        _lib.call("pcfm_rows_wgrad_bf16", _ptr(grad_y), grad_y.stride(0), _ptr(x), x.stride(0),
                  rows, m, n, _ptr(out), _ptr(ws), ws.numel(), _stream(x))
    return out


def _p(t):
    return t.data_ptr() if t is not None else None


def rows_colsum(x: torch.Tensor) -> torch.Tensor:
    """x (B, R, C) or (R, C), bf16 or fp32 -> fp32 (B, C) / (C,) sums over R
    (include/pcfm.h pcfm_rows_colsum)."""
    squeeze = x.dim() == 2
    x3 = x.unsqueeze(0) if squeeze else x
    x3 = x3.contiguous()
    b, rows, c = x3.shape
    if x3.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError("rows_colsum: bf16 or fp32 input")
    out = torch.empty((b, c), dtype=torch.float32, device=x3.device)
    ws = _workspace(_lib.query("pcfm_rows_colsum_workspace_bytes", b, rows, c), x3)
    with _timed("rows_colsum", x3.numel() * x3.element_size(), x3):
        _lib.call("pcfm_rows_colsum", _ptr(x3), int(x3.dtype == torch.bfloat16), b, rows, c,
                  _ptr(out), _ptr(ws), ws.numel(), _stream(x3))
    return out[0] if squeeze else out


def colsum_ok(x: torch.Tensor) -> bool:
    c = x.shape[-1]
    return (x.is_cuda and x.dim() in (2, 3) and x.dtype in (torch.bfloat16, torch.float32)
            and c % 2 == 0 and 0 < c <= 512)


def tgate_forward(head: torch.Tensor, glb: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    """head (B, C, N), glb (B, C), alpha (B,) fp32 -> (B, N, C) blend."""
    for tns, nm in ((head, "head"), (glb, "glb"), (alpha, "alpha")):
        _check(tns, nm, "f")
    b, c, n = head.shape
    out = torch.empty((b, n, c), dtype=torch.float32, device=head.device)
    with _timed("tgate_fwd", 8 * b * c * n, head):
        _lib.call("pcfm_tgate_fwd", _ptr(head), _ptr(glb), _ptr(alpha), b, c, n, _ptr(out),
                  _stream(head))
    return out


def tgate_backward(dout: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    """dout (B, N, C) -> dhead (B, C, N) = alpha[b] * dout^T."""
    dout = dout.contiguous()
    _check(dout, "dout", "f")
    b, n, c = dout.shape
    dhead = torch.empty((b, c, n), dtype=torch.float32, device=dout.device)
    with _timed("tgate_bwd", 8 * b * c * n, dout):
        _lib.call("pcfm_tgate_bwd", _ptr(dout), _ptr(alpha), b, c, n, _ptr(dhead), _stream(dout))
    return dhead


def head_film_fwd(h16, uprev, gprev, gamma, beta, sp1, shift, n: int, eps: float, hbias=None):
    """One FiLM block row pass (include/pcfm.h pcfm_head_film_fwd); hbias (B, W) f32
    is the per-batch input bias added to h16.
    Returns u f32 (R, W), a bf16 (R, W), mean f32 (R,), rstd f32 (R,)."""
    ref = h16 if h16 is not None else uprev
    rows, w = ref.shape
    b = rows // n
    dev = ref.device
    u = torch.empty((rows, w), dtype=torch.float32, device=dev)
    a = torch.empty((rows, w), dtype=torch.bfloat16, device=dev)
    mean = torch.empty((rows,), dtype=torch.float32, device=dev)
    rstd = torch.empty((rows,), dtype=torch.float32, device=dev)
    with _timed("head_film_fwd", rows * w * (2 if h16 is not None else 6) + rows * w * 6, ref):
        _lib.call("pcfm_head_film_fwd", _p(h16), _p(hbias), _p(uprev), _p(gprev), _p(gamma),
                  _p(beta),
                  _p(sp1), _p(shift), b, n, w, float(eps), _p(u), _p(a), _p(mean), _p(rstd),
                  _stream(ref))
    return u, a, mean, rstd


def head_silu_fwd(uprev, gprev, n: int):
    rows, w = uprev.shape
    a = torch.empty((rows, w), dtype=torch.bfloat16, device=uprev.device)
    _lib.call("pcfm_head_silu_fwd", _p(uprev), _p(gprev), rows // n, n, w, _p(a),
              _stream(uprev))
    return a


def head_film_bwd(dh_next, da16, u, h16, uprev, gprev, mean, rstd, gamma, beta, sp1, n: int,
                  want_dh: bool, hbias=None, shift=None):
    """Returns dh f32 (or None), dh16 bf16, dsp1 f32 (B, W), dshift f32 (B, W),
    dgamma f32 (W,), dbeta f32 (W,), dbias f32 (W,), and with hbias (h16's per-batch
    input bias) its gradient dbias_b f32 (B, W) as an 8th value.  u may be None when
    shift (the forward's bf16 (B, W) shift) is given: the kernel recomputes it."""
    rows, w = da16.shape
    b = rows // n
    dev = da16.device
    dh = torch.empty((rows, w), dtype=torch.float32, device=dev) if want_dh else None
    dh16 = torch.empty((rows, w), dtype=torch.bfloat16, device=dev)
    small = torch.empty((3 * b + 3, w), dtype=torch.float32, device=dev)
    dsp1, dshift = small[:b], small[b:2 * b]
    dgamma, dbeta, dbias = small[2 * b], small[2 * b + 1], small[2 * b + 2]
    dbias_b = small[2 * b + 3:] if hbias is not None else None
    ws = _workspace(_lib.query("pcfm_head_bwd_workspace_bytes", b, n, w), da16)
    if u is None and shift is None:
        raise ValueError("head_film_bwd: need u or shift")
    with _timed("head_film_bwd", rows * w * (4 + 2 + (4 if u is not None else 0)
                                             + (2 if h16 is not None else 6)
                                             + (4 if want_dh else 0) + 2), da16):
        _lib.call("pcfm_head_film_bwd", _p(dh_next), _p(da16), _p(u), _p(h16), _p(hbias),
                  _p(uprev), _p(gprev), _p(mean), _p(rstd), _p(gamma), _p(beta), _p(sp1),
                  _p(shift), b, n,
                  w, _p(dh), _p(dh16), _p(dsp1), _p(dshift), _p(dgamma), _p(dbeta), _p(dbias),
                  _p(dbias_b), _p(ws), ws.numel(), _stream(da16))
    if hbias is not None:
        return dh, dh16, dsp1, dshift, dgamma, dbeta, dbias, dbias_b
    return dh, dh16, dsp1, dshift, dgamma, dbeta, dbias


def head_silu_bwd(da16, uprev, gprev, n: int):
    """Returns dh f32, dh16 bf16, dbias f32 (W,)."""
    rows, w = da16.shape
    b = rows // n
    dev = da16.device
    dh = torch.empty((rows, w), dtype=torch.float32, device=dev)
    dh16 = torch.empty((rows, w), dtype=torch.bfloat16, device=dev)
    dbias = torch.empty((w,), dtype=torch.float32, device=dev)
    ws = _workspace(_lib.query("pcfm_head_bwd_workspace_bytes", b, n, w), da16)
    _lib.call("pcfm_head_silu_bwd", _p(da16), _p(uprev), _p(gprev), b, n, w, _p(dh), _p(dh16),
              _p(dbias), _p(ws), ws.numel(), _stream(da16))
    return dh, dh16, dbias


# --------------------------------------------------------------------------
# BatchNorm (batch statistics) + ReLU / LeakyReLU (include/pcfm.h)
# --------------------------------------------------------------------------
def _counter(t, like: torch.Tensor):
    """A BatchNorm num_batches_tracked buffer the kernel may increment: int64, one
    element, on the input's device (None passes through)."""
    if t is None:
        return None
    if t.dtype != torch.int64 or t.numel() != 1 or t.device != like.device:
        raise RuntimeError("num_batches_tracked: expected a one-element int64 tensor on the "
                           "input's device")
    return t


def bn_act_forward(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float,
                   slope: float, momentum: float, running_mean, running_var,
                   num_batches_tracked=None):
    """x (B, C, ...) fp32 contiguous -> (y, mean, invstd); running stats (and the int64
    num_batches_tracked counter, +1) updated in place."""
    _check(x, "input", "f")
    b, c = x.shape[0], x.shape[1]
    s = x.numel() // max(1, b * c)
    y = torch.empty_like(x)
    stats = torch.empty((2, c), dtype=torch.float32, device=x.device)
    ws = _workspace(_lib.query("pcfm_bn_workspace_bytes", b, c, s), x)
    with _timed("bn_act_fwd", 4 * 3 * x.numel(), x):
        _lib.call("pcfm_bn_act_fwd", _ptr(x), _ptr(weight), _ptr(bias), b, c, s, float(eps),
                  float(slope), float(momentum), _p(running_mean), _p(running_var),
                  _p(_counter(num_batches_tracked, x)), _ptr(y),
                  _ptr(stats[0]), _ptr(stats[1]), _ptr(ws), ws.numel(), _stream(x))
    return y, stats[0], stats[1]


def bn_act_forward_parts(x: torch.Tensor, stats: torch.Tensor, weight: torch.Tensor,
                         bias: torch.Tensor, eps: float, slope: float, momentum: float,
                         running_mean, running_var, num_batches_tracked=None):
    """bn_act_forward for x whose statistics came out of its producer
    (pointwise_forward_bnstats): the finalize + apply only -> (y, mean, invstd)."""
    _check(x, "input", "f")
    _check(stats, "stats", "f")
    b, c = x.shape[0], x.shape[1]
    s = x.numel() // max(1, b * c)
    y = torch.empty_like(x)
    out = torch.empty((2, c), dtype=torch.float32, device=x.device)
    with _timed("bn_act_fwd", 4 * 2 * x.numel(), x):
        _lib.call("pcfm_bn_act_fwd_parts", _ptr(x), _ptr(stats), int(stats.shape[1]),
                  _ptr(weight), _ptr(bias), b, c, s, float(eps), float(slope), float(momentum),
                  _p(running_mean), _p(running_var), _p(_counter(num_batches_tracked, x)),
                  _ptr(y), _ptr(out[0]), _ptr(out[1]), _stream(x))
    return y, out[0], out[1]


def bn_act_forward_split(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float,
                         slope: float, momentum: float, running_mean, running_var,
                         num_batches_tracked=None):
    """bn_act_forward for a voxel conv output x (B, C, R, R, R) whose activation only
    feeds the next voxel conv: -> (split(act(bn(x))) as conv3d_split lays it out,
    mean, invstd); running stats updated in place."""
    _check(x, "input", "f")
    b, c, r = x.shape[0], x.shape[1], x.shape[2]
    s = x.numel() // max(1, b * c)
    n = _lib.query("pcfm_conv3d_split_bytes", b, c, r)
    if n == 0 or c % 64 != 0:
        raise RuntimeError(f"bn_act_forward_split: unsupported shape {tuple(x.shape)}")
    ys = torch.empty(n, dtype=torch.uint8, device=x.device)
    stats = torch.empty((2, c), dtype=torch.float32, device=x.device)
    ws = _workspace(_lib.query("pcfm_bn_workspace_bytes", b, c, s), x)
    with _timed("bn_act_fwd", 4 * 3 * x.numel(), x):
        _lib.call("pcfm_bn_act_fwd_split", _ptr(x), _ptr(weight), _ptr(bias), b, c, s,
                  float(eps), float(slope), float(momentum), _p(running_mean), _p(running_var),
                  _p(_counter(num_batches_tracked, x)), _ptr(ys), _ptr(stats[0]), _ptr(stats[1]),
                  _ptr(ws), ws.numel(), _stream(x))
    return ys, stats[0], stats[1]


def bn_act_backward(dz: torch.Tensor, x: torch.Tensor, weight, bias, mean, invstd, slope: float,
                    want_dbias_in: bool = False):
    """-> (dx, dgamma, dbeta, dbias_in) with dbias_in = sum of dx over (b, s) per
    channel (the producer's bias gradient) or None."""
    dz = dz.contiguous()
    b, c = x.shape[0], x.shape[1]
    s = x.numel() // max(1, b * c)
    dx = torch.empty_like(x)
    dgb = torch.empty((3, c), dtype=torch.float32, device=x.device)
    ws = _workspace(_lib.query("pcfm_bn_workspace_bytes", b, c, s), x)
    with _timed("bn_act_bwd", 4 * 5 * x.numel(), x):
        _lib.call("pcfm_bn_act_bwd", _ptr(dz), _ptr(x), _ptr(weight), _ptr(bias), _ptr(mean),
                  _ptr(invstd), b, c, s, float(slope), _ptr(dx), _ptr(dgb[0]), _ptr(dgb[1]),
                  _ptr(dgb[2]) if want_dbias_in else None, _ptr(ws), ws.numel(), _stream(x))
    return dx, dgb[0], dgb[1], (dgb[2] if want_dbias_in else None)


def bn_act_backward_split(dz: torch.Tensor, x: torch.Tensor, weight, bias, mean, invstd,
                          slope: float, want_dbias_in: bool = False):
    """bn_act_backward for a voxel conv output x (B, C, R, R, R) whose dx only feeds
    that conv's backward: -> (split(dx) as conv3d_split lays it out, dgamma, dbeta,
    dbias_in or None); dx is never materialised in fp32."""
    dz = dz.contiguous()
    b, c, r = x.shape[0], x.shape[1], x.shape[2]
    s = x.numel() // max(1, b * c)
    n = _lib.query("pcfm_conv3d_split_bytes", b, c, r)
    wsb = _lib.query("pcfm_bn_act_bwd_split_workspace_bytes", b, c, s)
    if n == 0 or wsb == 0:
        raise RuntimeError(f"bn_act_backward_split: unsupported shape {tuple(x.shape)}")
    dxs = torch.empty(n, dtype=torch.uint8, device=x.device)
    dgb = torch.empty((3, c), dtype=torch.float32, device=x.device)
    ws = _workspace(wsb, x)
    with _timed("bn_act_bwd", 4 * 5 * x.numel(), x):
        _lib.call("pcfm_bn_act_bwd_split", _ptr(dz), _ptr(x), _ptr(weight), _ptr(bias),
                  _ptr(mean), _ptr(invstd), b, c, s, float(slope), _ptr(dxs), _ptr(dgb[0]),
                  _ptr(dgb[1]), _ptr(dgb[2]) if want_dbias_in else None, _ptr(ws), ws.numel(),
                  _stream(x))
    return dxs, dgb[0], dgb[1], (dgb[2] if want_dbias_in else None)


# PVConv's second voxel BatchNorm + LeakyReLU fused with SE3d and the
# devoxelization (include/pcfm.h, ABI 19): act(bn(x)) is never written
def bn_act_forward_rowmean(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float,
                           slope: float, momentum: float, running_mean, running_var,
                           num_batches_tracked=None):
    """BatchNorm statistics of x (B, C, ...) (running stats updated) and the per-(b, c)
    mean of act(bn(x)) -- SE3d's pooling -- without writing act(bn(x)):
    -> (rowmean (B, C), mean, invstd)."""
    _check(x, "input", "f")
    b, c = x.shape[0], x.shape[1]
    s = x.numel() // max(1, b * c)
    rowmean = torch.empty((b, c), dtype=torch.float32, device=x.device)
    stats = torch.empty((2, c), dtype=torch.float32, device=x.device)
    ws = _workspace(_lib.query("pcfm_bn_act_fwd_rowmean_workspace_bytes", b, c, s), x)
    with _timed("bn_act_fwd", 4 * 2 * x.numel(), x):
        _lib.call("pcfm_bn_act_fwd_rowmean", _ptr(x), _ptr(weight), _ptr(bias), b, c, s,
                  float(eps), float(slope), float(momentum), _p(running_mean), _p(running_var),
                  _p(_counter(num_batches_tracked, x)), _ptr(rowmean), _ptr(stats[0]),
                  _ptr(stats[1]), _ptr(ws), ws.numel(), _stream(x))
    return rowmean, stats[0], stats[1]


def trilinear_devoxelize_bn_scale_add(r: int, is_training: bool, coords: torch.Tensor,
                                      x: torch.Tensor, mean, invstd, weight, bias, slope: float,
                                      scale, add, add_bn=None):
    """trilinear_devoxelize_scale_add of act(bn(x)) with the given batch statistics;
    the activation is applied as the rows are staged -> [outs, inds, wgts].
    add_bn = (mean, invstd, weight, bias, slope) of the add operand: add enters as
    act(bn(add)) (PVConv's point-branch BatchNorm1d + ReLU, never written)."""
    _check(x, "x", "f")
    _check(coords, "coords", "f")
    b, c = x.shape[0], x.shape[1]
    n = coords.shape[2]
    r = int(r)
    dev = x.device
    for t, nm in ((mean, "mean"), (invstd, "invstd"), (weight, "weight"), (bias, "bias")):
        _check(t, nm, "f")
        if t.numel() != c:
            raise ValueError(f"trilinear_devoxelize_bn_scale_add: {nm} must have C values")
    if scale is not None:
        scale = scale.contiguous()
        _check(scale, "scale", "f")
        if scale.numel() != b * c:
            raise ValueError("trilinear_devoxelize_bn_scale_add: scale must be (B, C)")
    if add is not None:
        add = add.contiguous()
        _check(add, "add", "f")
        if tuple(add.shape) != (b, c, n):
            raise ValueError("trilinear_devoxelize_bn_scale_add: add must be (B, C, N)")
    outs = torch.empty((b, c, n), dtype=torch.float32, device=dev)
    if is_training:
        inds = torch.empty((b, 8, n), dtype=torch.int32, device=dev)
        wgts = torch.empty((b, 8, n), dtype=torch.float32, device=dev)
        pi, pw = _ptr(inds), _ptr(wgts)
    else:
        inds = torch.zeros((1,), dtype=torch.int32, device=dev)
        wgts = torch.zeros((1,), dtype=torch.float32, device=dev)
        pi, pw = None, None
    nbytes = 4 * b * (3 * n + c * r ** 3 + c * n * (2 if add is not None else 1)
                      + (16 * n if is_training else 0))
    abn = [None, None, None, None]
    aslope = 0.0
    if add_bn is not None:
        if add is None:
            raise ValueError("trilinear_devoxelize_bn_scale_add: add_bn without add")
        for t in add_bn[:4]:
            _check(t, "add_bn", "f")
            if t.numel() != c:
                raise ValueError("trilinear_devoxelize_bn_scale_add: add_bn entries must have C values")
        abn = [_ptr(t) for t in add_bn[:4]]
        aslope = float(add_bn[4])
    with _timed("trilinear_devoxelize_fwd", nbytes, x):
        _lib.call("pcfm_trilinear_devoxelize_bn_scale_add_fwd", _ptr(coords), _ptr(x), _ptr(mean),
                  _ptr(invstd), _ptr(weight), _ptr(bias), float(slope),
                  _ptr(scale) if scale is not None else None,
                  _ptr(add) if add is not None else None, *abn, aslope, b, c, n, r,
                  1 if is_training else 0, _ptr(outs), pi, pw, _stream(x))
    if devox_verify.enabled:
        devox_verify.bn(coords, x, (mean, invstd, weight, bias, slope), scale, add, add_bn, outs,
                        inds if is_training else None, wgts if is_training else None, r)
    return [outs, inds, wgts]


def bn_forward_stats(x: torch.Tensor, eps: float, momentum: float, running_mean, running_var,
                     num_batches_tracked=None, parts=None):
    """BatchNorm batch statistics of x (B, C, ...) only -> (mean, invstd); running stats
    and the counter updated.  parts: the producer's epilogue statistics
    (pointwise_forward_bnstats) instead of a statistics pass over x."""
    _check(x, "input", "f")
    b, c = x.shape[0], x.shape[1]
    s = x.numel() // max(1, b * c)
    stats = torch.empty((2, c), dtype=torch.float32, device=x.device)
    if parts is not None:
        _check(parts, "parts", "f")
        ws = _workspace(1, x)
        npart, nbytes = int(parts.shape[1]), 0
    else:
        ws = _workspace(_lib.query("pcfm_bn_workspace_bytes", b, c, s), x)
        npart, nbytes = 0, 4 * x.numel()
    with _timed("bn_act_fwd", nbytes, x):
        _lib.call("pcfm_bn_fwd_stats", _ptr(x), _ptr(parts) if parts is not None else None,
                  npart, b, c, s, float(eps), float(momentum), _p(running_mean),
                  _p(running_var), _p(_counter(num_batches_tracked, x)), _ptr(stats[0]),
                  _ptr(stats[1]), _ptr(ws), ws.numel(), _stream(x))
    return stats[0], stats[1]


def bn_se_backward_stats(g: torch.Tensor, x: torch.Tensor, mean, invstd, weight, bias,
                         slope: float) -> torch.Tensor:
    """rowstats (5, B, C): per (b, c) row of g (B, C, S) and x, with z = act(bn(x)),
    a = act'(bn(x)), xh = xhat: (sum z g, sum a g, sum a, sum a g xh, sum a xh)."""
    _check(g, "g", "f")
    _check(x, "x", "f")
    b, c = x.shape[0], x.shape[1]
    s = x.numel() // max(1, b * c)
    if g.shape != x.shape:
        raise ValueError("bn_se_backward_stats: g and x shapes differ")
    wsb = _lib.query("pcfm_bn_se_bwd_workspace_bytes", b, c, s)
    if wsb == 0:
        raise RuntimeError(f"bn_se_backward_stats: unsupported shape {tuple(x.shape)}")
    rowstats = torch.empty((5, b, c), dtype=torch.float32, device=x.device)
    ws = _workspace(wsb, x)
    with _timed("bn_act_bwd", 4 * 2 * x.numel(), x):
        _lib.call("pcfm_bn_se_bwd_stats", _ptr(g), _ptr(x), _ptr(mean), _ptr(invstd),
                  _ptr(weight), _ptr(bias), b, c, s, float(slope), _ptr(rowstats), _ptr(ws),
                  ws.numel(), _stream(x))
    return rowstats


def bn_se_backward_apply_split(g: torch.Tensor, x: torch.Tensor, mean, invstd, weight, bias,
                               se_scale: torch.Tensor, dmv: torch.Tensor, rowstats: torch.Tensor,
                               slope: float, want_dbias_in: bool = False):
    """bn_act_backward_split for dz = se_scale[b, c] * g + dmv[b, c] (never written),
    the sums from bn_se_backward_stats -> (dxs, dgamma, dbeta, dbias_in or None)."""
    b, c, r = x.shape[0], x.shape[1], x.shape[2]
    s = x.numel() // max(1, b * c)
    for t, nm in ((se_scale, "se_scale"), (dmv, "dmv")):
        _check(t, nm, "f")
        if t.numel() != b * c:
            raise ValueError(f"bn_se_backward_apply_split: {nm} must be (B, C)")
    _check(rowstats, "rowstats", "f")
    n = _lib.query("pcfm_conv3d_split_bytes", b, c, r)
    wsb = _lib.query("pcfm_bn_se_bwd_workspace_bytes", b, c, s)
    if n == 0 or wsb == 0:
        raise RuntimeError(f"bn_se_backward_apply_split: unsupported shape {tuple(x.shape)}")
    dxs = torch.empty(n, dtype=torch.uint8, device=x.device)
    dgb = torch.empty((3, c), dtype=torch.float32, device=x.device)
    ws = _workspace(wsb, x)
    with _timed("bn_act_bwd", 4 * 3 * x.numel(), x):
        _lib.call("pcfm_bn_se_bwd_apply_split", _ptr(g), _ptr(x), _ptr(mean), _ptr(invstd),
                  _ptr(weight), _ptr(bias), _ptr(se_scale), _ptr(dmv), _ptr(rowstats), b, c, s,
                  float(slope), _ptr(dxs), _ptr(dgb[0]), _ptr(dgb[1]),
                  _ptr(dgb[2]) if want_dbias_in else None, _ptr(ws), ws.numel(), _stream(x))
    return dxs, dgb[0], dgb[1], (dgb[2] if want_dbias_in else None)


def rows_max_bf16(h: torch.Tensor):
    """(values bf16 (B, C), indices int32 (B, C)) = max over dim 1 of h (B, N, C) bf16."""
    _check_cuda(h, "h")
    if h.dtype != torch.bfloat16 or h.dim() != 3 or not h.is_contiguous():
        raise RuntimeError("rows_max_bf16: h must be a contiguous (B, N, C) bf16 tensor")
    b, n, c = h.shape
    val = torch.empty((b, c), dtype=torch.bfloat16, device=h.device)
    idx = torch.empty((b, c), dtype=torch.int32, device=h.device)
    ws = _workspace(_lib.query("pcfm_rows_max_workspace_bytes", b, n, c), h)
    _lib.call("pcfm_rows_max_bf16", _ptr(h), b, n, c, _ptr(val), _ptr(idx), _ptr(ws), ws.numel(),
              _stream(h))
    return val, idx


# --------------------------------------------------------------------------
# GroupNorm + FiLM + residual (include/pcfm.h pcfm_gn_film_res_*)
# --------------------------------------------------------------------------
def gn_film_res_forward(x, weight, bias, gamma, beta, groups: int, eps: float):
    """out = x + GroupNorm(x) * (1 + gamma[:, :, None]) + beta[:, :, None] -> (out, mean, rstd)"""
    _check(x, "input", "f")
    b, c, n = x.shape
    gamma, beta = gamma.contiguous(), beta.contiguous()
    out = torch.empty_like(x)
    stats = torch.empty((2, b, groups), dtype=torch.float32, device=x.device)
    ws = _workspace(_lib.query("pcfm_gn_film_workspace_bytes", b, c, n, groups), x)
    with _timed("gn_film_res_fwd", 4 * 3 * x.numel(), x):
        _lib.call("pcfm_gn_film_res_fwd", _ptr(x), _ptr(weight), _ptr(bias), _ptr(gamma),
                  _ptr(beta), b, c, n, groups, float(eps), _ptr(out), _ptr(stats[0]),
                  _ptr(stats[1]), _ptr(ws), ws.numel(), _stream(x))
    return out, stats[0], stats[1]


def gn_film_res_forward_bnin(y, bn_mean, bn_invstd, bn_weight, bn_bias, slope: float, weight,
                             bias, gamma, beta, groups: int, eps: float):
    """gn_film_res_forward over z = act(bn(y)) (the PV block's post SharedMLP
    activation, computed as bn_act_forward does and never written) -> (out, mean, rstd)"""
    _check(y, "input", "f")
    b, c, n = y.shape
    for t, nm in ((bn_mean, "bn_mean"), (bn_invstd, "bn_invstd"), (bn_weight, "bn_weight"),
                  (bn_bias, "bn_bias")):
        _check(t, nm, "f")
        if t.numel() != c:
            raise ValueError(f"gn_film_res_forward_bnin: {nm} must have C values")
    gamma, beta = gamma.contiguous(), beta.contiguous()
    out = torch.empty_like(y)
    stats = torch.empty((2, b, groups), dtype=torch.float32, device=y.device)
    ws = _workspace(_lib.query("pcfm_gn_film_workspace_bytes", b, c, n, groups), y)
    with _timed("gn_film_res_fwd", 4 * 3 * y.numel(), y):
        _lib.call("pcfm_gn_film_res_fwd_bnin", _ptr(y), _ptr(bn_mean), _ptr(bn_invstd),
                  _ptr(bn_weight), _ptr(bn_bias), float(slope), _ptr(weight), _ptr(bias),
                  _ptr(gamma), _ptr(beta), b, c, n, groups, float(eps), _ptr(out),
                  _ptr(stats[0]), _ptr(stats[1]), _ptr(ws), ws.numel(), _stream(y))
    return out, stats[0], stats[1]


def gn_film_res_backward_bnin(dout, y, bn_mean, bn_invstd, bn_weight, bn_bias, slope: float,
                              weight, bias, gamma, mean, rstd, groups: int):
    """Backward of gn_film_res_forward_bnin -> (dz, dweight, dbias, dgamma (B, C),
    dbeta (B, C), bnpart (C, P, 2)): dz = dL/dz and the BatchNorm backward
    statistics for bn_act_backward_parts."""
    dout = dout.contiguous()
    b, c, n = y.shape
    P = _lib.query("pcfm_gn_bnin_parts", b, n)
    if P <= 0:
        raise RuntimeError(f"gn_film_res_backward_bnin: unsupported shape {tuple(y.shape)}")
    dz = torch.empty_like(y)
    small = torch.empty((2 * c + 2 * b * c,), dtype=torch.float32, device=y.device)
    dw, dbias = small[:c], small[c:2 * c]
    dgamma = small[2 * c:2 * c + b * c].view(b, c)
    dbeta = small[2 * c + b * c:].view(b, c)
    bnpart = torch.empty((c, P, 2), dtype=torch.float32, device=y.device)
    ws = _workspace(_lib.query("pcfm_gn_film_workspace_bytes", b, c, n, groups), y)
    with _timed("gn_film_res_bwd", 4 * 5 * y.numel(), y):
        _lib.call("pcfm_gn_film_res_bwd_bnin", _ptr(dout), _ptr(y), _ptr(bn_mean),
                  _ptr(bn_invstd), _ptr(bn_weight), _ptr(bn_bias), float(slope), _ptr(weight),
                  _ptr(bias), _ptr(gamma.contiguous()), _ptr(mean), _ptr(rstd), b, c, n, groups,
                  _ptr(dz), _ptr(dw), _ptr(dbias), _ptr(dgamma), _ptr(dbeta), _ptr(bnpart),
                  _ptr(ws), ws.numel(), _stream(y))
    return dz, dw, dbias, dgamma, dbeta, bnpart


def bn_act_backward_parts(dz: torch.Tensor, x: torch.Tensor, weight, bias, mean, invstd,
                          part: torch.Tensor, slope: float, want_dbias_in: bool = False):
    """bn_act_backward's apply pass on statistics a neighbouring kernel produced
    (part (C, P, 2) of (sum g, sum g * xhat)) -> (dx, dgamma, dbeta, dbias_in or None)."""
    dz = dz.contiguous()
    _check(part, "part", "f")
    b, c = x.shape[0], x.shape[1]
    s = x.numel() // max(1, b * c)
    dx = torch.empty_like(x)
    dgb = torch.empty((3, c), dtype=torch.float32, device=x.device)
    ws = _workspace(_lib.query("pcfm_bn_workspace_bytes", b, c, s), x)
    with _timed("bn_act_bwd", 4 * 3 * x.numel(), x):
        _lib.call("pcfm_bn_act_bwd_apply_parts", _ptr(dz), _ptr(x), _ptr(weight), _ptr(bias),
                  _ptr(mean), _ptr(invstd), _ptr(part), int(part.shape[1]), b, c, s,
                  float(slope), _ptr(dx), _ptr(dgb[0]), _ptr(dgb[1]),
                  _ptr(dgb[2]) if want_dbias_in else None, _ptr(ws), ws.numel(), _stream(x))
    return dx, dgb[0], dgb[1], (dgb[2] if want_dbias_in else None)


def gn_silu_forward(x, weight, bias, groups: int, eps: float):
    """out = SiLU(GroupNorm(x)) -> (out, mean, rstd)"""
    _check(x, "input", "f")
    b, c, n = x.shape
    out = torch.empty_like(x)
    stats = torch.empty((2, b, groups), dtype=torch.float32, device=x.device)
    ws = _workspace(_lib.query("pcfm_gn_film_workspace_bytes", b, c, n, groups), x)
    with _timed("gn_silu_fwd", 4 * 3 * x.numel(), x):
        _lib.call("pcfm_gn_silu_fwd", _ptr(x), _ptr(weight), _ptr(bias), b, c, n, groups,
                  float(eps), _ptr(out), _ptr(stats[0]), _ptr(stats[1]), _ptr(ws), ws.numel(),
                  _stream(x))
    return out, stats[0], stats[1]


def gn_silu_backward(dout, x, weight, bias, mean, rstd, groups: int):
    """-> (dx, dweight, dbias)"""
    dout = dout.contiguous()
    b, c, n = x.shape
    dx = torch.empty_like(x)
    small = torch.empty((2 * c,), dtype=torch.float32, device=x.device)
    dw, dbias = small[:c], small[c:]
    ws = _workspace(_lib.query("pcfm_gn_film_workspace_bytes", b, c, n, groups), x)
    with _timed("gn_silu_bwd", 4 * 5 * x.numel(), x):
        _lib.call("pcfm_gn_silu_bwd", _ptr(dout), _ptr(x), _ptr(weight), _ptr(bias), _ptr(mean),
                  _ptr(rstd), b, c, n, groups, _ptr(dx), _ptr(dw), _ptr(dbias), _ptr(ws),
                  ws.numel(), _stream(x))
    return dx, dw, dbias


def gn_film_res_backward(dout, x, weight, bias, gamma, mean, rstd, groups: int):
    """-> (dx, dweight, dbias, dgamma (B, C), dbeta (B, C))"""
    dout = dout.contiguous()
    b, c, n = x.shape
    dx = torch.empty_like(x)
    small = torch.empty((2 * c + 2 * b * c,), dtype=torch.float32, device=x.device)
    dw, dbias = small[:c], small[c:2 * c]
    dgamma = small[2 * c:2 * c + b * c].view(b, c)
    dbeta = small[2 * c + b * c:].view(b, c)
    ws = _workspace(_lib.query("pcfm_gn_film_workspace_bytes", b, c, n, groups), x)
    with _timed("gn_film_res_bwd", 4 * 5 * x.numel(), x):
        _lib.call("pcfm_gn_film_res_bwd", _ptr(dout), _ptr(x), _ptr(weight), _ptr(bias),
                  _ptr(gamma.contiguous()), _ptr(mean), _ptr(rstd), b, c, n, groups, _ptr(dx),
                  _ptr(dw), _ptr(dbias), _ptr(dgamma), _ptr(dbeta), _ptr(ws), ws.numel(),
                  _stream(x))
    return dx, dw, dbias, dgamma, dbeta
