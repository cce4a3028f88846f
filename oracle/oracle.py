"""Python face of the CPU oracle (pcfm_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product path (point-cloud-flow-matching_amd/) never does:
it has no CPU implementation and raises when its HIP library is missing.

Two layers:
  * numpy functions  (avg_voxelize_fwd, chamfer_fwd, ...): arrays in, arrays out;
  * `TorchBackend`: the reference's `_pvcnn_backend` function names over CPU
    torch tensors, so the reference-shaped Python layers (and this build's
    `modules` package) can run end to end on a CPU in tests (config C1).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

_lock = threading.Lock()
_lib = None


def build() -> str:
    """Compile liboracle.so with the committed recipe (oracle/Makefile)."""
    subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                build()
            _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


_I = ctypes.c_int


# ---------------------------------------------------------------------------
# numpy layer
# ---------------------------------------------------------------------------
def avg_voxelize_fwd(feat, coords, r):
    feat, coords = _f32(feat), _i32(coords)
    b, c, n = feat.shape
    s = r ** 3
    out = np.empty((b, c, s), np.float32)
    ind = np.empty((b, n), np.int32)
    cnt = np.empty((b, s), np.int32)
    lib().oracle_avg_voxelize_fwd(_p(feat), _p(coords), _I(b), _I(c), _I(n), _I(r), _p(out),
                                  _p(ind), _p(cnt))
    return out, ind, cnt


def avg_voxelize_bwd(grad_y, ind, cnt):
    grad_y, ind, cnt = _f32(grad_y), _i32(ind), _i32(cnt)
    b, c, s = grad_y.shape
    n = ind.shape[1]
    gx = np.empty((b, c, n), np.float32)
    lib().oracle_avg_voxelize_bwd(_p(grad_y), _p(ind), _p(cnt), _I(b), _I(c), _I(n), _I(s),
                                  _p(gx))
    return gx


def trilinear_devoxelize_fwd(coords, feat, r, training=True):
    coords, feat = _f32(coords), _f32(feat)
    b, c = feat.shape[:2]
    n = coords.shape[2]
    out = np.empty((b, c, n), np.float32)
    inds = np.zeros((b, 8, n), np.int32)
    wgts = np.zeros((b, 8, n), np.float32)
    lib().oracle_trilinear_devoxelize_fwd(_p(coords), _p(feat), _I(b), _I(c), _I(n), _I(r),
                                          _I(1 if training else 0), _p(out), _p(inds), _p(wgts))
    return out, inds, wgts


def trilinear_devoxelize_bwd(grad_y, inds, wgts, r):
    grad_y, inds, wgts = _f32(grad_y), _i32(inds), _f32(wgts)
    b, c, n = grad_y.shape
    gx = np.empty((b, c, r ** 3), np.float32)
    lib().oracle_trilinear_devoxelize_bwd(_p(grad_y), _p(inds), _p(wgts), _I(b), _I(c), _I(n),
                                          _I(r), _p(gx))
    return gx


def ball_query(centers, points, radius, u):
    centers, points = _f32(centers), _f32(points)
    b, _, m = centers.shape
    n = points.shape[2]
    idx = np.empty((b, m, u), np.int32)
    lib().oracle_ball_query(_p(centers), _p(points), _I(b), _I(m), _I(n),
                            ctypes.c_float(radius), _I(u), _p(idx))
    return idx


def grouping_fwd(feat, idx):
    feat, idx = _f32(feat), _i32(idx)
    b, c, n = feat.shape
    m, u = idx.shape[1:]
    out = np.empty((b, c, m, u), np.float32)
    lib().oracle_grouping_fwd(_p(feat), _p(idx), _I(b), _I(c), _I(n), _I(m), _I(u), _p(out))
    return out


def grouping_bwd(grad_y, idx, n):
    grad_y, idx = _f32(grad_y), _i32(idx)
    b, c, m, u = grad_y.shape
    gx = np.empty((b, c, n), np.float32)
    lib().oracle_grouping_bwd(_p(grad_y), _p(idx), _I(b), _I(c), _I(n), _I(m), _I(u), _p(gx))
    return gx


def chamfer_fwd(xyz1, xyz2):
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, n = xyz1.shape[:2]
    m = xyz2.shape[1]
    d1 = np.zeros((b, n), np.float32)
    d2 = np.zeros((b, m), np.float32)
    i1 = np.zeros((b, n), np.int32)
    i2 = np.zeros((b, m), np.int32)
    lib().oracle_chamfer_fwd(_p(xyz1), _p(xyz2), _I(b), _I(n), _I(m), _p(d1), _p(d2), _p(i1),
                             _p(i2))
    return d1, d2, i1, i2


def chamfer_bwd(xyz1, xyz2, gd1, gd2, idx1, idx2):
    xyz1, xyz2, gd1, gd2 = _f32(xyz1), _f32(xyz2), _f32(gd1), _f32(gd2)
    idx1, idx2 = _i32(idx1), _i32(idx2)
    b, n = xyz1.shape[:2]
    m = xyz2.shape[1]
    g1 = np.zeros((b, n, 3), np.float32)
    g2 = np.zeros((b, m, 3), np.float32)
    lib().oracle_chamfer_bwd(_p(xyz1), _p(xyz2), _I(b), _I(n), _I(m), _p(gd1), _p(gd2),
                             _p(idx1), _p(idx2), _p(g1), _p(g2))
    return g1, g2


def _emd_dtype(a):
    return np.float64 if np.asarray(a).dtype == np.float64 else np.float32


def emd_approxmatch(xyz1, xyz2):
    dt = _emd_dtype(xyz1)
    xyz1 = np.ascontiguousarray(xyz1, dtype=dt)
    xyz2 = np.ascontiguousarray(xyz2, dtype=dt)
    b, n = xyz1.shape[:2]
    m = xyz2.shape[1]
    match = np.zeros((b, m, n), dt)
    fn = lib().oracle_emd_approxmatch_f64 if dt == np.float64 else lib().oracle_emd_approxmatch_f32
    fn(_p(xyz1), _p(xyz2), _I(b), _I(n), _I(m), _p(match))
    return match


def emd_matchcost(xyz1, xyz2, match):
    dt = _emd_dtype(xyz1)
    xyz1, xyz2, match = (np.ascontiguousarray(a, dtype=dt) for a in (xyz1, xyz2, match))
    b, n = xyz1.shape[:2]
    m = xyz2.shape[1]
    cost = np.zeros((b,), dt)
    fn = lib().oracle_emd_matchcost_f64 if dt == np.float64 else lib().oracle_emd_matchcost_f32
    fn(_p(xyz1), _p(xyz2), _p(match), _I(b), _I(n), _I(m), _p(cost))
    return cost


def emd_matchcost_bwd(gcost, xyz1, xyz2, match):
    dt = _emd_dtype(xyz1)
    gcost, xyz1, xyz2, match = (np.ascontiguousarray(a, dtype=dt)
                                for a in (gcost, xyz1, xyz2, match))
    b, n = xyz1.shape[:2]
    m = xyz2.shape[1]
    g1 = np.zeros((b, n, 3), dt)
    g2 = np.zeros((b, m, 3), dt)
    fn = (lib().oracle_emd_matchcost_bwd_f64 if dt == np.float64
          else lib().oracle_emd_matchcost_bwd_f32)
    fn(_p(gcost), _p(xyz1), _p(xyz2), _p(match), _I(b), _I(n), _I(m), _p(g1), _p(g2))
    return g1, g2


# ---------------------------------------------------------------------------
# torch layer: the `_pvcnn_backend` surface over CPU tensors
# ---------------------------------------------------------------------------
def _torch_backend():
    import torch

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a))

    def npy(x):
        return x.detach().cpu().contiguous().numpy()

    def avg_voxelize_forward(features, coords, resolution):
        out, ind, cnt = avg_voxelize_fwd(npy(features), npy(coords), int(resolution))
        return [t(out), t(ind), t(cnt)]

    def avg_voxelize_backward(grad_y, indices, cnt):
        return t(avg_voxelize_bwd(npy(grad_y), npy(indices), npy(cnt)))

    def trilinear_devoxelize_forward(r, is_training, coords, features):
        out, inds, wgts = trilinear_devoxelize_fwd(npy(coords), npy(features), int(r),
                                                   bool(is_training))
        if not is_training:
            return [t(out), torch.zeros(1, dtype=torch.int32), torch.zeros(1)]
        return [t(out), t(inds), t(wgts)]

    def trilinear_devoxelize_backward(grad_y, indices, weights, r):
        return t(trilinear_devoxelize_bwd(npy(grad_y), npy(indices), npy(weights), int(r)))

    def ball_query_(centers_coords, points_coords, radius, num_neighbors):
        return t(ball_query(npy(centers_coords), npy(points_coords), float(radius),
                            int(num_neighbors)))

    def grouping_forward(features, indices):
        return t(grouping_fwd(npy(features), npy(indices)))

    def grouping_backward(grad_y, indices, n):
        return t(grouping_bwd(npy(grad_y), npy(indices), int(n)))

    return types.SimpleNamespace(
        avg_voxelize_forward=avg_voxelize_forward,
        avg_voxelize_backward=avg_voxelize_backward,
        trilinear_devoxelize_forward=trilinear_devoxelize_forward,
        trilinear_devoxelize_backward=trilinear_devoxelize_backward,
        ball_query=ball_query_,
        grouping_forward=grouping_forward,
        grouping_backward=grouping_backward,
    )


_torch_backend_obj = None


def TorchBackend():
    """The oracle as a `_pvcnn_backend`-shaped namespace (CPU torch tensors)."""
    global _torch_backend_obj
    if _torch_backend_obj is None:
        _torch_backend_obj = _torch_backend()
    return _torch_backend_obj
