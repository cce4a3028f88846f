"""Pure-PyTorch CPU backend: the native operators for tensors that are not on a
HIP device (BASELINE.json configs[0], "PVConv/Chamfer via pure-PyTorch
fallback" -- SURVEY.md sections 0.5 and 7.2).

The reference has no CPU path: its `_pvcnn_backend`, `chamfer_3D` and `emd_ext`
modules are JIT-built CUDA and reject CPU tensors
(third_party/pvcnn/modules/functional/src/utils.hpp:7-18).  `pcfm.ops` routes a
call here when its inputs are CPU tensors, so models.py / train.py run
unchanged on a machine without a GPU; tensors on a HIP device always take the
gfx950 kernels (and raise if libpcfm_hip.so is missing).

Every function restates the reference kernel it names with vectorised torch
ops (scatter_add_ / gather / blocked pairwise distances), same inputs, outputs,
dtypes and index conventions.  Arithmetic follows the reference's expressions:
  * voxel average: feat * (float)(1.0 / (double)cnt) per term (vox.cu:66-68);
  * trilinear weights x*y*z in that order, corner k = 4dx + 2dy + dz, hi
    corner only if the fraction is > 0 (trilinear_devox.cu:41-75);
  * squared distances with the fused form nvcc emits, fma(dz, dz, fma(dx, dx,
    dy*dy)), evaluated as an exact float64 product + one rounding per fma;
  * argmin ties keep the lowest index (chamfer3D.cu strict `<`).
Scatter sums run in torch's CPU scatter order, so vox-fwd / devox-bwd /
grouping-bwd / chamfer-bwd can differ from a sequential sum in the last bits,
as the reference's float atomics do.  Tests hold this module against the C
oracle (tests/test_cpu_ops.py); it never imports the oracle.
"""
from __future__ import annotations

import torch

__all__ = [
    "avg_voxelize_forward", "avg_voxelize_backward", "trilinear_devoxelize_forward",
    "trilinear_devoxelize_backward", "ball_query", "grouping_forward", "grouping_backward",
    "chamfer_forward", "chamfer_backward", "approxmatch_forward", "matchcost_forward",
    "matchcost_backward",
]

# rows of the query set per pairwise block (bounds the (rows, M) temporaries)
_BLOCK_ELEMS = 1 << 22


def _fma32(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    """float32 fma(a, b, c): the float64 product of two floats is exact, so one
    float64 add then the cast to float32 rounds (almost always) once."""
    return (a.double() * b.double() + c.double()).float()


def _sqdist(dx, dy, dz):
    """fma(dz, dz, fma(dx, dx, dy * dy)) in float32 (nvcc's contraction of
    dx*dx + dy*dy + dz*dz; chamfer3D.cu:32-35, ball_query.cu:36-38)."""
    if dx.dtype != torch.float32:
        return dx * dx + dy * dy + dz * dz
    return _fma32(dz, dz, _fma32(dx, dx, dy * dy))


# ---------------------------------------------------------------------------
# voxelization (vox.cu:18-110)
# ---------------------------------------------------------------------------
def _inv_count(cnt: torch.Tensor) -> torch.Tensor:
    """(float)(1.0 / (double)cnt) (vox.cu:66, :104); 0 where cnt == 0."""
    inv = (1.0 / cnt.double().clamp_min(1.0)).float()
    return torch.where(cnt > 0, inv, torch.zeros_like(inv))


def avg_voxelize_forward(features: torch.Tensor, coords: torch.Tensor, resolution: int):
    """grid_stats_kernel + avg_voxelize_kernel -> [out (b,c,r^3), ind (b,n), cnt (b,r^3)]."""
    b, c, n = features.shape
    r = int(resolution)
    s = r * r * r
    ind = coords[:, 0] * (r * r) + coords[:, 1] * r + coords[:, 2]  # int32 (b, n)
    ind64 = ind.long()
    cnt = torch.zeros((b, s), dtype=torch.int32)
    cnt.scatter_add_(1, ind64, torch.ones_like(ind))
    w = torch.gather(_inv_count(cnt), 1, ind64)  # 1/cnt of each point's voxel
    out = torch.zeros((b, c, s), dtype=torch.float32)
    out.scatter_add_(2, ind64[:, None, :].expand(b, c, n), features * w[:, None, :])
    return [out, ind.to(torch.int32), cnt]


def avg_voxelize_backward(grad_y: torch.Tensor, indices: torch.Tensor, cnt: torch.Tensor):
    """avg_voxelize_grad_kernel: grad_x[c, i] = grad_y[c, ind[i]] * (1 / cnt[ind[i]])."""
    b, c, _ = grad_y.shape
    n = indices.shape[1]
    ind64 = indices.long()
    w = torch.gather(_inv_count(cnt), 1, ind64)
    return torch.gather(grad_y, 2, ind64[:, None, :].expand(b, c, n)) * w[:, None, :]


# ---------------------------------------------------------------------------
# trilinear devoxelization (trilinear_devox.cu:21-162)
# ---------------------------------------------------------------------------
def _corners(coords: torch.Tensor, r: int):
    """(inds (b,8,n) int32, wgts (b,8,n) f32) with corner k = 4dx + 2dy + dz."""
    x, y, z = coords[:, 0], coords[:, 1], coords[:, 2]
    xl, yl, zl = torch.floor(x), torch.floor(y), torch.floor(z)
    x1, y1, z1 = x - xl, y - yl, z - zl
    x0, y0, z0 = 1.0 - x1, 1.0 - y1, 1.0 - z1
    wgts = torch.stack([x0 * y0 * z0, x0 * y0 * z1, x0 * y1 * z0, x0 * y1 * z1,
                        x1 * y0 * z0, x1 * y0 * z1, x1 * y1 * z0, x1 * y1 * z1], dim=1)
    base = xl.int() * (r * r) + yl.int() * r + zl.int()
    dz = (z1 > 0).int()
    dy = (y1 > 0).int() * r
    dx = (x1 > 0).int() * (r * r)
    inds = torch.stack([base, base + dz, base + dy, base + dy + dz, base + dx, base + dx + dz,
                        base + dx + dy, base + dx + dy + dz], dim=1)
    return inds.to(torch.int32), wgts


def trilinear_devoxelize_forward(r: int, is_training: bool, coords: torch.Tensor,
                                 features: torch.Tensor):
    """-> [outs (b,c,n), inds (b,8,n) | (1,), wgts (b,8,n) | (1,)]."""
    b, c = features.shape[0], features.shape[1]
    n = coords.shape[2]
    r = int(r)
    s = r * r * r
    inds, wgts = _corners(coords, r)
    valid = (inds >= 0) & (inds < s)  # coords outside [0, r-1] contribute 0
    gi = torch.where(valid, inds, torch.zeros_like(inds)).long()
    gw = torch.where(valid, wgts, torch.zeros_like(wgts))
    feats = features.reshape(b, c, s)

    def term(k):
        return torch.gather(feats, 2, gi[:, k:k + 1, :].expand(b, c, n))

    # w1*f1, then fma(w0, f0, .), then fma(wk, fk, .) for k = 2..7 (nvcc's
    # contraction of the left-to-right sum at :98-102)
    acc = gw[:, 1:2] * term(1)
    acc = _fma32(gw[:, 0:1].expand(b, c, n), term(0), acc)
    for k in range(2, 8):
        acc = _fma32(gw[:, k:k + 1].expand(b, c, n), term(k), acc)
    if is_training:
        return [acc, inds, wgts]
    return [acc, torch.zeros((1,), dtype=torch.int32), torch.zeros((1,), dtype=torch.float32)]


def trilinear_devoxelize_backward(grad_y: torch.Tensor, indices: torch.Tensor,
                                  weights: torch.Tensor, r: int):
    """trilinear_devoxelize_grad_kernel: grad_x[c, idx_k] += w_k * grad_y[c, i]."""
    b, c, n = grad_y.shape
    s = int(r) ** 3
    gx = torch.zeros((b, c, s), dtype=torch.float32)
    valid = (indices >= 0) & (indices < s)
    gi = torch.where(valid, indices, torch.zeros_like(indices)).long()
    gw = torch.where(valid, weights, torch.zeros_like(weights))
    for k in range(8):
        gx.scatter_add_(2, gi[:, k:k + 1, :].expand(b, c, n), gw[:, k:k + 1, :] * grad_y)
    return gx


# ---------------------------------------------------------------------------
# ball query + grouping (ball_query.cu:19-50, grouping.cu:18-77)
# ---------------------------------------------------------------------------
def ball_query(centers_coords: torch.Tensor, points_coords: torch.Tensor, radius: float,
               num_neighbors: int):
    """First u point indices k (ascending) with d^2 < radius^2 per center, the
    first hit repeated into the unused slots, all zeros when nothing is in range."""
    b, _, m = centers_coords.shape
    n = points_coords.shape[2]
    u = int(num_neighbors)
    r2 = torch.tensor(float(radius), dtype=torch.float32) ** 2
    out = torch.zeros((b, m, u), dtype=torch.int32)
    if n == 0 or m == 0 or u == 0:
        return out
    rows = max(1, _BLOCK_ELEMS // n)
    slot = torch.arange(u, dtype=torch.int64)[None, :]
    for bb in range(b):
        p = points_coords[bb]
        for j0 in range(0, m, rows):
            cc = centers_coords[bb, :, j0:j0 + rows]
            # dx = center - point (ball_query.cu:36-38)
            d2 = _sqdist(cc[0][:, None] - p[0][None], cc[1][:, None] - p[1][None],
                         cc[2][:, None] - p[2][None])
            hit = d2 < r2
            # the hits in ascending k: a stable sort on "not a hit" keeps index order
            order = torch.argsort((~hit).to(torch.int8), dim=1, stable=True)
            if u > n:
                order = torch.nn.functional.pad(order, (0, u - n))
            order = order[:, :u]
            nhit = hit.sum(dim=1, keepdim=True)
            take = torch.where(slot < nhit, order, order[:, :1])  # pad with the first hit
            take = torch.where(nhit > 0, take, torch.zeros_like(take))
            out[bb, j0:j0 + cc.shape[1]] = take.to(torch.int32)
    return out


def grouping_forward(features: torch.Tensor, indices: torch.Tensor):
    """out[b, c, m, u] = features[b, c, indices[b, m, u]]."""
    b, c, n = features.shape
    m, u = indices.shape[1], indices.shape[2]
    idx = indices.long().reshape(b, 1, m * u).expand(b, c, m * u)
    return torch.gather(features, 2, idx).reshape(b, c, m, u)


def grouping_backward(grad_y: torch.Tensor, indices: torch.Tensor, n: int):
    """grad_x[b, c, indices[b, m, u]] += grad_y[b, c, m, u]."""
    b, c, m, u = grad_y.shape
    idx = indices.long().reshape(b, 1, m * u).expand(b, c, m * u)
    gx = torch.zeros((b, c, int(n)), dtype=torch.float32)
    gx.scatter_add_(2, idx, grad_y.reshape(b, c, m * u))
    return gx


# ---------------------------------------------------------------------------
# Chamfer-3D (chamfer3D.cu:12-195)
# ---------------------------------------------------------------------------
def _nn(q: torch.Tensor, p: torch.Tensor):
    """Nearest p for each q: (dist (b, nq), idx (b, nq) int32), lowest index on ties."""
    b, nq, _ = q.shape
    npt = p.shape[1]
    dist = torch.zeros((b, nq), dtype=q.dtype)
    idx = torch.zeros((b, nq), dtype=torch.int32)
    if npt == 0 or nq == 0:
        return dist, idx
    rows = max(1, _BLOCK_ELEMS // npt)
    for bb in range(b):
        pb = p[bb]
        for j0 in range(0, nq, rows):
            qb = q[bb, j0:j0 + rows]
            # dx = candidate - query (chamfer3D.cu:32-35)
            d = _sqdist(pb[None, :, 0] - qb[:, None, 0], pb[None, :, 1] - qb[:, None, 1],
                        pb[None, :, 2] - qb[:, None, 2])
            val, arg = torch.min(d, dim=1)  # first minimum on ties
            dist[bb, j0:j0 + qb.shape[0]] = val
            idx[bb, j0:j0 + qb.shape[0]] = arg.to(torch.int32)
    return dist, idx


def chamfer_forward(xyz1, xyz2, dist1, dist2, idx1, idx2) -> None:
    """chamfer_cuda_forward: writes the caller-allocated outputs in place."""
    d, i = _nn(xyz1, xyz2)
    dist1.copy_(d)
    idx1.copy_(i)
    d, i = _nn(xyz2, xyz1)
    dist2.copy_(d)
    idx2.copy_(i)


def chamfer_backward(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1, idx2) -> None:
    """NmDistanceGradKernel (both directions): g = 2 * grad_dist; the query's
    gradient += g * (q - p), the matched point's -= it.  Accumulates, like the
    reference (the callers zero the gradients)."""
    for q, p, gd, ix, gq, gp in ((xyz1, xyz2, graddist1, idx1, gradxyz1, gradxyz2),
                                 (xyz2, xyz1, graddist2, idx2, gradxyz2, gradxyz1)):
        if q.shape[1] == 0 or p.shape[1] == 0:
            continue
        ixl = ix.long()
        matched = torch.gather(p, 1, ixl[:, :, None].expand(-1, -1, 3))
        t = (gd * 2.0)[:, :, None] * (q - matched)
        gq.add_(t)
        gp.scatter_add_(1, ixl[:, :, None].expand(-1, -1, 3), -t)


# ---------------------------------------------------------------------------
# approximate EMD (PyTorchEMD/cuda/emd_kernel.cu:24-353)
# ---------------------------------------------------------------------------
def _pair_sqdist(xyz1, xyz2):
    """(b, n, m) squared distances, dx = xyz2 - xyz1 (emd_kernel.cu:59-63)."""
    d = xyz2[:, None, :, :] - xyz1[:, :, None, :]
    return _sqdist(d[..., 0], d[..., 1], d[..., 2])


def approxmatch_forward(xyz1: torch.Tensor, xyz2: torch.Tensor) -> torch.Tensor:
    """approxmatch: 10 levels (level = -4^j, j = 7..-2, the last 0) of soft
    matching; -> match (b, m, n)."""
    b, n = xyz1.shape[0], xyz1.shape[1]
    m = xyz2.shape[1]
    dt = xyz1.dtype
    match = torch.zeros((b, n, m), dtype=dt)
    if n == 0 or m == 0:
        return match.transpose(1, 2).contiguous()
    multi_l = 1.0 if n >= m else float(m // n)
    multi_r = float(n // m) if n >= m else 1.0
    d2 = _pair_sqdist(xyz1, xyz2)
    rem_l = torch.full((b, n), multi_l, dtype=dt)
    rem_r = torch.full((b, m), multi_r, dtype=dt)
    for j in range(7, -3, -1):
        level = 0.0 if j == -2 else -(4.0 ** j)
        e = torch.exp(level * d2)  # (b, n, m)
        rat_l = rem_l / (torch.einsum("bnm,bm->bn", e, rem_r) + 1e-9)
        sum_r = torch.einsum("bnm,bn->bm", e, rat_l) * rem_r
        cons = torch.clamp(rem_r / (sum_r + 1e-9), max=1.0)
        rat_r = cons * rem_r
        rem_r = torch.clamp(rem_r - sum_r, min=0.0)
        w = e * rat_l[:, :, None] * rat_r[:, None, :]
        match += w
        rem_l = torch.clamp(rem_l - w.sum(dim=2), min=0.0)
    return match.transpose(1, 2).contiguous()


def matchcost_forward(xyz1: torch.Tensor, xyz2: torch.Tensor, match: torch.Tensor):
    """cost[b] = sum_{k,l} d2(k, l) * match[b, l, k]."""
    d2 = _pair_sqdist(xyz1, xyz2)  # (b, n, m)
    return (d2 * match.transpose(1, 2)).sum(dim=(1, 2))


def matchcost_backward(grad_cost: torch.Tensor, xyz1: torch.Tensor, xyz2: torch.Tensor,
                       match: torch.Tensor):
    """grad1[k] = g * sum_l 2 match[l, k] (x1_k - x2_l); grad2[l] = g * sum_k
    2 match[l, k] (x2_l - x1_k)."""
    mt = match.transpose(1, 2) * 2.0  # (b, n, m)
    g = grad_cost.to(xyz1.dtype)[:, None, None]
    g1 = (mt.sum(dim=2)[:, :, None] * xyz1 - torch.bmm(mt, xyz2)) * g
    g2 = (mt.sum(dim=1)[:, :, None] * xyz2 - torch.bmm(mt.transpose(1, 2), xyz1)) * g
    return [g1, g2]
