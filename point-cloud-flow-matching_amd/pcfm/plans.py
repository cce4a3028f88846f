"""Per-points caches of the PVConv scatter plans.

The hybrid backbone runs two PVConv blocks per stage on the SAME points
(reference models.py:371-389 `_PVStage`; PVConv returns its `coords` unchanged,
third_party/pvcnn/modules/pvconv.py:35-39), so everything that depends only on
the coordinates is computed once per stage instead of once per block:
  * the voxel-grid coordinates (Voxelization's normalise + round; the
    resolution-independent [0, 1] coordinates are shared across the stages too),
  * the voxelization plan (stable sort of the points by voxel, work units;
    also the backward's ind / cnt),
  * the devoxelization's corner indices / weights (inds, wgts) and
  * the devoxelization-backward plan (sort by base cell, sorted tap weights),
  * the occupancy masks of the voxelized grid (which voxel tiles / taps of
    PVConv's first convolution touch an occupied voxel).
Entries are keyed on the identity of the tensor they derive from (plus its
version counter) and die with it (weakref), so nothing outlives the step.
Results are bit-identical to recomputing (same kernels, same inputs).
PCFM_SHARE_PLANS=0 turns the sharing off (measurement switch).
"""
from __future__ import annotations

import os
import weakref
from typing import NamedTuple, Optional

import torch

ENABLED = os.environ.get("PCFM_SHARE_PLANS", "1") != "0"
# occupancy-masked first voxel convolution of PVConv (measurement switch)
OCCUPANCY = os.environ.get("PCFM_CONV_OCC", "1") != "0"
# ... computed at voxel granularity through voxel lists (measurement switch)
VOXEL_LISTS = os.environ.get("PCFM_CONV_VLIST", "1") != "0"


class Occupancy(NamedTuple):
    """What PVConv's first convolution may skip, from the voxelization's counts:
    tile masks (ops.conv3d_occupancy), voxel lists (ops.conv3d_vlists; None when
    off) and the counts themselves."""
    masks: torch.Tensor
    lists: Optional[torch.Tensor]
    cnt: torch.Tensor


class IdentityCache:
    """{(tensor identity, tag): value}, valid while the tensor lives unmodified."""

    def __init__(self):
        self._d = {}

    def get(self, t: torch.Tensor, tag):
        e = self._d.get((id(t), tag))
        if e is None:
            return None
        ref, version, value = e
        if ref() is not t or t._version != version:
            self._d.pop((id(t), tag), None)
            return None
        return value

    def put(self, t: torch.Tensor, tag, value):
        key = (id(t), tag)
        d = self._d

        def drop(_ref, key=key, d=d):
            e = d.get(key)
            if e is not None and e[0] is _ref:
                del d[key]

        d[key] = (weakref.ref(t, drop), t._version, value)
        return value

    def __len__(self):
        return len(self._d)


_cache = IdentityCache()


def _on(t: torch.Tensor) -> bool:
    return ENABLED and t.is_cuda


def grid_coords(vox, coords: torch.Tensor):
    """(norm_coords, vox_coords) of Voxelization `vox` for coords (shared)."""
    tag = ("grid", vox.r, bool(vox.normalize), float(vox.eps))
    hit = _cache.get(coords, tag) if _on(coords) else None
    if hit is not None:
        return hit
    if not _on(coords):
        norm = vox._grid_coords(coords.detach())
        return norm, torch.round(norm).to(torch.int32)
    # the normalised [0, 1] coordinates do not depend on the resolution: one
    # computation for every stage's voxelization of the same points
    utag = ("unit", bool(vox.normalize), float(vox.eps))
    unit = _cache.get(coords, utag)
    if unit is None:
        unit = _cache.put(coords, utag, vox._unit_coords(coords.detach()))
    norm = vox._scale_coords(unit)
    return _cache.put(coords, tag, (norm, torch.round(norm).to(torch.int32)))


def voxel_plan(vox_coords: torch.Tensor, r: int):
    """ops.avg_voxelize_plan(vox_coords, r), shared."""
    from pcfm import ops
    tag = ("vox", int(r))
    hit = _cache.get(vox_coords, tag)
    if hit is not None:
        return hit
    return _cache.put(vox_coords, tag, ops.avg_voxelize_plan(vox_coords, r))


def conv_occupancy(vox_coords: torch.Tensor, r: int) -> Optional[Occupancy]:
    """Occupancy of the voxelization plan's counts (shared per points): tile
    masks and voxel lists, or None when off or unsupported (r^3 % 256 != 0)."""
    from pcfm import ops
    if not (OCCUPANCY and _on(vox_coords)):
        return None
    tag = ("occ", int(r))
    hit = _cache.get(vox_coords, tag)
    if hit is not None:
        return hit[0]
    cnt = voxel_plan(vox_coords, r).cnt
    masks = ops.conv3d_occupancy(cnt, r)
    if masks is None:
        return None
    occ = Occupancy(masks, ops.conv3d_vlists(cnt, r) if VOXEL_LISTS else None, cnt)
    _cache.put(vox_coords, tag, (occ,))
    return occ


def devox_corners(norm_coords: torch.Tensor, r: int):
    """(inds, wgts) a devoxelization over norm_coords already produced, or None."""
    return _cache.get(norm_coords, ("corners", int(r))) if _on(norm_coords) else None


def put_devox_corners(norm_coords: torch.Tensor, r: int, inds, wgts) -> None:
    if _on(norm_coords):
        _cache.put(norm_coords, ("corners", int(r)), (inds, wgts))


def devox_bwd_plan(norm_coords: torch.Tensor, inds: torch.Tensor, wgts: torch.Tensor, r: int):
    """ops.trilinear_devoxelize_backward_plan(inds, wgts, r) for the corners of
    norm_coords, shared (autograd may hand each node its own tensor objects for
    the same saved inds, so the key is the points tensor)."""
    from pcfm import ops
    tag = ("devox_bwd", int(r))
    hit = _cache.get(norm_coords, tag) if _on(norm_coords) else None
    if hit is not None:
        return hit
    plan = ops.trilinear_devoxelize_backward_plan(inds, wgts, r)
    return _cache.put(norm_coords, tag, plan) if _on(norm_coords) else plan
