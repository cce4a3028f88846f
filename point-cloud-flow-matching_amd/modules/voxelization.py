"""Voxelization module: point coords -> voxel grid of averaged features.

Reference: third_party/pvcnn/modules/voxelization.py:8-28.  The coordinate
normalisation is the reference's exact sequence of torch ops (mean-centre,
scale by 2*max radius + eps, shift to [0,1], scale to [0, r-1], round
half-to-even), so voxel assignment is identical; the pooling itself runs in the
gfx950 scatter kernel (modules.functional.avg_voxelize).
"""
import torch
import torch.nn as nn

import modules.functional as F

__all__ = ["Voxelization"]


class Voxelization(nn.Module):
    def __init__(self, resolution, normalize=True, eps=0):
        super().__init__()
        self.r = int(resolution)
        self.normalize = normalize
        self.eps = eps

    def _unit_coords(self, coords: torch.Tensor) -> torch.Tensor:
        # the resolution-independent part (shared by the stages' voxelizations)
        centred = coords - coords.mean(2, keepdim=True)
        if self.normalize:
            radius = centred.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values
            return centred / (radius * 2.0 + self.eps) + 0.5
        return (centred + 1) / 2.0

    def _scale_coords(self, unit: torch.Tensor) -> torch.Tensor:
        return torch.clamp(unit * self.r, 0, self.r - 1)

    def _grid_coords(self, coords: torch.Tensor) -> torch.Tensor:
        return self._scale_coords(self._unit_coords(coords))

    def _coords(self, coords):
        # shared per points on a HIP device (pcfm.plans): a stage's PVConv
        # blocks normalise the same coordinates
        from pcfm import plans
        return plans.grid_coords(self, coords)

    def forward(self, features, coords):
        norm_coords, vox_coords = self._coords(coords)
        return F.avg_voxelize(features, vox_coords, self.r), norm_coords

    def forward_tee(self, features, coords):
        """forward() plus the features passed through for a second consumer, their
        two gradients summed inside the voxelization's backward gather."""
        norm_coords, vox_coords = self._coords(coords)
        grid, feats = F.avg_voxelize_tee(features, vox_coords, self.r)
        return grid, norm_coords, feats

    def extra_repr(self):
        tail = f", normalized eps = {self.eps}" if self.normalize else ""
        return f"resolution={self.r}{tail}"
