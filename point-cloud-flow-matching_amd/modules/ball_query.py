"""BallQuery module: neighbour coordinates (+ features) around centers.

Reference: third_party/pvcnn/modules/ball_query.py:9-34.
"""
import torch
import torch.nn as nn

import modules.functional as F

__all__ = ["BallQuery"]


class BallQuery(nn.Module):
    def __init__(self, radius, num_neighbors, include_coordinates=True):
        super().__init__()
        self.radius = radius
        self.num_neighbors = num_neighbors
        self.include_coordinates = include_coordinates

    def forward(self, points_coords, centers_coords, points_features=None):
        pts = points_coords.contiguous()
        ctr = centers_coords.contiguous()
        nbr = F.ball_query(ctr, pts, self.radius, self.num_neighbors)
        rel = F.grouping(pts, nbr) - ctr.unsqueeze(-1)
        if points_features is None:
            if not self.include_coordinates:
                raise AssertionError("No Features For Grouping")
            return rel
        grouped = F.grouping(points_features, nbr)
        return torch.cat([rel, grouped], dim=1) if self.include_coordinates else grouped

    def extra_repr(self):
        tail = ", include coordinates" if self.include_coordinates else ""
        return f"radius={self.radius}, num_neighbors={self.num_neighbors}{tail}"
