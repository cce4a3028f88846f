"""Functional PVCNN ops (reference: third_party/pvcnn/modules/functional/__init__.py).

The PointNet++-only helpers of the reference (furthest_point_sample, gather,
nearest_neighbor_interpolate, kl/huber loss) are outside this build's hot path
 and are not exported.
"""
from modules.functional.ball_query import ball_query
from modules.functional.devoxelization import trilinear_devoxelize
from modules.functional.grouping import grouping
from modules.functional.voxelization import avg_voxelize, avg_voxelize_tee

__all__ = ["ball_query", "trilinear_devoxelize", "grouping", "avg_voxelize", "avg_voxelize_tee"]
