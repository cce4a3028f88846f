"""Drop-in for the reference's PVCNN `modules` package
(third_party/pvcnn/modules/__init__.py), restricted to the flow model's hot
path: PVConv, SharedMLP, Voxelization, SE3d, BallQuery.  The PointNet++ /
frustum / KL modules are outside this build's scope.
"""
from modules.ball_query import BallQuery
from modules.pvconv import PVConv
from modules.se import SE3d
from modules.shared_mlp import SharedMLP
from modules.voxelization import Voxelization

__all__ = ["BallQuery", "PVConv", "SE3d", "SharedMLP", "Voxelization"]
