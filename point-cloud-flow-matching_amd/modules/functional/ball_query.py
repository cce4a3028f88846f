"""ball_query (no gradient).  Reference:
third_party/pvcnn/modules/functional/ball_query.py:8-19."""
from modules.functional import backend as _be

__all__ = ["ball_query"]


def ball_query(centers_coords, points_coords, radius, num_neighbors):
    """centers f32 [B, 3, M], points f32 [B, 3, N] -> i32 [B, M, U] neighbour indices."""
    return _be._backend.ball_query(centers_coords.contiguous(), points_coords.contiguous(),
                                   radius, num_neighbors)
