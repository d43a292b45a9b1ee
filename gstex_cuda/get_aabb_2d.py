"""gstex_cuda.get_aabb_2d — imported at nerfstudio/models/gstex.py:31."""
from gstex_amd.ops import get_aabb_2d, get_num_tiles_hit_2d, project_points  # noqa: F401
