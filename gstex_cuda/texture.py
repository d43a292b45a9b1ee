"""gstex_cuda.texture — imported at nerfstudio/models/gstex.py:29."""
from gstex_amd.ops import rasterize_gaussians, texture_gaussians  # noqa: F401
