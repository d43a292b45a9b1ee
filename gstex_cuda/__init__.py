"""Drop-in `gstex_cuda` package backed by the MI355X-native gstex_amd library.

Resolves every name nerfstudio/models/gstex.py:28-32, models/jagged_texture.py:7-8 and
scripts/exporter.py:40 import from the (un-vendored) reference extension, so those files run
unchanged.  All compute goes through libgstex_hip.so (HIP, gfx950); see include/gstex_hip.h.
"""
# Load the submodules first: importing a submodule binds its name on the package, which would
# otherwise shadow the same-named functions (texture_sample, texture_edit) re-exported below.
from . import _torch_impl, get_aabb_2d as _m_aabb, sh, texture, texture_edit as _m_edit  # noqa: F401
from . import texture_sample as _m_sample  # noqa: F401
from gstex_amd.ops import (  # noqa: F401,E402
    get_aabb_2d,
    get_num_tiles_hit_2d,
    num_sh_bases,
    project_points,
    rasterize_gaussians,
    spherical_harmonics,
    texture_edit,
    texture_gaussians,
    texture_sample,
)

__all__ = [
    "get_aabb_2d",
    "get_num_tiles_hit_2d",
    "num_sh_bases",
    "project_points",
    "rasterize_gaussians",
    "spherical_harmonics",
    "texture_edit",
    "texture_gaussians",
    "texture_sample",
]
