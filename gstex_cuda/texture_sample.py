"""gstex_cuda.texture_sample — imported at nerfstudio/models/jagged_texture.py:7."""
from gstex_amd.ops import texture_sample  # noqa: F401
