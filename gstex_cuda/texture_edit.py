"""gstex_cuda.texture_edit — imported at nerfstudio/models/gstex.py:30."""
from gstex_amd.ops import texture_edit  # noqa: F401
