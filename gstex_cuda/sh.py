"""gstex_cuda.sh — imported at nerfstudio/models/gstex.py:32 and scripts/exporter.py:40."""
from gstex_amd.ops import num_sh_bases, spherical_harmonics  # noqa: F401
