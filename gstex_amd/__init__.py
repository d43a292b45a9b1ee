"""gstex_amd — MI355X-native (gfx950) differentiable rasterizer for GStex's per-primitive-textured
2D Gaussian splats.  Native code: libgstex_hip.so (C-ABI: include/gstex_hip.h); Python surface:
gstex_amd.ops (re-exported as the drop-in `gstex_cuda` package)."""
__version__ = "0.1.0"
