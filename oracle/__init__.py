"""CPU oracle for the gstex_amd hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker / the timed CPU baseline; the product (``gstex_amd``,
``gstex_cuda``) never imports it.

What it is: a plain PyTorch (CPU, fp32 + fp64) restatement of the textured-2DGS rasterizer whose
native source the reference does not ship (``/root/reference/.gitmodules:1-3`` points at the
un-vendored ``victor-rong/GStex_cuda``; no commit is pinned and nothing is installed here, see
SURVEY.md §0 and §8c).  Every function cites the reference call site whose contract it follows
and the device function of ``gstex_amd/csrc`` whose fp32 operation order it restates.

Parity status
-------------
* Host-side helpers (texel layout, query UVs, charting, UV frames, SH2RGB, quaternion frames) are
  PINNED against golden vectors generated from the reference's own pure-torch functions
  (``tests/golden/make_golden.py`` → ``tests/golden/*.npz``).
* The rasterizer itself (binning/sort order, composite forward, backward) is **parity unpinned**
  with respect to the reference CUDA kernels: they are absent, and the reference has no tests,
  fixtures or golden images for this path.  The oracle is pinned instead by
  closed-form known-answer tests (tests/test_oracle.py), finite differences of its own
  forward, and the call-site contracts.
"""
