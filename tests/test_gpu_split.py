"""The split backward (gstex_raster_bwd with GSTEX_BWD_SPLIT, ABI 15): texel gradients by the
pixel-major kernel alone (TEXONLY) and splat gradients by the splat-parallel kernel (one splat per lane, transmittance
and colour-behind by lane scans), for the photometric C = 3 backward with float-atomic splat sums -- an experiment kept
off by default.  Held to the same oracle tolerances as the default path: the photometric parity cases
of test_gpu_parity.py and the deep bench-scene windows of test_gpu_deep.py, run with the switch on."""
import pytest

from gstex_amd import ops
from helpers import make_case, make_window_case

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def split(monkeypatch):
    monkeypatch.setattr(ops, "BWD_SPLIT", True)


@pytest.mark.parametrize("name", ["tex3_default", "no_aa", "no_reg", "settings0", "2dgs_T0", "opaque", "background",
                                  "ragged_17x33", "big_texel_blocks"])
def test_split_backward_photometric(name):
    from test_gpu_parity import _check_raster

    _check_raster(name, ("img", "alpha", "tex"))


def test_split_backward_cfg3_deep_window():
    from test_gpu_deep import _check

    _check("split cfg3 96x96", make_window_case(200_000, 1e7, 800, 800, 96), outputs=("img", "alpha", "tex"),
           min_depth=1500)


def test_split_backward_cfg2_window():
    from test_gpu_deep import _check

    _check("split cfg2 128x128", make_window_case(50_000, 1e6, 800, 800, 128), outputs=("img", "alpha", "tex"),
           min_depth=200)


def test_split_backward_cfg1_exact():
    from test_gpu_deep import _check

    _check("split cfg1 256x256", make_case(n=1000, n_texels=0, H=256, W=256, seed=42, opacity=0.1),
           outputs=("img", "alpha", "tex"))


def test_lane_scans():
    """The splat-parallel kernel's DPP lane scans (row_shr steps, row_bcast:15 / 31, wave_shr:1) on one wave."""
    import ctypes

    import torch

    from gstex_amd import _lib

    lib = _lib.load()
    fn = lib.gstex_debug_lane_scans
    fn.argtypes = [ctypes.c_void_p] * 3
    fn.restype = ctypes.c_int32
    g = torch.Generator().manual_seed(0)
    x = (0.5 + 0.5 * torch.rand(64, generator=g)).cuda()
    out = torch.full((192,), float("nan"), device="cuda")
    assert fn(x.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    o = out.cpu().double()
    xd = x.cpu().double()
    print("mul", o[:64].tolist())
    print("add", o[64:128].tolist())
    print("shift", o[128:].tolist())
    torch.testing.assert_close(o[:64], torch.cumprod(xd, 0), rtol=1e-5, atol=0)
    torch.testing.assert_close(o[64:128], torch.cumsum(xd, 0), rtol=1e-5, atol=0)
    assert o[128] == 0 and torch.equal(o[129:], xd[:63])
