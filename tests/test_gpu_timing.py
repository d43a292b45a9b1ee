"""The fence-free timing events bench.py measures the roofline kernel with (gstex_timing_event_*, ABI 14) agree with
torch's default events on the same work."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_timing_events_match_torch_events():
    from gstex_amd import _lib

    x = torch.empty(1 << 28, device="cuda", dtype=torch.float32)  # 1 GiB of fills: ~0.15 ms each
    x.fill_(1.0)
    torch.cuda.synchronize()
    ours, theirs = [], []
    for _ in range(5):
        a, b = _lib.TimingEvent(), _lib.TimingEvent()
        c, d = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c.record()
        a.record()
        for _ in range(4):
            x.fill_(2.0)
        b.record()
        d.record()
        torch.cuda.synchronize()
        ours.append(a.elapsed_time(b))
        theirs.append(c.elapsed_time(d))
    o, t = sorted(ours)[2], sorted(theirs)[2]
    assert o > 0.0 and abs(o - t) <= 0.1 * t + 0.02, (ours, theirs)
