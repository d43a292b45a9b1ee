"""Multi-view data parallelism (one process per device): the flat-buffer gradient all-reduce of
gstex_amd.dist.GradSync, exercised with world_size 2 on the gloo backend (CPU)."""
import os
import socket
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gstex_amd.dist import GradSync


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Params:
    def __init__(self, rank, n_tex):
        g = torch.Generator().manual_seed(7)
        self.means = torch.nn.Parameter(torch.randn(10, 3, generator=g))
        self.unused = torch.nn.Parameter(torch.randn(4, 3, generator=g))  # like features_dc: no grad
        self.texture = torch.nn.Parameter(torch.randn(n_tex, 3, generator=g))

    def parameters(self):
        return [self.means, self.unused, self.texture]


def _worker(rank, world, port, q, overlap=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = _Params(rank, 6)
        sync = GradSync(p, world, overlap_tail=overlap)
        sync.zero()
        # rank-dependent "loss": gradients differ per rank (independent cameras)
        ((rank + 1) * p.means.sum() + (rank + 2) * (p.texture ** 2).sum()).backward()
        assert p.means.grad.data_ptr() == sync.flat.data_ptr(), "grads must be views of the flat buffer"
        assert (sync._work is not None) == overlap, "the texel-gradient collective starts inside backward"
        sync.all_reduce()
        exp_means = torch.full((10, 3), (1 + 2) / 2.0)
        exp_tex = 2 * p.texture.detach() * ((2 + 3) / 2.0)
        ok1 = torch.allclose(p.means.grad, exp_means) and torch.allclose(p.texture.grad, exp_tex)
        ok1 = ok1 and torch.all(p.unused.grad == 0)
        # rechart: the texel store changes size -> the buffer is rebuilt and still reduces correctly
        p.texture = torch.nn.Parameter(torch.ones(9, 3))
        sync.zero()
        ((rank + 1) * p.texture.sum()).backward()
        sync.all_reduce()
        ok2 = torch.allclose(p.texture.grad, torch.full((9, 3), 1.5)) and sync.flat.numel() == 30 + 12 + 27
        q.put((rank, bool(ok1), bool(ok2)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_grad_all_reduce_world2(overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, overlap)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
    assert sorted(r[0] for r in res) == [0, 1]
    assert all(r[1] for r in res), "flat all-reduce did not average the gradients"
    assert all(r[2] for r in res), "flat buffer not rebuilt after the texel store changed size"
