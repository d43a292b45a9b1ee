#!/usr/bin/env python3
"""bench.py's process-group setup on the box's one GPU (torchrun, world 1): the device bound before
init_process_group(backend "nccl" = RCCL, device_id=...), then an async all_reduce, a barrier and a wait -- the calls
the N > 1 bench makes, which a one-GPU box can otherwise not run."""
import os

import torch
import torch.distributed as dist

local_rank = int(os.environ.get("LOCAL_RANK", "0"))
dev = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method="env://", device_id=dev)
x = torch.arange(1 << 20, device=dev, dtype=torch.float32)
w = dist.all_reduce(x, op=dist.ReduceOp.SUM, async_op=True)
w.wait()
dist.barrier()
torch.cuda.synchronize()
assert float(x[12345]) == 12345.0
print(f"RCCL init OK: world {dist.get_world_size()}, backend {dist.get_backend()}, device {dev}")
dist.destroy_process_group()
