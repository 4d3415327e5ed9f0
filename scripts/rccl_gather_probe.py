#!/usr/bin/env python3
"""RCCL rehearsal of bench.py's frame gather on a 1-GPU box: a world-size-1 "nccl" process group, the
frame-in-flight pattern (two slot streams, async gather issued inside the slot's stream context, work
handle waited before the packed buffer is refilled), checked against the packed frame.  RCCL refuses
two ranks on one device, so the N > 1 data movement itself is only exercised by the driver's 8-GPU run."""
import os

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29531")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
streams = [torch.cuda.Stream(dev) for _ in range(2)]
n = 1 << 20
packed = [torch.zeros((1, n), device=dev) for _ in range(2)]
lists = [[torch.empty_like(packed[0])] for _ in range(2)]
pending = [None, None]
for k in range(8):
    s = k % 2
    with torch.cuda.stream(streams[s]):
        if pending[s] is not None:
            pending[s].wait()
            assert torch.equal(lists[s][0], packed[s]), k
        packed[s].fill_(float(k))
        pending[s] = dist.gather(packed[s], lists[s], dst=0, async_op=True)
for s in range(2):
    pending[s].wait()
torch.cuda.synchronize()
assert float(lists[0][0][0, 0]) == 6.0 and float(lists[1][0][0, 0]) == 7.0
dist.destroy_process_group()
print("rccl gather rehearsal ok")
