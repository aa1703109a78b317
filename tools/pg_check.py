"""bench.py's N>1 process groups at world 1 on the one-GPU box: an RCCL
("nccl") default group with a gloo group beside it (the host-side wait of
the C-ABI multi-GPU leg), a barrier on each and an all-reduce.

usage: python tools/pg_check.py
"""
import os, torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)
g = dist.new_group(backend="gloo")
dist.barrier(group=g)
t = torch.ones(1, device="cuda"); dist.all_reduce(t); dist.barrier()
print("ok", t.item(), flush=True)
dist.destroy_process_group()
