"""Probe: can two ranks share the box's one GPU over RCCL (backend "nccl")?
Run under torchrun --nproc-per-node 2.  Every rank uses cuda:0."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((29410,), float(rank + 1), device="cuda:0")
dist.all_reduce(t)
torch.cuda.synchronize()
print("rank", rank, "all_reduce ok:", float(t[0]), flush=True)
dist.destroy_process_group()
