"""Probe: can RCCL run several ranks on one GPU (for rehearsing bench --gpus N)?"""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", device_id=dev)
x = torch.full((world * 4,), rank, dtype=torch.uint8, device=dev)
y = torch.empty_like(x)
dist.all_to_all_single(y, x, [4] * world, [4] * world)
torch.cuda.synchronize()
print(rank, "ok", y.tolist(), flush=True)
dist.destroy_process_group()
