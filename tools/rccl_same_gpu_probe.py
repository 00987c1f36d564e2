"""Probe: can two ranks on ONE MI355X form an RCCL ("nccl") group and run the
sharded path's all_gather_into_tensor?  (The 8-GPU node the sharded search is
built for is not available to this repo; this checks the device collective
itself at world 2.)  Run as:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 tools/rccl_same_gpu_probe.py
"""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x = torch.full((4,), float(rank + 1), device="cuda:0")
    out = torch.empty(4 * world, device="cuda:0")
    dist.all_gather_into_tensor(out, x)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_gather -> {out.tolist()}", flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
