"""Can two ranks share cuda:0 under the nccl (RCCL) backend on the 1-GPU box?  One all_reduce of a device tensor and
one of a float64 vector (the sharded_evaluate / sharded_shapley shapes).  python scripts/r06/nccl_probe.py"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    t = torch.full((4,), float(rank + 1), device="cuda:0")
    dist.all_reduce(t)
    d = torch.arange(6, dtype=torch.float64, device="cuda:0") * (rank + 1)
    dist.all_reduce(d)
    torch.cuda.synchronize()
    print(f"rank {rank}: {t.tolist()} {d.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(worker, args=(2, port), nprocs=2, join=True)
    print("nccl two ranks on one GPU: ok")
