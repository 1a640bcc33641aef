#!/usr/bin/env python3
"""Can two ranks share one GPU over RCCL on this box?  Rehearsal aid for
bench.py's N > 1 path on a one-GPU machine (the driver owns the 8-GPU runs).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29533 tools/rccl_probe.py

Every rank binds device LOCAL_RANK % device_count, inits the nccl (RCCL)
backend, and runs an all_reduce, a batch_isend_irecv pair and a barrier;
rank 0 prints one JSON line."""
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = torch.cuda.device_count()
    dev = local % max(n, 1)
    torch.cuda.set_device(dev)
    t0 = time.time()
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    rank, world = dist.get_rank(), dist.get_world_size()
    x = torch.full((1024,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    ok_ar = float(x[0].item()) == world * (world + 1) / 2
    peer = (rank + 1) % world
    src = (rank - 1) % world
    send = torch.full((4096,), float(rank), device="cuda")
    recv = torch.empty((4096,), device="cuda")
    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, send, peer), dist.P2POp(dist.irecv, recv, src)])
    for r in reqs:
        r.wait()
    torch.cuda.synchronize()
    ok_p2p = float(recv[0].item()) == float(src)
    dist.barrier()
    if rank == 0:
        print(json.dumps({"world": world, "devices": n, "device": dev, "backend": dist.get_backend(),
                          "all_reduce_ok": ok_ar, "p2p_ok": ok_p2p, "seconds": round(time.time() - t0, 2)}),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
