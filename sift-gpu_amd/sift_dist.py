"""Multi-GPU batch mode: images are independent, so a batch
is sharded across ranks with no data-path collective; the one exchange step is
the keypoint gather to rank 0 (RCCL over xGMI with the "nccl" backend, gloo on
CPU for tests).

Gather protocol, per step:
  1. all_gather of each rank's keypoint total (one int32 per rank) and of its
     per-image offsets (batch+1 int32) -- tiny;
  2. point-to-point: every rank r != dst sends its packed 28-byte keypoint
     records (exactly count_r of them) and rank dst posts one receive per
     peer, all in one batch_isend_irecv group, so the transfers run on the
     peers' xGMI links in parallel rather than through a ring.
Descriptors stay sharded (optionally gathered the same way).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

KP_WORDS = 7  # 28-byte cv::KeyPoint record as 7 int32 words


def shard(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block of images [start, end) owned by `rank` (image b -> rank floor(b*W/B))."""
    return total * rank // world, total * (rank + 1) // world


def gather_keypoints(kpts: torch.Tensor, offs: torch.Tensor, dst: int = 0,
                     desc: torch.Tensor | None = None):
    """Gather every rank's keypoints (and per-image offsets, optionally
    descriptors) to rank `dst`.

    kpts: (cap, 7) int32, offs: (batch+1,) int32 with offs[-1] = local total
    (may exceed cap; records beyond cap were not written and are not sent).
    Returns on dst: (list of per-rank kpt tensors, list of per-rank offsets,
    list of per-rank descriptor tensors or None); on other ranks: None.
    """
    world, rank = dist.get_world_size(), dist.get_rank()
    cap = kpts.shape[0]
    n_local = offs[-1:].to(torch.int32).clone()
    counts = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(counts, n_local)
    all_offs = [torch.zeros_like(offs) for _ in range(world)]
    dist.all_gather(all_offs, offs.contiguous())
    counts = [min(int(c.item()), cap) for c in counts]
    ops = []
    recv_k, recv_d = {}, {}
    if rank == dst:
        for r in range(world):
            if r == dst or counts[r] == 0:
                continue
            recv_k[r] = torch.empty((counts[r], KP_WORDS), dtype=kpts.dtype, device=kpts.device)
            ops.append(dist.P2POp(dist.irecv, recv_k[r], r))
            if desc is not None:
                recv_d[r] = torch.empty((counts[r], desc.shape[1]), dtype=desc.dtype, device=desc.device)
                ops.append(dist.P2POp(dist.irecv, recv_d[r], r))
    elif counts[rank] > 0:
        ops.append(dist.P2POp(dist.isend, kpts[:counts[rank]].contiguous(), dst))
        if desc is not None:
            ops.append(dist.P2POp(dist.isend, desc[:counts[rank]].contiguous(), dst))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != dst:
        return None
    ks, ds = [], []
    for r in range(world):
        if r == dst:
            ks.append(kpts[:counts[r]])
            ds.append(desc[:counts[r]] if desc is not None else None)
        else:
            ks.append(recv_k.get(r, torch.empty((0, KP_WORDS), dtype=kpts.dtype, device=kpts.device)))
            ds.append(recv_d.get(r) if desc is not None else None)
    return ks, all_offs, (ds if desc is not None else None)
