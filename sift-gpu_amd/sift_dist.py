"""Multi-GPU batch mode: images are independent, so a batch
is sharded across ranks with no data-path collective; the one exchange step is
the keypoint gather to rank `dst` (RCCL over xGMI with the "nccl" backend,
gloo on CPU for tests).

Gather protocol for one step's results:
  1. metadata: every rank's per-image keypoint offsets (its shard's batch + 1
     int32, padded to the largest shard) are all_gathered on a gloo group from
     pinned host copies -- host integers, so sizing the transfers never reads a
     device value back (no `.item()`, no device synchronisation);
  2. data: every rank r != dst sends exactly its count_r packed 28-byte
     keypoint records (and optionally descriptors) and rank dst posts one
     receive per peer, all in one batch_isend_irecv group, so the transfers
     run on the peers' xGMI links in parallel rather than through a ring.

`GatherPipeline` overlaps the gather of step i-1 with the compute of step i:
results are double-buffered (two slots), the offsets are copied to pinned host
memory behind each step's compute, and the host only ever waits for the
event of the step BEFORE the one just enqueued, so the GPU stays busy.  The
transfers run on a side stream that waits (on the device) for that step's
event, and the next compute into the same slot waits for the transfers.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

KP_WORDS = 7  # 28-byte cv::KeyPoint record as 7 int32 words


def shard(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block of images [start, end) = [floor(rank B / W), floor((rank + 1) B / W))
    owned by `rank` (the C ABI's sift_multi_shard)."""
    return total * rank // world, total * (rank + 1) // world


def shard_sizes(total: int, world: int) -> list[int]:
    return [b - a for a, b in (shard(total, world, r) for r in range(world))]


_META = {}


def _meta_group():
    """A gloo group for host-side metadata (the default group itself under
    gloo); created once per process group (a collective call on every rank)."""
    if dist.get_backend() == "gloo":
        return None
    key = id(dist.group.WORLD)
    if key not in _META:
        _META[key] = dist.new_group(backend="gloo")
    return _META[key]


class GatherPipeline:
    """Keypoint (and optional descriptor) gather to `dst`, one step behind compute.

    batches: every rank's batch size (shard_sizes), known on every rank.
    cap:     rows of each slot's kpts / desc buffers (records past cap are
             never written by the library and never sent).
    Usage per step i:   pipe.wait_slot(s); <enqueue compute into slot s>;
                        pipe.mark(s, offs_s); res = pipe.gather(prev slot, ...)
    and once at the end pipe.gather(last slot, ...).
    """

    def __init__(self, batches: list[int], cap: int, dst: int = 0, slots: int = 2, meta_group="auto",
                 timing: bool = False):
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        assert len(batches) == self.world
        self.batches, self.cap, self.dst = list(batches), cap, dst
        self.maxb = max(batches)
        self.meta = _meta_group() if meta_group == "auto" else meta_group
        self.cuda = torch.cuda.is_available() and dist.get_backend() != "gloo"
        pin = self.cuda
        self.host_offs = [torch.zeros(self.maxb + 1, dtype=torch.int32, pin_memory=pin) for _ in range(slots)]
        self.done = [None] * slots        # transfers of this slot finished (device event)
        self.ready = [None] * slots       # compute of this slot finished (device event)
        self.side = torch.cuda.Stream() if self.cuda else None
        # evidence for the bench line at N > 1: what this rank received per
        # peer and how long the side stream's transfers took
        self.gathers = 0
        self.recv_counts = [0] * self.world   # records received from each rank (dst only)
        self.sent_records = 0                 # records this rank sent (rank != dst)
        # (start, end) device events of each transfer group: only with
        # timing=True (bench.py), folded into _span_ms once complete so a long
        # run keeps a bounded list
        self.timing = timing
        self._spans = []
        self._span_ms = 0.0

    # -- compute side ---------------------------------------------------------
    def wait_slot(self, s: int):
        """The next compute into slot s must not overwrite records still being sent."""
        if self.cuda and self.done[s] is not None:
            torch.cuda.current_stream().wait_event(self.done[s])

    def mark(self, s: int, offs: torch.Tensor):
        """After enqueueing slot s's compute: copy its offsets to pinned host
        memory behind it (async) and remember the point."""
        b = self.batches[self.rank]
        self.host_offs[s][:b + 1].copy_(offs[:b + 1], non_blocking=True)
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            self.ready[s] = ev

    # -- gather side ----------------------------------------------------------
    def gather(self, s: int, kpts: torch.Tensor, desc: torch.Tensor | None = None):
        """Gather slot s (marked earlier) to dst.  Returns on dst
        (per-rank keypoint tensors, per-rank offsets (host), per-rank
        descriptors or None); None elsewhere.  The received tensors are
        complete once the side stream's work is done (pipe.sync())."""
        if self.cuda:
            self.ready[s].synchronize()   # the step before the one just enqueued: already done or nearly
        local = self.host_offs[s]
        allo = [torch.zeros(self.maxb + 1, dtype=torch.int32) for _ in range(self.world)]
        dist.all_gather(allo, local.clone() if self.cuda else local, group=self.meta)
        offs = [allo[r][:self.batches[r] + 1] for r in range(self.world)]
        counts = [min(int(o[-1]), self.cap) for o in offs]   # host ints: no device read
        recv_k, recv_d = {}, {}
        self.gathers += 1
        if self.rank == self.dst:
            for r in range(self.world):
                if r != self.dst:
                    self.recv_counts[r] += counts[r]
        else:
            self.sent_records += counts[self.rank]

        def post():
            # receive buffers are allocated here, on the stream that uses them
            ops = []
            if self.rank == self.dst:
                for r in range(self.world):
                    if r == self.dst or counts[r] == 0:
                        continue
                    recv_k[r] = torch.empty((counts[r], KP_WORDS), dtype=kpts.dtype, device=kpts.device)
                    ops.append(dist.P2POp(dist.irecv, recv_k[r], r))
                    if desc is not None:
                        recv_d[r] = torch.empty((counts[r], desc.shape[1]), dtype=desc.dtype, device=desc.device)
                        ops.append(dist.P2POp(dist.irecv, recv_d[r], r))
            elif counts[self.rank] > 0:
                ops.append(dist.P2POp(dist.isend, kpts[:counts[self.rank]], self.dst))
                if desc is not None:
                    ops.append(dist.P2POp(dist.isend, desc[:counts[self.rank]], self.dst))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()   # on CUDA: makes the current (side) stream wait, not the host

        if self.cuda:
            self.side.wait_event(self.ready[s])
            with torch.cuda.stream(self.side):
                t0 = None
                if self.timing:
                    t0 = torch.cuda.Event(enable_timing=True)
                    t0.record(self.side)
                post()
                ev = torch.cuda.Event(enable_timing=self.timing)
                ev.record(self.side)
                self.done[s] = ev
                if self.timing:
                    self._spans.append((t0, ev))
                    self._fold_spans()
        else:
            post()
        if self.rank != self.dst:
            return None
        ks, ds = [], []
        for r in range(self.world):
            if r == self.dst:
                ks.append(kpts[:counts[r]])
                ds.append(desc[:counts[r]] if desc is not None else None)
            else:
                ks.append(recv_k.get(r, kpts.new_empty((0, KP_WORDS))))
                ds.append(recv_d.get(r, desc.new_empty((0, desc.shape[1]))) if desc is not None else None)
        return ks, offs, (ds if desc is not None else None)

    def sync(self):
        if self.cuda:
            self.side.synchronize()

    def _fold_spans(self, keep: int = 8):
        """Adds the completed transfer spans (all but the newest `keep`) into
        _span_ms and drops their events."""
        while len(self._spans) > keep and self._spans[0][1].query():
            a, b = self._spans.pop(0)
            self._span_ms += a.elapsed_time(b)

    def reset_stats(self):
        self.gathers, self.sent_records = 0, 0
        self.recv_counts = [0] * self.world
        self._spans = []
        self._span_ms = 0.0

    def stats(self) -> dict:
        """Per-rank gather evidence since the last reset_stats(); call after
        sync().  transfer_ms = summed device time of the side stream's
        transfer groups (each from its start, i.e. after the step's compute,
        to the last receive/send completing)."""
        ms = None
        if self.cuda and self.timing:
            ms = self._span_ms + sum(a.elapsed_time(b) for a, b in self._spans)
        return {"backend": dist.get_backend(), "world_size": self.world, "rank": self.rank,
                "gathers": self.gathers, "received_records_per_rank": list(self.recv_counts),
                "sent_records": self.sent_records, "transfer_ms": ms}


class PipelinedSteps:
    """bench.py's step loop at N > 1: step i computes into slot i % 2 while
    step i-1's results are gathered to dst.

    bufs: per slot (kpts, desc, offs).  compute(kpts, desc, offs) enqueues one
    step.  on_result(step, gathered) is called on dst with each step's
    GatherPipeline.gather result (received tensors complete after sync())."""

    def __init__(self, pipe: GatherPipeline, bufs, with_desc: bool = False, on_result=None):
        assert len(bufs) == 2
        self.pipe, self.bufs, self.with_desc, self.on_result = pipe, bufs, with_desc, on_result
        self.i = 0

    def _gather(self, step):
        k, d, _ = self.bufs[step % 2]
        out = self.pipe.gather(step % 2, k, d if self.with_desc else None)
        if out is not None and self.on_result is not None:
            self.on_result(step, out)

    def step(self, compute):
        s = self.i % 2
        self.pipe.wait_slot(s)
        compute(*self.bufs[s])
        self.pipe.mark(s, self.bufs[s][2])
        if self.i > 0:
            self._gather(self.i - 1)
        self.i += 1

    def flush(self):
        """Gather the last step and wait for the side stream."""
        if self.i > 0:
            self._gather(self.i - 1)
        self.pipe.sync()
        self.i = 0


def gather_keypoints(kpts: torch.Tensor, offs: torch.Tensor, dst: int = 0,
                     desc: torch.Tensor | None = None, batches: list[int] | None = None):
    """One-shot gather of every rank's keypoints (and per-image offsets,
    optionally descriptors) to rank `dst` (GatherPipeline with one slot,
    waited for).  batches: every rank's batch size; default: every rank's
    len(offs) - 1, exchanged with one all_gather on the metadata group (shards
    may be uneven: sift_dist.shard gives them so whenever total % world != 0)."""
    world = dist.get_world_size()
    b = offs.shape[0] - 1
    if batches is None:
        mine = torch.tensor([b], dtype=torch.int64)
        allb = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allb, mine, group=_meta_group())
        batches = [int(x.item()) for x in allb]
    assert len(batches) == world and batches[dist.get_rank()] == b, (batches, b)
    pipe = GatherPipeline(batches, kpts.shape[0], dst, slots=1)
    pipe.mark(0, offs)
    out = pipe.gather(0, kpts, desc)
    pipe.sync()
    return out
