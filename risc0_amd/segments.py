"""Segment-per-GPU sharding and timing.

Segments are independent proofs (risc0/zkvm/src/host/server/prove/prover_impl.rs:84-94
proves them in a loop; r0vm/src/actors/mod.rs:449-462 runs one worker process per
GPU). Here: one process per GPU (torch.distributed.run), segment i goes to rank
i mod world, and there is no collective on the prove path — the process group
(gloo) only carries the start/stop barriers and the max-over-ranks of the wall time.
"""
import time


def segments_for_rank(rank, world, n_segments):
    """Round-robin assignment of global segment indices to one rank."""
    return list(range(rank, n_segments, world))


def timed_segments(prove, segments, warmup, sync, dist=None):
    """Run `prove(seg)` for `warmup` untimed segments, then time every segment in
    `segments` between barrier+sync brackets. Returns (wall seconds, max over ranks)."""
    for i in range(warmup):
        prove(segments[i % len(segments)] if segments else i)
    sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for s in segments:
        prove(s)
    sync()
    t = time.perf_counter() - t0
    tmax = t
    if dist is not None:
        import torch
        tt = torch.tensor([t], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        tmax = float(tt[0])
        dist.barrier()
    return t, tmax
