"""World-size-2 gloo run of the segment-per-GPU harness (risc0_amd/segments.py) on
the CPU: sharding covers every segment exactly once, ranks never exchange segment
data, and the reported time is the max over ranks."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from risc0_amd.segments import segments_for_rank, timed_segments


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_segments, q):
    import time

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    done = []
    # rank 1 is made slower so the max-over-ranks is observable
    segs = segments_for_rank(rank, world, n_segments)
    t, tmax = timed_segments(lambda s: (done.append(s), time.sleep(0.02 * (1 + rank))), segs, warmup=1,
                             sync=lambda: None, dist=dist)
    q.put((rank, segs, done[1:], t, tmax))
    dist.destroy_process_group()


def test_round_robin_covers_all_segments():
    for world in (1, 2, 3, 8):
        got = sorted(s for r in range(world) for s in segments_for_rank(r, world, 64))
        assert got == list(range(64))


@pytest.mark.timeout(120)
def test_two_rank_gloo_timing_is_max_over_ranks():
    world, n = 2, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=100) for _ in range(world))
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    assert sorted(s for r in res for s in r[2]) == list(range(n))
    ts = [r[3] for r in res]
    for r in res:
        assert abs(r[4] - max(ts)) < 1e-9
    assert res[1][3] > res[0][3]
