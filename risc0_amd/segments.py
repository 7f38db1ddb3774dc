"""Segment-per-GPU sharding, timing and the local multi-GPU launcher.

Segments are independent proofs (risc0/zkvm/src/host/server/prove/prover_impl.rs:84-94
proves them in a loop; r0vm/src/actors/mod.rs:449-462 runs one worker process per
GPU). Here: one process per GPU, segment i goes to rank i mod world, and there is no
collective on the prove path — the process group (gloo) only carries the start/stop
barriers, the max-over-ranks of the wall time and the host-side gather of the results
(seal digests), as r0vm's receipt gather does.

The processes come either from an outside launcher (torch.distributed.run sets RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_*) or from launch_local(), which plays r0vm's role of
spawning one worker per GPU before anything touches a device.
"""
import os
import socket
import subprocess
import sys
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


def gather_results(local, dist=None):
    """Host-side gather of per-rank results (e.g. {segment: seal digest}) into one dict on
    every rank; no device data moves."""
    if dist is None:
        return dict(local)
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, dict(local))
    merged = {}
    for d in out:
        merged.update(d)
    return merged


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def narrow_visible_devices(local_rank, env):
    """Bind a rank to one GPU as r0vm binds each worker (CUDA_VISIBLE_DEVICES=idx,
    r0vm/src/actors/mod.rs:449-462): HIP_VISIBLE_DEVICES becomes the rank's one device — the
    local_rank-th entry of an inherited list, else the local_rank-th device the runtime sees
    (HIP indexes within ROCR_VISIBLE_DEVICES when that is set). The rank then opens ordinal 0.
    Marks env with R0_RANK_BOUND so a second call (the rank itself, after launch_local bound
    it) leaves it alone. Returns the HIP ordinal to open (0).
    An inherited list shorter than the ranks is a misconfigured launch: the ranks then share
    its devices round-robin, with a warning and R0_RANKS_SHARE_DEVICES=1 (bench.py reports
    it in its config line), rather than ending the job."""
    if env.get("R0_RANK_BOUND") == "1":
        return 0
    inherited = env.get("HIP_VISIBLE_DEVICES") or env.get("CUDA_VISIBLE_DEVICES")
    if inherited:
        devs = [d for d in inherited.split(",") if d.strip() != ""]
        if not devs:
            raise RuntimeError(f"no device in HIP_VISIBLE_DEVICES={inherited}")
        if local_rank >= len(devs):
            print(f"warning: local rank {local_rank} has no device of its own in HIP_VISIBLE_DEVICES={inherited}; "
                  f"sharing device {devs[local_rank % len(devs)].strip()}", file=sys.stderr)
            env["R0_RANKS_SHARE_DEVICES"] = "1"
        env["HIP_VISIBLE_DEVICES"] = devs[local_rank % len(devs)].strip()
    else:
        env["HIP_VISIBLE_DEVICES"] = str(local_rank)
    env.pop("CUDA_VISIBLE_DEVICES", None)
    env["R0_RANK_BOUND"] = "1"
    return 0


def rank_env(rank, world, port, base=None):
    """The environment torch.distributed.run gives rank `rank` of a one-node job, with the
    rank bound to its own GPU (narrow_visible_devices) before the child starts."""
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if env.get("R0_BENCH_SHARE_GPUS") != "1":  # rehearsal: the ranks share the visible devices
        narrow_visible_devices(rank, env)
    return env


def launch_local(world, argv, timeout=None):
    """Start `world` copies of `argv` (one per GPU: rank r sees only device r, as its
    ordinal 0), each with the rank environment above, and wait for all of them. Rank 0's stdout passes through;
    the other ranks' stdout is dropped (only rank 0 reports), stderr passes through.
    Returns the worst exit code. The caller must not have touched a GPU: the children
    open the devices."""
    port = free_port()
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen(argv, env=rank_env(r, world, port),
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    deadline = None if timeout is None else time.monotonic() + timeout
    for p in procs:
        try:
            left = None if deadline is None else max(1.0, deadline - time.monotonic())
            code = p.wait(timeout=left)
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    q.kill()
            code = 124
        if code != 0 and rc == 0:
            rc = code
    return rc


def maybe_launch(n_gpus, script, argv=None):
    """If this process is not already one rank of a job (no WORLD_SIZE) and n_gpus > 1,
    run the script as n_gpus local ranks and exit with their status. Returns otherwise."""
    if n_gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    args = sys.argv[1:] if argv is None else argv
    sys.exit(launch_local(n_gpus, [sys.executable, script] + list(args)))
