#!/usr/bin/env python3
"""Benchmark: RISC-V cycles proved per second at segment po2=20 (BASELINE.json metric).

A step proves one rv32im segment of 2^po2 cycles on one GPU the way the reference's
prove_core does (circuit/rv32im/src/prove/hal/mod.rs:143-224), from the segment's
preflight trace: the trace (a segment of one run of the datasheet's loop guest, restated
preflight, cut into consecutive segments where the executor cuts them) starts in page-locked
host memory, and the native segment pipeline (r0hip_prove_trace_segments) uploads it,
generates the witness, accumulates, proves to the seal (Vec<u32>) and checks the receipt on
the host, with in_flight segments on the GPU and the next trace uploading, as r0vm's GPU
worker queue runs segments. --witness times the prove core alone on a resident synthetic witness.
Multi-GPU: one process per GPU, whole segments sharded per rank, no data-path
collective (gloo only for the barriers, the max-time reduce and the host-side gather of
seal digests). The ranks come from torch.distributed.run, or — when `--gpus N` is given
without a launcher — from risc0_amd.segments.launch_local, which starts N rank processes
(rank r on device r) before anything touches a GPU, as r0vm spawns one worker per GPU.

Prints ONE JSON line (rank 0). Extra diagnostics go to stderr.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

P = 15 * 2**27 + 1


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a multiple of the segments in flight; enough segments that the pipeline's fill and drain
    # (the first trace's upload, the last segments finishing alone: ~20 ms per run) are a small
    # share — 3% of 12 segments, 1.5% of 24
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--po2", type=int, default=20)
    ap.add_argument("--circuit", default="rv32im")
    ap.add_argument("--hashfn", default="poseidon2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prove-only", action="store_true",
                    help="trace mode: skip the prove_only leg (profiling runs count only trace proofs)")
    ap.add_argument("--witness", action="store_true",
                    help="rv32im: time the prove core on a resident synthetic witness instead of the default "
                         "trace -> witness generation -> accumulation -> seal unit")
    ap.add_argument("--guest", default="loop_s", choices=["loop_s", "random_loop"],
                    help="trace mode: loop_s = the datasheet's benchmark guest (risc0/zkvm/examples/loop.s under the "
                         "v1compat kernel, datasheet.rs iteration counts); random_loop = a random 32-instruction "
                         "RV32IM body repeated until the segment suspends")
    ap.add_argument("--session", type=int, default=None,
                    help="trace mode, configs[3]: ONE loop.s session cut into this many consecutive segments "
                         "(tests/rv32im_trace.LoopSession); segment i goes to rank i mod N, every segment is proved "
                         "once in the timed region (steps = the rank's segments). Default for the loop guest up to "
                         "po2=22: N x --steps segments")
    ap.add_argument("--no-session", action="store_true",
                    help="trace mode: cycle --traces distinct single-segment traces per rank instead (the round-5 form)")
    ap.add_argument("--traces", type=int, default=None,
                    help="trace mode: distinct preflight traces per rank, cycled over the timed segments "
                         "(default 4 up to po2=22, 1 above)")
    ap.add_argument("--resident-steps", type=int, default=None,
                    help="trace mode: segments of the side leg that proves trace 0 from device memory "
                         "(r0hip_prove_segment_trace_resident; the round-4 headline); default --steps, 0 = skip")
    ap.add_argument("--e2e-steps", type=int, default=6,
                    help="segments of the witness end-to-end (pinned host witness groups -> H2D -> seal) leg; "
                         "0 = skip")
    ap.add_argument("--accum-steps", type=int, default=8,
                    help="segments of the leg that runs the rv32im accumulation inside the prover on the "
                         "resident witness (r0hip_prove_segment_accum), as the reference's prove_core does; "
                         "reported beside value as with_accumulation; 0 = skip")
    ap.add_argument("--per-op-steps", type=int, default=3,
                    help="trace mode: segments of the per_op_abi leg (rank 0): trace 0 proved by the reference prover "
                         "over the per-op r0hip_* symbols only (integration/hal_prover.cpp), as a Rust HipHal would "
                         "drive them; 0 = skip")
    ap.add_argument("--no-verify", action="store_true",
                    help="trace mode: skip the receipt check of each seal in the pipeline (A/B runs only)")
    ap.add_argument("--cpu-po2", type=int, default=None,
                    help="segment size of the CPU baseline proof (default: the bench's own po2, at most 20)")
    ap.add_argument("--inflight", type=int, default=None,
                    help="segments in flight per GPU (host threads, each with its own HIP stream); "
                         "default 6 up to po2=18, 3 up to po2=20, 2 up to po2=22, 1 above (one po2=24 segment needs ~150 GB)")
    return ap.parse_args()


def synthetic_witness(rng, circuit, po2):
    """Uniform canonical BabyBear words, seed 0x5249534330 + segment."""
    n = 1 << po2
    gs = circuit["group_sizes"]
    draw = lambda k: rng.integers(0, P, size=k, dtype=np.uint64).astype(np.uint32)
    return draw(gs[1] * n), draw(gs[2] * n), draw(gs[0] * n), draw(circuit["output_size"])


def main():
    args = parse()
    from risc0_amd.segments import maybe_launch
    maybe_launch(args.gpus, os.path.abspath(__file__))  # no WORLD_SIZE and --gpus > 1: spawn the ranks
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        # gloo reports its connections on the C++ stdout ("[Gloo] Rank 0 is connected ..."):
        # send that to stderr, so stdout carries only rank 0's JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", init_method="env://")
            dist.barrier()
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    import risc0_amd as r
    with open(os.path.join(ROOT, "risc0_amd", "circuits", args.circuit + ".taps.json")) as f:
        circ = json.load(f)
    device = 0
    if os.environ.get("R0_BENCH_SHARE_GPUS") == "1":
        # rehearsal of the N-rank path on fewer GPUs (tools/rehearsal/gpu_ranks.sh): ranks
        # share the visible devices round-robin; never set for a measurement
        import torch
        device = local_rank % max(1, torch.cuda.device_count())
        print(f"rank {rank}: R0_BENCH_SHARE_GPUS=1, device {device}", file=sys.stderr)
    elif world > 1:
        # one GPU per rank process, bound before the first HIP call as r0vm binds its workers
        # (r0vm/src/actors/mod.rs:449-462); launch_local has already done it for its children
        from risc0_amd.segments import narrow_visible_devices
        device = narrow_visible_devices(local_rank, os.environ)
        print(f"rank {rank}: HIP_VISIBLE_DEVICES={os.environ['HIP_VISIBLE_DEVICES']}", file=sys.stderr)
    hal = r.HipHal(args.hashfn, device=device)
    version = 2 if args.circuit == "rv32im" else None

    # inputs resident in HBM before the timed region: one witness set per rank
    rng = np.random.default_rng(0x5249534330 + rank)
    if args.po2 <= 22:
        code, data, accum, glob = synthetic_witness(rng, circ, args.po2)
        dc, dd, da, dg = (hal.copy_from_elem(k, v) for k, v in
                          (("code", code), ("data", data), ("accum", accum), ("global", glob)))
        host_witness = (code, data, accum, glob)
    else:
        # above po2=22 the host draw + upload would take minutes: draw on the device
        # (r0hip_fill_uniform, same distribution); no end-to-end leg at these sizes
        glob = synthetic_witness(rng, {"group_sizes": [0, 0, 0], "output_size": circ["output_size"]}, 0)[3]
        n = 1 << args.po2
        dc, dd, da = (hal.alloc_elem(k, circ["group_sizes"][g] * n) for k, g in (("code", 1), ("data", 2), ("accum", 0)))
        for i, b in enumerate((dc, dd, da)):
            r.check(r.lib().r0hip_fill_uniform(b.ptr, b.size, 0x5249534330 + rank * 8 + i))
        dg = hal.copy_from_elem("global", glob)
        host_witness = None

    from risc0_amd.segments import segments_for_rank, timed_segments, gather_results
    import hashlib
    import threading
    # global segment ids of this rank (segment-per-GPU, no collective on the prove path);
    # every segment of a rank proves the rank's resident inputs
    segs = segments_for_rank(rank, world, world * args.steps)
    # segments in flight per GPU: small segments are latency-bound (6 at po2<=18 measured
    # 5.32 -> 4.67 ms for recursion po2=18), po2=20 gains nothing past 3, po2>22 fits one
    inflight = args.inflight if args.inflight is not None else (6 if args.po2 <= 18 else 3 if args.po2 <= 20 else 2 if args.po2 <= 22 else 1)
    k = max(1, min(inflight, len(segs) or 1))
    # per-thread globals buffer: prove_segment zeroizes it in place; the witness
    # groups are only read and are shared
    globs = [dg] + [hal.copy_from_elem("global", glob) for _ in range(k - 1)]
    trace_mode = args.circuit == "rv32im" and not args.witness
    if trace_mode and args.guest == "loop_s" and not args.no_session and args.session is None and args.po2 <= 22:
        # the default workload: N x steps consecutive segments of one loop.s run, segment i on
        # rank i mod N (configs[1] per segment, configs[3] across the ranks)
        args.session = world * args.steps
    # recursion: a whole proof from the program and its preflight (RecursionProverImpl::prove,
    # circuit/recursion/src/prove/mod.rs:160-230: witness generation, ZK noise, accumulation,
    # prove), the lift/join shape with random programs (the lift/join .zkr files are not in the
    # reference checkout)
    program_mode = args.circuit == "recursion" and not args.witness

    def prove_witness(slot):
        return r.prove_segment(hal, args.circuit, args.po2, dc, dd, da, globs[slot], version=version)

    rt = trace = None
    traces, tjobs = [], []
    if trace_mode:
        # the headline unit is the reference's prove_core (prove/hal/mod.rs:143-224): a
        # preflight trace in host memory -> upload -> witness generation -> accumulation ->
        # seal, through the native segment pipeline as r0vm's GPU worker runs it. Each rank
        # builds --traces distinct traces (restated preflight: tests/rv32im_trace.py) into
        # page-locked memory before the timed region, and the timed segments cycle through them.
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import rv32im_trace as T  # the input generator: a restated preflight (test infrastructure, no oracle)
        ntr = args.traces if args.traces is not None else (4 if args.po2 <= 22 else 1)
        t0 = time.perf_counter()
        if args.session:
            # configs[3]: this rank's segments of one session, built in parallel worker processes
            # from the session's state at each (the executor's pass fast-forwards the others)
            mine = segments_for_rank(rank, world, args.session)
            args.steps = len(mine)
            tjobs, trace0 = session_jobs(r, args, mine)
            traces = [trace0] + [None] * (len(tjobs) - 1)
            ntr = 0
        for i in range(max(1, ntr) if not args.session else 0):
            seed = 0x5249534330 + 64 * rank + i
            if args.guest == "loop_s":
                # the datasheet's iteration count, shortened by a few iterations per trace so the
                # traces differ in their rows as well as in their seeds
                t_ = T.loop_s_trace(args.po2, T.loop_s_iterations(args.po2) - 37 * i, seed=seed)
            else:
                t_ = T.loop_trace(args.po2, body_len=32, seed=seed)
            cyc, tx = t_.arrays()
            idx, off, val = t_.injector_arrays()
            tjobs.append(r.TraceJob(*(r.pinned_copy(a) for a in (t_.global_words(), idx, off, val, cyc, tx)),
                                    t_.table_split_cycle, bigint=t_.bigint_array(),
                                    bigint_records=t_.bigint_records()))
            traces.append(t_)
        trace = traces[0]
        cyc, tx = trace.arrays()
        idx, off, val = trace.injector_arrays()
        bi = trace.bigint_array()
        rt = r.ResidentTrace(hal, args.po2, trace.global_words(), idx, off, val, cyc, tx, trace.table_split_cycle,
                             bigint=bi if len(bi) else None)
        bigint_records = trace.bigint_records() or None
        del cyc, tx, idx, off, val
        print(f"rank {rank}: {len(tjobs)} {args.guest} traces built in {time.perf_counter() - t0:.1f} s (trace 0: "
              f"{tjobs[0].table_split} rows before the tables, {tjobs[0].txns.size} memory transactions, "
              f"{tjobs[0].h2d_bytes() / 1e6:.0f} MB to upload)", file=sys.stderr)

    progs = []
    if program_mode:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import recursion_program as RP  # restated recursion preflight (test infrastructure, no oracle)
        nprog = args.traces if args.traces is not None else 2
        t0 = time.perf_counter()
        n = 1 << args.po2
        for i in range(max(1, nprog)):
            prng = np.random.default_rng(0x5249534330 + 64 * rank + i)
            prog, inp = RP.random_program(prng, n - RP.ZK_CYCLES - 1)
            pf = RP.preflight(prog, inp)
            wom, cyc_, iops = RP.trace_arrays(pf)
            u = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.uint32).reshape(-1))  # once, not per proof
            progs.append({"prog": prog, "pf": pf, "ctrl": hal.copy_from_elem("ctrl", RP.ctrl_group(prog, args.po2)),
                          "wom": u(wom), "cycles": u(cyc_), "iops": u(iops), "seed": 0x5EED + 64 * rank + i})
        print(f"rank {rank}: {len(progs)} recursion programs built in {time.perf_counter() - t0:.1f} s "
              f"({len(progs[0]['prog'].rows)} rows in program 0)", file=sys.stderr)

    def timed_leg(prove_one, label):
        phase_tot, last = {}, {}
        lock = threading.Lock()

        def prove_on(slot, n):
            for _ in range(n):
                seal, mix = prove_one(slot)
                prof = r.last_profile()
                with lock:
                    last["seal"], last["mix"] = seal, mix
                    for key, v in prof.items():
                        phase_tot[key] = phase_tot.get(key, 0.0) + v

        def prove_batch(batch):
            # `batch` segments over k host threads (r0vm-style queue depth)
            n = len(batch)
            share = [n // k + (1 if i < n % k else 0) for i in range(k)]
            ts = [threading.Thread(target=prove_on, args=(i, share[i])) for i in range(k) if share[i]]
            for t_ in ts:
                t_.start()
            for t_ in ts:
                t_.join()

        prove_batch([None] * max(args.warmup, k))  # warm every thread's stream, pool and tables
        phase_tot.clear()
        _t, t = timed_segments(prove_batch, [segs], 0, hal.synchronize, dist)
        phases = {key: round(v / args.steps, 3) for key, v in phase_tot.items()}
        if rank == 0:
            print(json.dumps({label + "_phases_ms": phases, "seal_words": int(last["seal"].size)}), file=sys.stderr)
        return t, last["seal"], last["mix"]

    resident = per_op = None
    if trace_mode:
        batch = [tjobs[i % len(tjobs)] for i in range(args.steps)]
        out = {}

        def pipeline(jobs_):
            # every seal checked by the native verifier beside the proofs (the worker unit returns
            # only receipts that verified, prover_impl.rs:262-280); a failed check fails the bench
            res = r.prove_trace_segments(hal, args.po2, jobs_, in_flight=k, per_job=True, verify=not args.no_verify)
            bad = [e for _, _, e, _, _ in res if e]
            if bad:
                raise RuntimeError(f"{len(bad)} of {len(res)} segments failed: {bad[0]}")
            out["res"] = [(sl, m) for sl, m, _, _, _ in res]
            out["verify_ms"] = [v for _, _, _, v, _ in res]
            out["prove_ms"] = [pm for _, _, _, _, pm in res]
        pipeline([tjobs[i % len(tjobs)] for i in range(max(args.warmup, k + 1))])  # warm every set, thread, pool
        _t, t = timed_segments(pipeline, [batch], 0, hal.synchronize, dist)
        seal, mix = out["res"][0]  # job 0 proved trace 0
        seals_distinct = len({sl.tobytes() for sl, _ in out["res"]})
        verify_ms = sum(out["verify_ms"]) / len(out["verify_ms"])
        t0 = time.perf_counter()
        pipeline([tjobs[0]])
        t_one = time.perf_counter() - t0
        # the one segment's latency, split: the prover's share (upload wait, witness generation,
        # accumulation, proof, seal to host), the receipt check after it, the rest (call set-up:
        # trace sets, threads; the Python wrapper)
        one_split = {"prove_ms": round(out["prove_ms"][0], 2), "verify_ms": round(out["verify_ms"][0], 2),
                     "other_ms": round(1000.0 * t_one - out["prove_ms"][0] - out["verify_ms"][0], 2)}
        rsteps = args.steps if args.resident_steps is None else args.resident_steps
        if rsteps > 0:
            t_r, seal_r, _ = timed_leg(lambda slot: r.prove_segment_trace_resident(hal, rt, bigint_records=bigint_records),
                                       "resident_trace")
            assert np.array_equal(seal_r, seal), "the resident trace's seal differs from the pipeline's"
            resident = {"value": round(world * args.steps * (1 << args.po2) / t_r, 1), "unit": "cycles/s",
                        "ms_per_step": round(1000.0 * t_r / args.steps, 3), "segments_in_flight_per_gpu": k,
                        "note": "trace 0 resident in HBM before the timed region (r0hip_prove_segment_trace_resident "
                                "from k host threads): the round-4 headline, no H2D"}
        if not args.no_prove_only:
            t_w, seal_w, _ = timed_leg(prove_witness, "prove_only")
        if args.per_op_steps > 0 and rank == 0:
            per_op = per_op_leg(hal, args, tjobs[0], seal, mix)
    elif program_mode:
        import itertools
        counter = itertools.count()

        def prove_program(slot, j=None):
            p = progs[next(counter) % len(progs) if j is None else j]
            return r.prove_recursion(hal, args.po2, p["ctrl"], p["wom"], p["cycles"], p["iops"], p["seed"])
        t, _, _ = timed_leg(prove_program, "program")
        seal, mix = prove_program(0, 0)  # program 0's seal, for the CPU parity check
        program_valid = r.verify_seal("recursion", hal.suite, seal, check_validity=True) == args.po2
        if not args.no_prove_only:
            t_w, seal_w, _ = timed_leg(prove_witness, "prove_only")
    else:
        t, seal, mix = timed_leg(prove_witness, "prove")
    mem = r.mem_stats()  # this rank's device footprint with k segments in flight
    # host-side gather of one seal digest per rank (the receipts stay on their hosts)
    digests = gather_results({rank: hashlib.sha256(seal.tobytes()).hexdigest()[:16]}, dist)
    # ranks that had to share a device (segments.narrow_visible_devices, or the rehearsal switch)
    shared = gather_results({rank: os.environ.get("R0_RANKS_SHARE_DEVICES") == "1"
                             or os.environ.get("R0_BENCH_SHARE_GPUS") == "1"}, dist)
    # a session's segments split unevenly when N does not divide it: the whole session counts
    cycles_total = (args.session if args.session else world * args.steps) * (1 << args.po2)
    value = cycles_total / t
    ms_per_step = 1000.0 * t / args.steps
    prove_only = None
    if (trace_mode or program_mode) and not args.no_prove_only:
        prove_only = {"value": round(cycles_total / t_w, 1), "unit": "cycles/s",
                      "ms_per_step": round(1000.0 * t_w / args.steps, 3),
                      "seal_sha256_rank0": hashlib.sha256(seal_w.tobytes()).hexdigest()[:16],
                      "note": "the prove core alone (r0hip_prove_segment) on a uniform synthetic witness (code, data "
                              "and accum groups) resident in HBM: no witness generation, no accumulation"}

    # kernel-level timing of the dominant kernel + roofline (rank 0)
    roofline = None
    cpu = None
    e2e = None
    acc_leg = None
    if rank == 0:
        prove_timed = ((lambda: r.prove_segment_trace_resident(hal, rt, bigint_records=bigint_records)) if trace_mode
                       else (lambda: prove_program(0, 0)) if program_mode else (lambda: prove_witness(0)))
        roofline = kernel_roofline(r, args, prove_timed, ms_per_step)
        # the side legs keep 2 in flight below po2 21 unless --inflight says otherwise: the
        # pipeline's uploader and a third prover measured slower there (63.1 against 57.6 ms)
        kl = k if args.inflight is not None else min(k, 2)
        if args.e2e_steps > 0 and host_witness is not None:
            e2e = end_to_end(r, hal, args, host_witness, kl, version)
        if args.accum_steps > 0 and args.circuit == "rv32im" and host_witness is not None:
            acc_leg = with_accumulation(r, hal, args, host_witness, kl, version)
        if not args.no_cpu_baseline and world == 1:
            cpu = (cpu_baseline_trace(args, trace, seal, mix) if trace_mode else
                   cpu_baseline_program(args, progs[0], seal, mix) if program_mode else
                   cpu_baseline(args, circ, seal, mix))
    del host_witness

    if rank == 0:
        workload = (f"{args.circuit} segment po2={args.po2}, {args.hashfn} hashfn, from its preflight trace in page-locked "
                    "host memory: upload -> witness generation -> accumulation -> seal on host (the reference's "
                    "prove_core), through the native segment pipeline (r0hip_prove_trace_segments), each receipt "
                    "checked by the native verifier before it is returned"
                    if trace_mode else
                    f"recursion segment po2={args.po2}, {args.hashfn} hashfn, from the program (control group resident) "
                    "and its preflight in host memory: witness generation -> ZK noise -> accumulation -> seal on host "
                    "(RecursionProverImpl::prove, r0hip_prove_recursion)"
                    if program_mode else
                    f"{args.circuit} segment po2={args.po2}, {args.hashfn} hashfn, witness resident in HBM -> seal on host")
        if trace_mode and args.session:
            data = (f"synthetic: ONE run of the datasheet's loop guest (risc0/zkvm/examples/loop.s under a restated "
                    f"v1compat kernel) cut into {args.session} consecutive po2={args.po2} segments where the executor "
                    "cuts them (tests/rv32im_trace.LoopSession: each resumes from the previous one's final memory and "
                    "root); segment i on rank i mod N, each proved once")
        elif trace_mode and args.guest == "loop_s":
            data = (f"synthetic: the datasheet's loop guest (risc0/zkvm/examples/loop.s under a restated v1compat kernel; "
                    f"{T.loop_s_iterations(args.po2)} iterations less 37 per trace, datasheet.rs:42-58), preflight restated "
                    f"from the reference executor (tests/rv32im_trace.py); {len(traces)} distinct seeded traces per rank, "
                    "cycled over the segments")
        elif trace_mode:
            data = (f"synthetic (a loop guest: random 32-instruction RV32IM body, repeated until the segment suspends; "
                    f"preflight restated from the reference executor, tests/rv32im_trace.py; {len(traces)} distinct "
                    "seeded traces per rank)")
        elif program_mode:
            data = (f"synthetic: {len(progs)} random recursion programs per rank (micro ops, Poseidon2 load/partial/"
                    "store, IOP reads, mix_rng; tests/recursion_program.py with its restated preflight), "
                    f"{len(progs[0]['prog'].rows)} rows in program 0; the lift/join programs are not in the "
                    "reference checkout")
        else:
            data = "synthetic (uniform BabyBear witness, seeded per segment)"
        line = {
            "metric": f"RISC-V cycles proved/sec at segment po2={args.po2}",
            "value": round(value, 1),
            "unit": "cycles/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (BabyBear Montgomery, exact modular integer)",
            "data": data,
            "config": {"workload": workload,
                       "circuit": args.circuit, "po2": args.po2, "hashfn": args.hashfn,
                       "segments_per_gpu": args.steps, "segments_in_flight_per_gpu": k,
                       # the runtime's default (4) unless the caller's environment sets another count
                       "hip_hw_queues_per_process": int(os.environ.get("GPU_MAX_HW_QUEUES") or 4),
                       "parallelism": f"segment-per-gpu x{world}",
                       "seal_sha256_by_rank": [digests[i] for i in range(world)],
                       **({"session_segments": args.session} if args.session else {}),
                       **({"guest": args.guest, "distinct_traces_per_rank": len(traces),
                           "distinct_seals_rank0": seals_distinct,
                           "h2d_bytes_per_segment": int(tjobs[0].h2d_bytes()),
                           "receipts_verified": not args.no_verify, "verify_ms_per_segment": round(verify_ms, 2),
                           "ms_one_segment_unpipelined": round(1000.0 * t_one, 1),
                           "one_segment_split": one_split} if trace_mode else {}),
                       **({"programs_per_rank": len(progs), "seal_valid_rank0": bool(program_valid)}
                          if program_mode else {}),
                       "ranks_share_devices": any(shared[i] for i in range(world))},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "device_memory_gb": {"peak_reserved": round(mem["peak_reserved"] / 1e9, 2),
                                 "peak_live": round(mem["peak_live"] / 1e9, 2)},
        }
        if prove_only:
            line["prove_only"] = prove_only
        if e2e:
            line["end_to_end"] = e2e
        if resident:
            line["resident_trace"] = resident
        if per_op:
            line["per_op_abi"] = per_op
        if acc_leg:
            line["with_accumulation"] = acc_leg
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()
    if rank == 0 and cpu and (cpu.get("seal_equal") is False or cpu.get("mix_equal") is False):
        # full-size oracle parity failed: the line above carries both digests
        print("bench: GPU seal differs from the CPU oracle's on the same input", file=sys.stderr)
        sys.exit(1)


def session_jobs(r, args, mine):
    """configs[3]'s input for this rank: segments `mine` of ONE loop.s session of args.session
    segments (tests/rv32im_trace.LoopSession). The executor's pass fast-forwards the session here
    (a fraction of a second per segment); this rank's first segment is built in this process (its
    Trace feeds the CPU baseline), the others in worker processes from the session's state at each.
    Returns (TraceJobs in page-locked memory, the first segment's Trace)."""
    import concurrent.futures as cf
    import multiprocessing as mp
    import rv32im_trace as T
    it = T.loop_s_session_iterations(args.po2, args.session)
    seed = 0x5249534330
    S = T.LoopSession(args.po2, it, seed=seed)
    states, tr0 = {}, None
    t0 = time.perf_counter()
    for k in range(max(mine) + 1):
        if k == mine[0]:
            tr0 = S._advance(build=True)
            continue
        if k in mine:
            states[k] = S.state()
        S._advance(build=False)
    assert S.terminated == (max(mine) == args.session - 1), "the session does not end at its last segment"
    print(f"session of {args.session} segments: fast-forwarded to segment {max(mine)} in "
          f"{time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)

    def job(g, idx, off, val, cyc, tx, split, bi, recs):
        return r.TraceJob(*(r.pinned_copy(a) for a in (g, idx, off, val, cyc, tx)), split, bigint=bi,
                          bigint_records=recs)
    cyc, tx = tr0.arrays()
    jobs = {mine[0]: job(tr0.global_words(), *tr0.injector_arrays(), cyc, tx, tr0.table_split_cycle,
                         tr0.bigint_array(), tr0.bigint_records())}
    workers = max(1, min(8, len(states)))
    if states:
        with cf.ProcessPoolExecutor(workers, mp_context=mp.get_context("spawn"), initializer=_session_worker_init,
                                    initargs=(os.path.join(ROOT, "tests"),)) as ex:
            futs = {ex.submit(_build_segment, args.po2, it, seed, st): k for k, st in states.items()}
            for n, f in enumerate(cf.as_completed(futs)):
                out = f.result()
                jobs[futs[f]] = job(*out[:9])
                if n % 8 == 7:
                    print(f"  {n + 1}/{len(states)} segments built", file=sys.stderr, flush=True)
    return [jobs[k] for k in mine], tr0


def _session_worker_init(tests_dir):
    sys.path.insert(0, tests_dir)


def _build_segment(po2, iterations, seed, state):
    import rv32im_trace as T
    return T.build_session_segment(po2, iterations, seed, state)


def per_op_leg(hal, args, job, pipeline_seal, pipeline_mix):
    """The drop-in path's own number: trace 0 proved by the reference prover over ONLY the per-op
    r0hip_* symbols (integration/hal_prover.cpp: the injector scatter, r0hip_rv32im_witgen, the
    Prover's make_coeffs / commit_group / finalize / fri_prove and the accumulation, one
    synchronous call per Hal method, has_unified_memory() = false, the node reads of Merkle openings
    from the HAL buffer's host mirror of each node heap), what a Rust HipHal behind
    risc0_zkp::hal::Hal delivers; one
    segment at a time, from the trace in host memory. Its seal must equal the pipeline's."""
    sys.path.insert(0, os.path.join(ROOT, "integration"))
    import halprover
    halprover.prove_trace(hal, args.po2, job)  # warm the calling thread's pool and the driver
    phases, seal = {}, None
    t0 = time.perf_counter()
    for _ in range(args.per_op_steps):
        seal, mix = halprover.prove_trace(hal, args.po2, job)
        for k_, v in halprover.last_profile().items():
            phases[k_] = phases.get(k_, 0.0) + v / args.per_op_steps
    t = time.perf_counter() - t0
    return {"value": round(args.per_op_steps * (1 << args.po2) / t, 1), "unit": "cycles/s",
            "ms_per_step": round(1000.0 * t / args.per_op_steps, 3), "steps": args.per_op_steps,
            "seal_equal": bool(np.array_equal(seal, pipeline_seal)), "mix_equal": bool(np.array_equal(mix, pipeline_mix)),
            "host_phases_ms": {k_: round(v, 2) for k_, v in phases.items()},
            "note": "trace 0 through the reference prover over the per-op C ABI only (integration/hal_prover.cpp, "
                    "libr0hip_halprover.so), one segment at a time; seal compared with the pipeline's seal of trace 0"}


HBM_PEAK_GBS = 8000.0
# Chip VALU issue roof in wave64 instructions/s: 256 CUs x 4 SIMDs, one wave64 instruction
# per 4 cycles per SIMD at 2.4 GHz. That is the measured issue cost of the 32-bit integer
# VOP3 ops these kernels are made of (v_mad_u64_u32, v_mul_lo_u32, v_min_u32, v_lshl_add_u64:
# 29-34 T lane-instructions/s in profiles/archive/r1_valu_rates.txt) and the unit SQ_ACTIVE_INST_VALU
# counts in (ACTIVE_INST_VALU x 4 = SQ_INSTS_VALU exactly, profiles/archive/r2a_pmc_valu.json).
VALU_PEAK_GIPS = 256 * 4 * 2.4e9 / 4 / 1e9
# The binding resource of each launcher family: the hash, eval_check and
# evaluate_any kernels are integer-VALU-issue bound; the NTT/eltwise ones move bytes.
VALU_BOUND = {"eval_check", "hash_rows", "merkle_fold", "batch_evaluate_any"}


def kernel_roofline(r, args, prove, ms_per_step):
    """Time every kernel family of one proof with HIP events on the library stream
    (r0hip_kernel_times) and quote the dominant one against the resource that binds it:
    VALU instruction issue (SQ_INSTS_VALU per launch from the committed PMC pass of this
    bench, over the measured launch time) for the integer-arithmetic kernels, HBM otherwise;
    the HBM view is always reported beside it."""
    # the main thread has its own stream/pool: warm it first so no first-use
    # allocation lands inside a timed launcher
    prove()
    r.set_kernel_timing(True)
    prove()
    times = r.kernel_times()
    r.set_kernel_timing(False)
    if not times:
        return None
    name, (ms, calls, alg_bytes, alg_mm) = max(times.items(), key=lambda kv: kv[1][0])
    print(json.dumps({"kernel_times_ms": {k: [round(v[0], 3), v[1]] for k, v in times.items()}}), file=sys.stderr)
    avg_s = ms / 1000.0 / calls
    per_launch = alg_bytes / calls
    gbs = per_launch / avg_s / 1e9
    hbm = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}
    traffic, tsrc = pmc_traffic(name, calls, args)
    fam = name.split("_poseidon2")[0].split("_sha")[0]
    insts, busy, vsrc = pmc_valu(fam, args)
    vsrc, vmatch = vsrc if vsrc else (None, None)
    if fam in VALU_BOUND and insts:
        gips = insts / avg_s / 1e9
        out = {"kernel": name, "bound": "valu", "achieved": round(gips, 1), "peak": VALU_PEAK_GIPS,
               "unit": "G VALU instructions/s (wave64)", "frac": round(gips / VALU_PEAK_GIPS, 4),
               "valu_insts_per_launch": int(insts), "issue_busy_frac": busy, "valu_source": vsrc,
               "valu_source_matches_library": vmatch,
               "note": "integer modular arithmetic bound by VALU issue: executed VALU instructions per launch "
                       "(PMC SQ_INSTS_VALU) over the launch time, against 1024 SIMDs x one wave64 instruction "
                       "per 4 cycles at 2.4 GHz. Full-rate 32-bit ops issue in 2 cycles, so this frac is an upper "
                       "bound: eval_check_issue prices each instruction at its own cost. issue_busy_frac is the "
                       "same count over the SIMD cycles at the measured clock (SQ_ACTIVE_INST_VALU)"}
        ec = ec_issue(args, avg_s, insts) if fam == "eval_check" else None
        if ec:
            out["eval_check_issue"] = ec
    else:
        out = {"kernel": name, "bound": "hbm", **hbm}
    out.update({"traffic": traffic, "alg_bytes_per_launch": int(per_launch), "avg_launch_ms": round(avg_s * 1000, 4)})
    if alg_mm:
        # the program's field multiplications (as the reference's poly_fp writes them) per second:
        # a rate, not a roof (the kernels need fewer instructions per product than a canonical
        # Montgomery multiply, so no hardware peak bounds it)
        out["alg_modmul"] = {"per_launch": int(alg_mm / calls), "achieved": round(alg_mm / calls / avg_s / 1e12, 3),
                             "unit": "T modmul/s"}
    seg = segment_valu(args, ms_per_step)
    if seg:
        out["segment_valu"] = seg
    if out["bound"] != "hbm":
        out["hbm"] = hbm
    if tsrc:
        out["traffic_source"] = tsrc
    return out


def ec_issue(args, avg_s, insts):
    """eval_check's launch against issue roofs that price each instruction at its own cost, from
    the committed instruction mix of the generated kernels (profiles/r*_ec_inst_mix.json,
    tools/ec_inst_mix.py: per-kernel static VALU counts of the straight-line kernels, equal to the
    PMC per-wave counts): the guide's cycles (2 for full-rate 32-bit ops, 4 for the rest) at
    2.4 GHz, and the chip rates measured for each instruction alone (r1_valu_rates.txt)."""
    path = pmc_summary_file("ec_inst_mix", prefix="")
    if path is None or args.circuit != "rv32im":
        return None
    with open(path) as f:
        d = json.load(f)
    waves = insts / d["valu_per_point"]  # wave64 launches of the whole program
    t_cyc = waves * d["issue_cycles_per_point"] / (256 * 4 * 2.4e9)
    t_meas = waves * d["measured_rate_s_per_wave"]
    t4 = insts * 4 / (256 * 4 * 2.4e9)
    return {"valu_per_point": d["valu_per_point"], "issue_cycles_per_point": d["issue_cycles_per_point"],
            "full_rate_share": round(sum(k["full_rate_share"] * k["valu_per_wave"] for k in d["kernels"].values())
                                     / d["valu_per_point"], 4),
            "frac_4cycle": round(t4 / avg_s, 4), "frac_issue_weighted": round(t_cyc / avg_s, 4),
            "frac_measured_rates": round(t_meas / avg_s, 4),
            "min_ms_issue_weighted": round(t_cyc * 1e3, 3), "min_ms_measured_rates": round(t_meas * 1e3, 3),
            "source": os.path.relpath(path, ROOT), "source_matches_library": d.get("lib_sha256_16") == lib_fingerprint(),
            "note": "the launch time against the time its instructions need at full issue: every instruction at 4 "
                    "cycles (frac_4cycle, as frac), at the guide's cost (2 cycles for full-rate 32-bit ops, 4 for "
                    "64-bit / multiply / VOP3-only ops; frac_issue_weighted, the lower bound), and at the chip rate "
                    "measured for each instruction alone at 4 waves per SIMD (frac_measured_rates, which carries the "
                    "clock the chip holds under integer load)"}


def segment_valu(args, ms_per_step):
    """the whole segment's executed VALU instructions (every kernel of a proof, from the committed
    PMC pass of this bench) against the issue roof and the bench's own time per segment: how much
    of the step the GPU needs at full 4-cycle issue"""
    if args.circuit != "rv32im" or args.po2 != 20 or args.hashfn != "poseidon2":
        return None
    path = pmc_summary_file("valu")
    if path is None:
        return None
    with open(path) as f:
        ks = json.load(f)["kernels"]
    proofs = ks.get("ec_rv32im::k0<true>", ks.get("ec_rv32im::k0<false>", {})).get("dispatches")
    if not proofs:
        return None
    per_proof = sum(d["insts_valu"] for d in ks.values()) / proofs
    ms = per_proof / (VALU_PEAK_GIPS * 1e9) * 1e3
    return {"valu_insts_per_segment": int(per_proof), "ms_at_issue_peak": round(ms, 2), "ms_per_step": round(ms_per_step, 3),
            "frac": round(ms / ms_per_step, 4), "source": os.path.relpath(path, ROOT),
            "note": "every kernel's executed VALU instructions per proof (PMC SQ_INSTS_VALU over the run's proofs) at "
                    "one wave64 instruction per 4 cycles on 1024 SIMDs at 2.4 GHz, over the bench's ms per segment"}


def lib_fingerprint():
    """first 16 hex digits of the sha256 of the loaded libr0hip.so: the committed PMC summaries
    record the library they were measured on (tools/gpu_round.sh), so a stale count is visible"""
    import hashlib
    from risc0_amd import hal
    with open(hal.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def pmc_summary_file(kind, prefix="pmc_"):
    """the committed PMC summary to quote (profiles/r<round><tag>_pmc_<kind>.json): the newest one
    measured on the loaded library (its lib_sha256_16), else the newest. Round tags order by
    round, then tag length, then tag (r5z < r5aa < r5an), not as plain strings."""
    import glob
    import re

    def key(path):
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{prefix}{kind}.json")), key=key)
    if not files:
        return None
    lib = lib_fingerprint()
    for path in reversed(files):
        with open(path) as f:
            if json.load(f).get("lib_sha256_16") == lib:
                return path
    return files[-1]


def pmc_valu(family, args):
    """VALU instructions per launch of `family` and the time-weighted share of SIMD cycles
    issuing VALU, from the newest committed rocprofv3 --pmc summary of this bench
    (profiles/r*_pmc_valu.json, tools/pmc_summary.py). PMC counters cannot be read inside
    the timed process, so these are the committed measurement, labelled by file."""
    if args.circuit != "rv32im" or args.po2 != 20 or args.hashfn != "poseidon2":
        return None, None, None
    path = pmc_summary_file("valu")
    if path is None:
        return None, None, None
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from rocprof_families import family as fam_of
    with open(path) as f:
        doc = json.load(f)
    ks = doc["kernels"]
    matches = doc.get("lib_sha256_16") == lib_fingerprint()
    insts = tot = busy = 0.0
    for k, d in ks.items():
        if fam_of(k) != family or not d["dispatches"]:
            continue
        # per launcher call: every kernel of the family runs once per call (eval_check: the
        # 30 generated kernels), so average each kernel over its own dispatches
        insts += d["insts_valu"] / d["dispatches"] if family == "eval_check" else d["insts_valu"]
        util = d["active_inst_valu"] * 4 / (256 * 4 * d["gui_active_cycles"]) if d["gui_active_cycles"] else 0
        tot += d["ms"]
        busy += d["ms"] * min(util, 1.0)
    if family != "eval_check":
        insts = None  # launches per proof differ per kernel: only eval_check is quoted per launch
    if tot == 0:
        return None, None, None
    return insts, round(busy / tot, 3), (os.path.relpath(path, ROOT), matches)


def mixed_arm_rows(data, n):
    """The bench's uniform rv32im data rows with the instruction selectors (data columns
    1..13) zeroed so each cycle takes one random instruction arm of the accumulation step."""
    rng = np.random.default_rng(0x41434355)
    arms = rng.integers(0, 13, n)
    data = data.reshape(211, n).copy()
    for j, col in enumerate(range(1, 14)):
        data[col, arms > j] = 0  # the first nonzero selector wins (if / else-if mux)
    data[32, arms == 12] = 0     # the big-integer arm's polyOp decodes one-hot (0 = nop)
    return data.reshape(-1)


def with_accumulation(r, hal, args, witness, k, version):
    """The prove core as the reference's rv32im prove_core runs it (prove/hal/mod.rs:205-212):
    commit code and data, draw mix, run the accumulation on the device (all three phases,
    r0hip_prove_segment_accum), commit accum, finalize. The accum group starts INVALID as
    the witness generator allocates it (a device fill inside the timed region). Data rows are
    the bench's uniform words with the instruction selectors (data columns 1..13) zeroed so
    each cycle takes one random instruction arm (mixed arms in every wavefront, the
    accumulation step's divergent case). Reported beside `value`, never as it."""
    import threading
    n = 1 << args.po2
    code, data, _accum, glob = witness
    data = mixed_arm_rows(data, n)
    dc, dd = hal.copy_from_elem("code", code), hal.copy_from_elem("data", data)
    accs = [hal.alloc_elem("accum", 103 * n) for _ in range(k)]
    globs = [hal.copy_from_elem("global", glob) for _ in range(k)]
    acc_ms, per = [], []

    def run(slot, count):
        for _ in range(count):
            r.check(r.lib().r0hip_memset32(accs[slot].ptr, 0xFFFFFFFF, accs[slot].size))
            t0 = time.perf_counter()
            r.prove_segment_accum(hal, "rv32im", args.po2, dc, dd, accs[slot], n, globs[slot], version=version)
            prof = r.last_profile()
            acc_ms.append(prof.get("accumulate", 0.0))
            per.append((slot, round(1000 * (time.perf_counter() - t0), 1), {k_: round(v, 1) for k_, v in prof.items()}))

    def batch(count):
        share = [count // k + (1 if i < count % k else 0) for i in range(k)]
        ts = [threading.Thread(target=run, args=(i, share[i])) for i in range(k) if share[i]]
        for t_ in ts:
            t_.start()
        for t_ in ts:
            t_.join()

    batch(2 * k)  # warm every thread's stream, pool and scratch
    acc_ms.clear()
    hal.synchronize()
    m0 = r.mem_stats()["mallocs"]
    t0 = time.perf_counter()
    batch(args.accum_steps)
    hal.synchronize()
    t = time.perf_counter() - t0
    mallocs = r.mem_stats()["mallocs"] - m0
    print(json.dumps({"with_accumulation_proofs": per[-args.accum_steps:]}), file=sys.stderr)
    return {"value": round(args.accum_steps * n / t, 1), "unit": "cycles/s",
            "ms_per_step": round(1000 * t / args.accum_steps, 3), "steps": args.accum_steps,
            "segments_in_flight_per_gpu": k,
            "accumulate_phase_ms": round(sum(acc_ms) / max(1, len(acc_ms)), 3),
            "hipmallocs_in_timed_region": mallocs,
            "note": "prove core including the rv32im accumulation on the device (r0hip_prove_segment_accum); "
                    "data rows take one random instruction arm per cycle"}


def end_to_end(r, hal, args, witness, k, version):
    """PCIe-inclusive leg (prove core vs end-to-end) through the native
    segment pipeline (r0hip_prove_segments): every segment's witness groups start in
    page-locked host memory; an uploader thread fills one of k+1 device buffer sets while
    k prover threads run (r0vm's GPU_QUEUE_DEPTH). Reported beside
    `value`, never as it."""
    import ctypes
    lib = r.lib()
    hosts = []
    try:
        for a in witness:
            p = ctypes.c_void_p()
            r.check(lib.r0hip_host_alloc(ctypes.byref(p), a.size * 4))
            hosts.append(p.value)
            np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32)), shape=(a.size,))[:] = a
        h2d_bytes = sum(a.size * 4 for a in witness)
        jobs = lambda n: [tuple(hosts)] * n
        r.prove_segments(hal, args.circuit, args.po2, jobs(k), version=version, in_flight=k)  # warm
        t0 = time.perf_counter()
        r.prove_segments(hal, args.circuit, args.po2, jobs(1), version=version, in_flight=1)
        t_one = time.perf_counter() - t0
        t0 = time.perf_counter()
        r.prove_segments(hal, args.circuit, args.po2, jobs(args.e2e_steps), version=version, in_flight=k)
        t = time.perf_counter() - t0
        dev_acc = None
        if args.circuit == "rv32im":
            # witgen's output only (code, data with mixed instruction arms, globals): each
            # prover accumulates on the device, the accum group never crosses PCIe
            p = ctypes.c_void_p()
            r.check(lib.r0hip_host_alloc(ctypes.byref(p), witness[1].size * 4))
            hosts.append(p.value)
            np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32)),
                                  shape=(witness[1].size,))[:] = mixed_arm_rows(witness[1], 1 << args.po2)
            ajobs = lambda n: [(hosts[0], p.value, None, hosts[3])] * n
            r.prove_segments(hal, args.circuit, args.po2, ajobs(k), version=version, in_flight=k)  # warm
            t0 = time.perf_counter()
            r.prove_segments(hal, args.circuit, args.po2, ajobs(args.e2e_steps), version=version, in_flight=k)
            ta = time.perf_counter() - t0
            dev_acc = {"value": round(args.e2e_steps * (1 << args.po2) / ta, 1), "unit": "cycles/s",
                       "ms_per_step": round(1000.0 * ta / args.e2e_steps, 3),
                       "h2d_bytes_per_segment": int(witness[0].size * 4 + witness[1].size * 4 + witness[3].size * 4),
                       "note": "code, data (mixed instruction arms) and globals from pinned host memory; the "
                               "accumulation runs on the device inside each proof (job h_accum = NULL)"}
    finally:
        for hp in hosts:
            r.check(lib.r0hip_host_free(hp))
    return {"value": round(args.e2e_steps * (1 << args.po2) / t, 1), "unit": "cycles/s",
            "ms_per_step": round(1000.0 * t / args.e2e_steps, 3), "steps": args.e2e_steps, "segments_in_flight_per_gpu": k,
            "h2d_bytes_per_segment": int(h2d_bytes), "ms_one_segment_unpipelined": round(1000.0 * t_one, 1),
            "note": f"witness in pinned host memory; native pipeline (r0hip_prove_segments): an uploader fills "
                    f"{k + 1} device buffer sets ahead of {k} prover threads, so H2D overlaps proving; a prover "
                    f"starts a segment while its later witness groups still upload (per-group gate)",
            **({"with_device_accumulation": dev_acc} if dev_acc else {})}


def pmc_traffic(family, calls, args):
    """HBM bytes per launch of `family` from the newest committed rocprofv3 PMC summary
    (profiles/r*_pmc_traffic.json, FETCH_SIZE/WRITE_SIZE passes of this same bench
    command, gfx950-corrected by tools/pmc_traffic.py). PMC counters cannot be read from
    inside the timed process, so the value is the committed measurement, labelled."""
    if args.circuit != "rv32im" or args.po2 != 20 or args.hashfn != "poseidon2":
        return None, None
    path = pmc_summary_file("traffic")
    if path is None:
        return None, None
    with open(path) as f:
        d = json.load(f)["per_proof"].get(family)
    if not d:
        return None, None
    return int((d["read_bytes"] + d["write_bytes"]) / calls), os.path.relpath(path, ROOT)


# how oracle/Makefile builds the CPU baseline's code: the reference's own C++ (poly_fp, the
# rv32im and recursion witness generation and accumulation) at the level its cargo build gives
# it, the oracle's restated CpuHal/Prover at -O3; both for the build host's x86-64 baseline ISA
REF_BUILD = ("oracle/_ref: g++ -O3 -ffunction-sections -fdata-sections -fno-var-tracking -g0 -std=c++17 (cc::Build "
             "under cargo's release profile: risc0/build_kernel/src/lib.rs:141-151, Cargo.toml:86-87); "
             "liboracle.so: g++ -O3 -std=c++17; every core the process may use (`cores`)")


def host_cores():
    """CPUs this process may use on the box: the affinity mask, capped by the cgroup CPU
    quota (cgroup v2 cpu.max or v1 cfs_quota/period) when one is set."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota:
        n = min(n, max(1, int(quota)))
    return n


def cpu_baseline_trace(args, trace, gpu_seal, gpu_mix):
    """The reference's prove_core from the same preflight trace on the host CPU: the compiled
    reference witness generation (risc0_circuit_rv32im_cpu_witgen, parallel mode) and
    accumulation (risc0_circuit_rv32im_cpu_accum) from oracle/_ref around the CPU oracle
    prover (C++ restatement of CpuHal + Prover, eval_check through the reference's compiled
    poly_fp), on every host core the process may use. Its seal and mix are compared with the
    last timed GPU seal and mix of that trace (`seal_equal`), as the reference prover verifies
    its own receipt before returning it (zkvm/src/host/server/prove/prover_impl.rs:277-280);
    main() exits nonzero on a mismatch."""
    try:
        cores = host_cores()
        os.environ["ORACLE_THREADS"] = str(cores)  # read once, at the oracle's first parallel op
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle
        import rv32im_accum_ref as RA
        import rv32im_witgen_ref as W
        if oracle.ref_lib() is None or not RA.available():
            return None
        compare = trace.po2 <= 20
        if not compare:  # a po2 > 20 segment would take the CPU path most of an hour: time the po2=20 guest
            import rv32im_trace as T
            trace = T.loop_s_trace(20, seed=0x5249534330) if args.guest == "loop_s" else \
                T.loop_trace(20, body_len=32, seed=0x5249534330)
        import hashlib
        suite = {"poseidon2": oracle.POSEIDON2, "sha-256": oracle.SHA256, "poseidon_254": oracle.POSEIDON254}[args.hashfn]
        rows = 1 << trace.po2
        data, glob, cyc, tx = W.inputs(trace)  # PreflightResults::new's injector and globals (not timed)
        oracle.op_times(reset=True)
        t0 = time.perf_counter()
        d, g = W.run(data, glob, cyc, tx, trace.table_split_cycle, rows, W.MODE_PARALLEL, trace.bigint_array())
        t_wg = time.perf_counter() - t0
        d = np.where(d == W.INVALID, 0, d).astype(np.uint32)
        g = np.where(g == W.INVALID, 0, g).astype(np.uint32)
        acc_s = []
        records = trace.bigint_records()

        def fill(mix):
            ta = time.perf_counter()
            init = None
            if records:  # WitnessGenerator::accum's BigIntAccum injection (witgen/mod.rs:187-205)
                import bigint_accum as BA
                init = BA.inject(np.full(RA.ACCUM_COLS * rows, W.INVALID, np.uint32), rows, mix, records)
            a = RA.accum(d, g, mix, rows, rows, accum_init=init)
            a = np.where(a == W.INVALID, 0, a).astype(np.uint32)
            acc_s.append(time.perf_counter() - ta)
            return a
        cseal, cmix, _, _ = oracle.prove_segment_cb("rv32im", suite, trace.po2, np.zeros(rows, np.uint32), d, g, fill,
                                                    RA.ACCUM_COLS * rows, version=2)
        t = time.perf_counter() - t0
        ops = {"witgen (reference risc0_circuit_rv32im_cpu_witgen)": round(t_wg, 3),
               "accumulate (reference risc0_circuit_rv32im_cpu_accum)": round(sum(acc_s), 3)}
        ops.update({k: round(v[0], 3) for k, v in sorted(oracle.op_times().items(), key=lambda kv: -kv[1][0])})
        ops["other (zeroize, transcript, openings, host polys)"] = round(t - sum(ops.values()), 3)
        dig = lambda a: hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint32).tobytes()).hexdigest()
        return {"value": round(rows / t, 1), "unit": "cycles/s", "cores": int(oracle.num_threads()), "kind": "port",
                "sample": f"one rv32im segment at po2={trace.po2} ({args.hashfn}) from the bench's own preflight trace, "
                          f"{t:.1f} s wall: the reference's compiled witgen and accumulation (oracle/_ref) and the "
                          "oracle prover with the reference's compiled poly_fp",
                "seconds_by_hal_op": ops, "build": REF_BUILD,
                "seal_equal": bool(np.array_equal(cseal, gpu_seal)) if compare else None,
                "mix_equal": bool(np.array_equal(cmix, gpu_mix)) if compare else None,
                "oracle_seal_sha256": dig(cseal), "gpu_seal_sha256": dig(gpu_seal),
                "oracle_mix_sha256": dig(cmix), "gpu_mix_sha256": dig(gpu_mix),
                "parity_note": ("CPU prove_core of rank 0's trace 0 against the GPU seal the timed pipeline proved from "
                                "that trace" if compare else "po2=20 sample; no parity at the bench's size")}
    except Exception as e:  # the baseline is reported, never required
        print(f"cpu baseline failed: {e}", file=sys.stderr)
        return None


def cpu_baseline_program(args, p, gpu_seal, gpu_mix):
    """The reference's recursion prove path on the host for rank 0's program 0: the compiled
    reference witness generation (risc0_circuit_recursion_cpu_witgen) and accumulation
    (risc0_circuit_recursion_cpu_accum) from oracle/_ref, the ZK noise words
    r0hip_prove_recursion draws (oracle.splitmix_fill of the same seeds), and the CPU oracle
    prover, on every host core the process may use; seal and mix compared with the GPU's."""
    try:
        cores = host_cores()
        os.environ["ORACLE_THREADS"] = str(cores)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle
        import accum_ir as A
        import recursion_program as RP
        if oracle.ref_lib() is None or not RP.available():
            return None
        import hashlib
        suite = {"poseidon2": oracle.POSEIDON2, "sha-256": oracle.SHA256, "poseidon_254": oracle.POSEIDON254}[args.hashfn]
        po2, n, zk = args.po2, 1 << args.po2, RP.ZK_CYCLES
        oracle.op_times(reset=True)
        t0 = time.perf_counter()
        ctrl, data, glob = RP.witgen(p["prog"], p["pf"], po2, raw=True)
        t_wg = time.perf_counter() - t0
        data = data.reshape(RP.DATA, n)
        data[:, n - zk:] = oracle.splitmix_fill(p["seed"], RP.DATA * zk).reshape(RP.DATA, zk)
        data = np.where(data == RP.INVALID, 0, data).astype(np.uint32).reshape(-1)
        glob = np.where(glob == RP.INVALID, 0, glob).astype(np.uint32)
        acc0 = np.full((RP.ACCUM, n), RP.INVALID, np.uint32)
        acc0[:, n - zk:] = oracle.splitmix_fill(p["seed"] + 1, RP.ACCUM * zk).reshape(RP.ACCUM, zk)
        acc0 = acc0.reshape(-1)
        acc_s = []

        def fill(mix):
            ta = time.perf_counter()
            acc = acc0.copy()
            A.ref_accum(ctrl, glob, data, mix, acc, len(p["prog"].rows), n)
            acc[acc == RP.INVALID] = 0
            acc_s.append(time.perf_counter() - ta)
            return acc
        cseal, cmix, _, _ = oracle.prove_segment_cb("recursion", suite, po2, ctrl, data, glob, fill, RP.ACCUM * n)
        t = time.perf_counter() - t0
        ops = {"witgen (reference risc0_circuit_recursion_cpu_witgen)": round(t_wg, 3),
               "accumulate (reference risc0_circuit_recursion_cpu_accum)": round(sum(acc_s), 3)}
        ops.update({k: round(v[0], 3) for k, v in sorted(oracle.op_times().items(), key=lambda kv: -kv[1][0])})
        ops["other (noise, zeroize, transcript, openings)"] = round(t - sum(ops.values()), 3)
        dig = lambda a: hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint32).tobytes()).hexdigest()
        return {"value": round(n / t, 1), "unit": "cycles/s", "cores": int(oracle.num_threads()), "kind": "port",
                "sample": f"one recursion segment at po2={po2} ({args.hashfn}) from rank 0's program 0, {t:.1f} s wall: "
                          "the reference's compiled recursion witgen and accumulation (oracle/_ref) and the oracle prover",
                "seconds_by_hal_op": ops, "build": REF_BUILD,
                "seal_equal": bool(np.array_equal(cseal, gpu_seal)), "mix_equal": bool(np.array_equal(cmix, gpu_mix)),
                "oracle_seal_sha256": dig(cseal), "gpu_seal_sha256": dig(gpu_seal),
                "parity_note": "CPU recursion prove of rank 0's program 0 against the GPU seal of the same program"}
    except Exception as e:  # the baseline is reported, never required
        print(f"cpu baseline failed: {e}", file=sys.stderr)
        return None


def cpu_baseline(args, circ, gpu_seal=None, gpu_mix=None):
    """The CPU oracle (C++ restatement of CpuHal + Prover, eval_check through the
    reference's compiled poly_fp) proving one segment of the bench's own config, with the
    per-Hal-op breakdown, on every host core the process may use.

    Its witness is rank 0's (same seed, same draw), so when the sizes agree the oracle
    seal and mix are compared with the last timed GPU seal and mix: every bench line then
    carries full-size oracle parity (`seal_equal`, both SHA-256 digests), as the reference
    prover verifies its own receipt before returning it
    (zkvm/src/host/server/prove/prover_impl.rs:277-280). main() exits nonzero on a
    mismatch."""
    try:
        cores = host_cores()
        os.environ["ORACLE_THREADS"] = str(cores)  # read once, at the oracle's first parallel op
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        if oracle.ref_lib() is None:
            return None
        po2 = args.cpu_po2 if args.cpu_po2 is not None else min(args.po2, 20)  # po2=24 would take ~30 min
        rng = np.random.default_rng(0x5249534330)
        code, data, accum, glob = synthetic_witness(rng, circ, po2)
        suite = {"poseidon2": oracle.POSEIDON2, "sha-256": oracle.SHA256, "poseidon_254": oracle.POSEIDON254}[args.hashfn]
        oracle.op_times(reset=True)
        t0 = time.perf_counter()
        cseal, cmix, _ = oracle.prove_segment(args.circuit, suite, po2, code, data, accum, glob,
                                              version=2 if args.circuit == "rv32im" else None)
        t = time.perf_counter() - t0
        ops = {k: round(v[0], 3) for k, v in sorted(oracle.op_times().items(), key=lambda kv: -kv[1][0])}
        ops["other (transcript, openings, host polys)"] = round(t - sum(ops.values()), 3)
        import hashlib
        dig = lambda a: hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint32).tobytes()).hexdigest()
        parity = {"seal_equal": None, "oracle_seal_sha256": dig(cseal), "oracle_mix_sha256": dig(cmix)}
        if gpu_seal is not None and po2 == args.po2 and args.po2 <= 22:
            parity.update({"seal_equal": bool(np.array_equal(cseal, gpu_seal)),
                           "mix_equal": bool(np.array_equal(cmix, gpu_mix)),
                           "gpu_seal_sha256": dig(gpu_seal), "gpu_mix_sha256": dig(gpu_mix),
                           "parity_note": "oracle prover on rank 0's own witness (same seed and draw) against "
                                          "the last timed GPU seal of that witness"})
        return {"value": round((1 << po2) / t, 1), "unit": "cycles/s", "cores": int(oracle.num_threads()),
                "kind": "port",
                "sample": f"one {args.circuit} segment at po2={po2} ({args.hashfn}), {t:.1f} s wall; "
                          "eval_check uses the reference's compiled C++ poly_fp",
                "seconds_by_hal_op": ops, **parity}
    except Exception as e:  # the baseline is reported, never required
        print(f"cpu baseline failed: {e}", file=sys.stderr)
        return None


if __name__ == "__main__":
    main()
