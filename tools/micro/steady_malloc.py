#!/usr/bin/env python3
"""Which device allocations a warm pool still makes: the scenario of
tests/test_gpu_parity.py::test_steady_state_proving_makes_no_hipmalloc (two fresh host
threads proving the first golden seal case at once, per batch), warmed until the first batch
that allocates nothing, then BATCHES more batches, each bracketed on stderr so that
R0HIP_TRACE_MALLOC=1 output shows the allocations of every batch that made any.

  R0HIP_TRACE_MALLOC=1 python3 tools/micro/steady_malloc.py [BATCHES]
"""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), ROOT, os.path.join(ROOT, "tests")]
import oracle as o  # noqa: E402  (the CPU checker, for the golden case's witness only)
import risc0_amd as r  # noqa: E402
import test_golden as G  # noqa: E402


def main():
    batches = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    o.build(ref=True)
    case = G.INDEX["seals"][0]
    h = r.HipHal(case["suite"])
    code, data, accum, glob = G.seal_inputs(o, case["circuit"], case["po2"])
    bufs = [h.copy_from_elem("x", x) for x in (code, data, accum)]
    globs = [h.copy_from_elem("x", glob) for _ in range(2)]
    version = 2 if case["circuit"] == "rv32im" else None
    r.trim()

    def batch():
        ts = [threading.Thread(target=lambda i=i: r.prove_segment(h, case["circuit"], case["po2"], *bufs, globs[i],
                                                                   version=version)) for i in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()

    for k in range(10):
        m0 = r.mem_stats()["mallocs"]
        batch()
        if k and r.mem_stats()["mallocs"] == m0:
            break
    print(f"warm after {k + 1} batches", flush=True)
    for b in range(batches):
        m0 = r.mem_stats()["mallocs"]
        os.write(2, f"batch {b} begins\n".encode())
        batch()
        os.write(2, f"batch {b} ends\n".encode())
        print(f"batch {b}: {r.mem_stats()['mallocs'] - m0} mallocs", flush=True)


if __name__ == "__main__":
    main()
