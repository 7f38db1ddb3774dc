#!/usr/bin/env python3
"""The bench's pipelined unit alone, for a rocprofv3 --kernel-trace run: 4 distinct rv32im
po2=20 loop-guest traces in page-locked memory, a warm-up batch, an idle gap, then one batch of
N trace jobs at `in_flight` segments (tools/pipeline_occupancy.py reads the last batch).

  python tools/micro/pipeline_trace.py [N=24] [in_flight=3]
"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import risc0_amd as r  # noqa: E402
import rv32im_trace as T  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    po2 = 20
    hal = r.HipHal("poseidon2")
    jobs = []
    for i in range(4):
        t = T.loop_s_trace(po2, iterations=T.ITERATIONS_FULL_PO2_20_SEGMENT - 37 * i, seed=1 + i)
        cyc, tx = t.arrays()
        idx, off, val = t.injector_arrays()
        jobs.append(r.TraceJob(*(r.pinned_copy(a) for a in (t.global_words(), idx, off, val, cyc, tx)),
                               t.table_split_cycle))
    batch = [jobs[i % 4] for i in range(n)]
    r.prove_trace_segments(hal, po2, batch[:2 * k], in_flight=k)  # warm pools, sets and tables
    time.sleep(0.5)  # an idle gap that marks the measured batch in the kernel trace
    t0 = time.perf_counter()
    r.prove_trace_segments(hal, po2, batch, in_flight=k)
    dt = time.perf_counter() - t0
    print(f"{n} trace jobs at {k} in flight: {1000 * dt / n:.2f} ms per segment")


if __name__ == "__main__":
    main()
