#!/usr/bin/env python3
"""One rv32im po2=20 loop-guest segment through the segment pipeline's trace jobs from
page-locked host memory, after warm-up calls: bench.py's ms_one_segment_unpipelined alone,
for a rocprofv3 --kernel-trace --memory-copy-trace timeline (tools/timeline.py)."""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import risc0_amd as r  # noqa: E402
import rv32im_trace as T  # noqa: E402


def main():
    po2 = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    hal = r.HipHal("poseidon2")
    t = T.loop_s_trace(po2, seed=3)
    cyc, tx = t.arrays()
    idx, off, val = t.injector_arrays()
    job = r.TraceJob(*(r.pinned_copy(a) for a in (t.global_words(), idx, off, val, cyc, tx)), t.table_split_cycle)
    r.prove_trace_segments(hal, po2, [job] * 3, in_flight=2)  # warm the pools, sets and tables
    for _ in range(3):
        time.sleep(0.2)  # an idle GPU before the measured segment
        t0 = time.perf_counter()
        r.prove_trace_segments(hal, po2, [job], in_flight=1)
        print(f"one trace job: {1000 * (time.perf_counter() - t0):.1f} ms ({job.h2d_bytes() / 1e6:.0f} MB uploaded)")


if __name__ == "__main__":
    main()
