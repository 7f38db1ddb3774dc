#!/usr/bin/env python3
"""How busy the GPU is while the segment pipeline runs, from a rocprofv3 --kernel-trace of
tools/micro/pipeline_trace.py: the measured batch is the kernels after the trace's longest
idle gap. Reports the share of the batch's wall time with no kernel running, with only
latency-bound kernels (Merkle tree tops and narrow layers, small NTT passes, witgen/copy
helpers) running, and with at least one VALU-heavy kernel running; and per family the summed
kernel time against its union (overlap).

  python tools/pipeline_occupancy.py gpurun_out/TAG/trace
"""
import csv
import glob
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from rocprof_families import family  # noqa: E402

HEAVY = ("eval_check", "hash_rows", "ntt_evaluate", "ntt_interpolate")


def heavy(name):
    f = family(name)
    if f in HEAVY:
        return True
    return "p2_fold_kernel" in name  # the wide Merkle layers; quads and tops are latency-bound


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(d):
    kf = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(kf)))
    # the measured batch: after the longest gap between the end of everything so far and the next start
    best, cut, end = 0, 0, ks[0][1]
    for i in range(1, len(ks)):
        if ks[i][0] - end > best:
            best, cut = ks[i][0] - end, i
        end = max(end, ks[i][1])
    batch = ks[cut:]
    t0, t1 = batch[0][0], max(k[1] for k in batch)
    wall = t1 - t0
    busy = union([(s, e) for s, e, _ in batch])
    hv = union([(s, e) for s, e, n in batch if heavy(n)])
    print(f"batch: {len(batch)} kernels over {wall / 1e6:.2f} ms (idle gap before it {best / 1e6:.1f} ms)")
    print(f"  no kernel running          {100 * (wall - busy) / wall:5.1f} %")
    print(f"  only latency-bound kernels {100 * (busy - hv) / wall:5.1f} %")
    print(f"  a VALU-heavy kernel        {100 * hv / wall:5.1f} %")
    fams = {}
    for s, e, n in batch:
        fams.setdefault(family(n), []).append((s, e))
    print("family                     sum ms   union ms")
    for f, iv in sorted(fams.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        print(f"{f[:24]:24s} {sum(e - s for s, e in iv) / 1e6:8.2f} {union(iv) / 1e6:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
