#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel + memory-copy trace of the last N seconds of a run:
H2D copy spans and the kernel busy time, to see what one segment's latency is made of.
  python tools/timeline.py DIR [WINDOW_MS]"""
import csv
import glob
import sys


def main(d, window_ms=400.0):
    ks = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]))
    cs = []
    for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            cs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", ""), int(r.get("Bytes", 0) or 0)))
    end = max(e for _, e, _ in ks)
    t0 = end - window_ms * 1e6
    ks = sorted(k for k in ks if k[0] >= t0)
    cs = sorted(c for c in cs if c[0] >= t0)
    # split into segments by gaps > 5 ms without kernels
    segs, cur = [], [ks[0]]
    for k in ks[1:]:
        if k[0] - max(x[1] for x in cur) > 5e6:
            segs.append(cur)
            cur = []
        cur.append(k)
    segs.append(cur)
    for s in segs:
        a, b = s[0][0], max(x[1] for x in s)
        busy, last = 0, a
        for k0, k1, _ in s:
            busy += max(0, k1 - max(k0, last))
            last = max(last, k1)
        cpy = [c for c in cs if a - 60e6 <= c[0] <= b]
        h2d = [c for c in cpy if c[3] > 1 << 20]
        print(f"kernels {len(s)}: span {(b - a) / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms")
        if h2d:
            print(f"  large copies {len(h2d)}: first start {(h2d[0][0] - a) / 1e6:+.1f} ms, last end "
                  f"{(max(c[1] for c in h2d) - a) / 1e6:+.1f} ms, {sum(c[3] for c in h2d) / 1e9:.2f} GB")
            for c in h2d:
                print(f"    {(c[0] - a) / 1e6:+8.2f} .. {(c[1] - a) / 1e6:+8.2f} ms {c[3] / 1e6:8.1f} MB "
                      f"{c[3] / max(1, c[1] - c[0]):.1f} GB/s {c[2]}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 400.0)
