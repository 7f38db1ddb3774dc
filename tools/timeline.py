#!/usr/bin/env python3
"""What one segment's latency is made of, from a rocprofv3 --kernel-trace
--memory-copy-trace run of tools/micro/one_segment.py (tools/rehearsal/gpu_oneseg.sh):
the last segment's copies (start/end relative to its large data copy) and the GPU's
kernel-busy time in 8 ms windows.

  python tools/timeline.py gpurun_out/oneseg2/trace
"""
import csv
import glob
import sys


def main(d):
    kf = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    cf = glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)[0]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(kf)))
    cs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"].replace("MEMORY_COPY_", ""))
                for r in csv.DictReader(open(cf)))
    big = [c for c in cs if c[1] - c[0] > 1e6]
    # the last segment's copies: the last run of large copies with < 20 ms between them
    first = len(big) - 1
    while first > 0 and big[first][0] - big[first - 1][1] < 20e6:
        first -= 1
    base = big[first][0]
    for c in cs:
        if c[0] >= base - 1e6:
            print(f"copy {(c[0] - base) / 1e6:+8.2f} .. {(c[1] - base) / 1e6:+8.2f} ms  {c[2]}")
    mine = [k for k in ks if k[0] >= base - 2e6]
    print(f"kernels: first start {(mine[0][0] - base) / 1e6:+.2f} ms, last end {(max(k[1] for k in mine) - base) / 1e6:+.2f} ms")

    def busy(a, b):
        t, last = 0, a
        for k0, k1 in mine:
            s, e = max(k0, last, a), min(k1, b)
            if e > s:
                t += e - s
                last = e
        return t / 1e6

    end = (max(k[1] for k in mine) - base) / 1e6
    a = -2.0
    while a < end:
        print(f"{a:6.0f} .. {a + 8:4.0f} ms  busy {busy(base + a * 1e6, base + (a + 8) * 1e6):4.1f} ms")
        a += 8


if __name__ == "__main__":
    main(sys.argv[1])
