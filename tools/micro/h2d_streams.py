#!/usr/bin/env python3
"""H2D bandwidth from page-locked host memory with 1, 2 and 4 concurrent streams (each copy
on its own stream and host thread, as the segment pipeline's uploader would split a trace):
whether one DMA queue saturates the link for a 167 MB preflight trace."""
import threading
import time

import torch

MB = 1 << 20


def run(total_mb, nstreams, reps=5):
    part = total_mb * MB // nstreams
    src = [torch.empty(part, dtype=torch.uint8).pin_memory() for _ in range(nstreams)]
    dst = [torch.empty(part, dtype=torch.uint8, device="cuda") for _ in range(nstreams)]
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    best = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()

        def go(i):
            with torch.cuda.stream(streams[i]):
                dst[i].copy_(src[i], non_blocking=True)
            streams[i].synchronize()
        ts = [threading.Thread(target=go, args=(i,)) for i in range(nstreams)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        dt = time.perf_counter() - t0
        best = max(best, total_mb * MB / dt / 1e9)
    return best


if __name__ == "__main__":
    for n in (1, 2, 4):
        print(f"167 MB in {n} stream(s): {run(167, n):.1f} GB/s (best of 5)")
    for n in (1, 2):
        print(f"1320 MB in {n} stream(s): {run(1320, n):.1f} GB/s (best of 5)")
