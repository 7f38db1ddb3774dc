#!/usr/bin/env python3
"""Choose the eval_check sub-expressions to materialise across kernels.

The constraint program is split into kernels under a cost budget, and a sub-expression
used by terms in several kernels is recomputed in each (rv32im at budget 4000: 1.19x the
program's work). Greedy: schedule, find the node whose cone cost x (kernels using it - 1)
is largest, materialise it (computed once, stored per point: 4 B Fp / 16 B FpExt, read by
later kernels), reschedule; N steps.

  python tools/pick_ec_mat.py CIRCUIT N     # writes "mat" into <circuit>.ectune.json and
                                            # clears its per-kernel tuning (partition changed)
"""
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_eval_check as G  # noqa: E402

BUDGET = 4000


def kernel_roots(k):
    return [r for it in k for r in ([it[3]] if it[2] == "mat" else G.term_roots(it[3]))]


def main(circuit, n):
    pg = G.Program(circuit)
    prog = pg.cone_cost([pg.res])
    chosen = []
    for step in range(n + 1):
        pg.mat = set(chosen)
        _terms, kernels = G.schedule(pg, BUDGET)
        work = sum(pg.cone_cost(kernel_roots(k)) for k in kernels)
        print(f"{len(chosen):3d} materialised: {len(kernels)} kernels, work {work} ({work / prog:.3f}x)", flush=True)
        if step == n:
            break
        cnt = collections.Counter(v for k in kernels for v in pg.cone(kernel_roots(k)) if v not in pg.mat)
        best = None
        for v, c in cnt.items():
            if c < 2 or pg.byid[v][0] in "clge":
                continue
            gain = pg.cone_cost([v]) * (c - 1)
            if best is None or gain > best[0]:
                best = (gain, v)
        if best is None:
            break
        chosen.append(best[1])
    path = os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".ectune.json")
    t = json.load(open(path)) if os.path.exists(path) else {"budget": BUDGET, "order": "dfs"}
    t["mat"] = chosen
    t["kernels"] = {}
    t["measured_total_us"] = None
    with open(path, "w") as f:
        json.dump(t, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
