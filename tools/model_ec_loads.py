#!/usr/bin/env python3
"""Load density of each rv32im eval_check kernel (tap loads + materialised reads per unit of
the generator's VALU cost model) against its measured VALU issue share
(profiles/archive/r3t_pmc_valu.txt): does the load density predict which kernels stall?
(a load-aware split.)

  model_ec_loads.py [BUDGET] > profiles/r4_ec_load_density.txt
"""
import os
import re
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_eval_check as G  # noqa: E402


def main():
    budget = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    pg = G.Program("rv32im")
    pg.mat = set(G.mat_config("rv32im", budget))
    _, kernels = G.schedule(pg, budget)
    valu = {}
    for line in open(os.path.join(ROOT, "profiles", "archive", "r3t_pmc_valu.txt")):
        m = re.match(r"ec_rv32im::k(\d+)<false>\s+([\d.]+)\s+(\d+)\s+([\d.]+)\s+([\d.]+)", line)
        if m:
            valu[int(m.group(1))] = (float(m.group(2)) / int(m.group(3)), float(m.group(5)))
    rows = []
    print("kernel  items  cost  taps  mat_reads  density(%)  ms/proof  valu%")
    for ki, k in enumerate(kernels):
        roots = []
        for it in k:
            roots += [it[3]] if it[2] == "mat" else G.term_roots(it[3])
        cone, rs = pg.cone(roots), set(roots)
        taps = sum(1 for v in cone if pg.byid[v][0] == "l")
        matr = sum(1 for v in cone if v in pg.mat and v not in rs)
        cost = pg.cone_cost(roots)
        dens = 100.0 * (taps + matr) / cost
        ms, vp = valu.get(ki, (float("nan"), float("nan")))
        rows.append((dens, vp, ms))
        print(f"k{ki:<6} {len(k):5d} {cost:5d} {taps:5d} {matr:10d} {dens:11.1f} {ms:9.3f} {vp:6.1f}")
    d = np.array([r[0] for r in rows])
    v = np.array([r[1] for r in rows])
    ok = ~np.isnan(v)
    print(f"correlation(load density, VALU%) over {ok.sum()} kernels: {np.corrcoef(d[ok], v[ok])[0, 1]:+.2f}")
    stalled = [i for i, r in enumerate(rows) if r[1] < 85]
    print("stalled (<85% VALU):", " ".join(f"k{i}({rows[i][0]:.1f})" for i in stalled))
    print("densest:", " ".join(f"k{i}({rows[i][0]:.1f}, {rows[i][1]:.0f}%)" for i in sorted(range(len(rows)),
                                                                                key=lambda i: -rows[i][0])[:5]))


if __name__ == "__main__":
    main()
