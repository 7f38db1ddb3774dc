#!/usr/bin/env python3
"""Model of the column-packed term split for eval_check.

The generator (tools/gen_eval_check.py: schedule) splits poly_fp's accumulation chains
into terms until each term's dependency cone fits the kernel budget, then packs terms
into kernels in program order. Each kernel reloads every trace column its terms tap, so
the tap traffic is the sum over kernels of the distinct (argument, column) pairs read.

This tool re-splits terms more finely and re-packs them by column affinity (greedy:
seed with the largest remaining item, then add the item whose marginal cost plus
W x new columns, relative to its own size, is smallest, while the kernel's cone stays
under the budget). It prices each plan in:
  cols — distinct column reads summed over kernels (each = 4 B x domain of HBM reads);
  cost — the generator's op cost of every kernel's cone (shared nodes once per kernel)
         plus each term's own factor products (poly_mix power, distributed factors).

Two scopes: "all" re-plans every term; "stalled" re-plans only the terms of the kernels
below 85% VALU issue in the latest PMC run, leaving the others as they are.
Finer splitting only stays cheap through plain accumulations (ACC + T*pm); splitting
through ACC + T*U*pm distributes U over every sub-term, so those are split only as far
as the budget forces (as the generator does).

  model_ec_colpack.py [--stalled K,K,...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_eval_check as G  # noqa: E402

BUD = 4000


class Model:
    def __init__(self):
        self.pg = G.Program("rv32im")
        self.pg.mat = set(G.mat_config("rv32im", BUD))
        self.terms, self.kernels = G.schedule(self.pg, BUD)
        self.C = {v: self.pg.cost(v) for v in self.pg.byid if self.pg.byid[v][0] != "r"}

    def info(self, kind, x):
        pg, byid, ty = self.pg, self.pg.byid, self.pg.types
        roots = [x] if kind == "mat" else G.term_roots(x)
        rs = set(roots)
        full = pg.cone(roots)
        cone = set(v for v in full if not (v in pg.mat and v not in rs))
        cols = set((byid[v][2], byid[v][3]) for v in cone if byid[v][0] == "l")
        extra = 0
        if kind == "term":
            e = ty[x[0]] == "e"
            for f in x[1]:
                if f[0] == "v":
                    ue = ty[f[1]] == "e"
                    extra += 16 if (e and ue) else (4 if (e or ue) else 1)
                    e = e or ue
                else:
                    extra += 20 if e else 8
        return dict(cone=cone, cols=cols, extra=extra, cost=sum(self.C[v] for v in cone) + extra,
                    needs=set(v for v in full if v in pg.mat and v not in rs), kind=kind, x=x)

    def stats(self, items):
        cone, cols, ex = set(), set(), 0
        for m in items:
            cone |= m["cone"]
            cols |= m["cols"]
            ex += m["extra"]
        return len(cols), sum(self.C[v] for v in cone) + ex

    def split_plain(self, t, sb):
        """split a term through plain accumulations until its cone cost is <= sb"""
        out, res = [t], []
        while out:
            t = out.pop()
            ins = self.pg.byid[t[0]]
            m = self.info("term", t)
            if ins[0] == "a" and m["cost"] > sb:
                out += [(ins[2], t[1]), (ins[3], t[1] + [("pm", ins[4])])]
            else:
                res.append(m)
        return res

    def pack(self, pool, W):
        """greedy column-affinity packing under the budget, honouring materialisation order"""
        C = self.C
        done = set(m["x"] for m in pool if False)
        produced_here = set(m["x"] for m in pool if m["kind"] == "mat")
        left, out = set(range(len(pool))), []
        while left:
            ready = [i for i in left if (pool[i]["needs"] & produced_here) <= done]
            seed = max(ready, key=lambda i: (pool[i]["kind"] == "mat", pool[i]["cost"] + W * len(pool[i]["cols"])))
            K, kcone, kc, cost = [seed], set(pool[seed]["cone"]), set(pool[seed]["cols"]), pool[seed]["cost"]
            cand = set(ready) - {seed}
            while True:
                best, bs = None, 1e18
                for i in cand:
                    m = pool[i]
                    dc = sum(C[v] for v in m["cone"] - kcone) + m["extra"]
                    if cost + dc > BUD:
                        continue
                    dn = len(m["cols"] - kc)
                    sc = (dc + W * dn) / (m["cost"] + W * len(m["cols"]) + 1)
                    if sc < bs:
                        best, bs, bdc = i, sc, dc
                if best is None:
                    break
                K.append(best)
                kcone |= pool[best]["cone"]
                kc |= pool[best]["cols"]
                cost += bdc
                cand.discard(best)
            left -= set(K)
            done |= set(pool[i]["x"] for i in K if pool[i]["kind"] == "mat")
            out.append((len(kc), cost))
        return out


def main():
    stalled = None
    if len(sys.argv) > 2 and sys.argv[1] == "--stalled":
        stalled = [int(x) for x in sys.argv[2].split(",")]
    M = Model()
    scope = stalled if stalled is not None else list(range(len(M.kernels)))
    base = [M.stats([M.info(it[2], it[3]) for it in M.kernels[i]]) for i in scope]
    print(f"scope: {'kernels ' + ','.join(map(str, scope)) if stalled else 'all kernels'}")
    print(f"committed plan: kernels {len(scope)} cols {sum(b[0] for b in base)} cost {sum(b[1] for b in base)}")
    for sb in (4000, 2000, 1000, 500, 250):
        pool = []
        for i in scope:
            for it in M.kernels[i]:
                pool += [M.info("mat", it[3])] if it[2] == "mat" else M.split_plain(it[3], sb)
        for W in (4, 16, 64):
            out = M.pack(pool, W)
            c, k = sum(o[0] for o in out), sum(o[1] for o in out)
            b0, b1 = sum(b[0] for b in base), sum(b[1] for b in base)
            print(f"split <= {sb:4d}  W {W:2d}: items {len(pool):4d} kernels {len(out):2d} cols {c:5d} "
                  f"({100 * (c / b0 - 1):+.1f}%) cost {k:6d} ({100 * (k / b1 - 1):+.1f}%)", flush=True)


if __name__ == "__main__":
    main()
