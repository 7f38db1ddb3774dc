#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel name:
duration, VALU issue utilisation (ACTIVE_INST_VALU quad-cycles / (SIMDs x kernel quad-cycles)),
wave-parked fraction and instructions per wave."""
import collections
import csv
import re
import sys

SIMDS = 256 * 4
XCDS = 8


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    return n.replace("r0::", "")[:60]


def main(path, json_out=None):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Dispatch_Id"] not in disp[k]:
            disp[k].add(r["Dispatch_Id"])
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    rows = []
    for k, d in agg.items():
        gui = d.get("GRBM_GUI_ACTIVE", 0) / XCDS  # summed over the 8 XCDs
        ms = dur[k]
        clk = gui / (ms * 1e-3) / 1e9 if ms else 0
        valu = d.get("SQ_ACTIVE_INST_VALU", 0)
        util = valu * 4 / (SIMDS * gui) if gui else 0
        wc = d.get("SQ_WAVE_CYCLES", 0)
        park = d.get("SQ_WAIT_ANY", 0) / wc if wc else 0
        rows.append((ms, k, len(disp[k]), clk, util, park, d.get("SQ_INSTS_VALU", 0) / max(d.get("SQ_WAVES", 1), 1)))
    rows.sort(reverse=True)
    if json_out:
        # per-kernel totals over the run, for bench.py's instruction roof (SQ_INSTS_VALU per
        # launch) and issue-busy share
        import json
        out = {}
        for k, d in agg.items():
            gui = d.get("GRBM_GUI_ACTIVE", 0) / XCDS
            out[k] = {"ms": dur[k], "dispatches": len(disp[k]), "insts_valu": d.get("SQ_INSTS_VALU", 0),
                      "active_inst_valu": d.get("SQ_ACTIVE_INST_VALU", 0), "waves": d.get("SQ_WAVES", 0),
                      "gui_active_cycles": gui}
        with open(json_out, "w") as f:
            json.dump({"source": path, "kernels": out}, f, indent=1, sort_keys=True)
    print(f"{'kernel':60s} {'ms':>8s} {'n':>4s} {'GHz':>5s} {'valu%':>6s} {'park%':>6s} {'valu/wave':>10s}")
    for ms, k, n, clk, util, park, ipw in rows:
        print(f"{k:60s} {ms:8.3f} {n:4d} {clk:5.2f} {100 * util:6.1f} {100 * park:6.1f} {ipw:10.0f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
