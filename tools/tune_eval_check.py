#!/usr/bin/env python3
"""Per-kernel autotuning of the generated eval_check kernels (register target and load
prefetch distance), measured on an MI355X.

  python tools/tune_eval_check.py build [CIRCUIT]     # variants -> risc0_amd/lib_variants/
  gpurun -- 'python tools/tune_eval_check.py measure'  # rocprofv3 per-kernel times
  python tools/tune_eval_check.py pick [CIRCUIT]      # -> risc0_amd/circuits/<c>.ectune.json

Each measure run also times `libr0hip_tune_ref.so` (copy the in-tree build there first):
`pick` compares every variant with the reference of its own run.

The kernel partition depends only on the cost budget, so kernel k of every variant
computes the same terms; `pick` keeps, per kernel, the variant with the lowest mean
duration and the generator then emits each kernel with its own settings.
"""
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "risc0_amd", "csrc")
VAR = os.path.join(ROOT, "risc0_amd", "lib_variants")
OUT = os.path.join(ROOT, "gpurun_out", "tune")
CIRCUIT = "rv32im"
GRID = [(w, pf) for w in (1, 2) for pf in (128, 256, 512, 768, 1024)]
BUDGET = 4000
MARGIN = float(os.environ.get("TUNE_MARGIN", "0.05"))


def build(circuit):
    os.makedirs(VAR, exist_ok=True)
    for f in glob.glob(os.path.join(VAR, "libr0hip_tune_*.so")):
        os.remove(f)
    for w, pf in GRID:
        shutil.rmtree(os.path.join(CSRC, "gen", circuit), ignore_errors=True)
        # the committed per-kernel choices other than these two (canon, pinb) stay
        env = dict(os.environ, EC_WAVES=str(w), EC_PF=str(pf), EC_KEEPTUNE="1")
        subprocess.run(["make", "-j8", f"EC_BUDGET_{circuit}={BUDGET}"], cwd=CSRC, env=env, check=True,
                       stdout=subprocess.DEVNULL)
        shutil.copy(os.path.join(ROOT, "risc0_amd", "lib", "libr0hip.so"),
                    os.path.join(VAR, f"libr0hip_tune_w{w}_pf{pf}.so"))
        print("built", w, pf, flush=True)
    shutil.rmtree(os.path.join(CSRC, "gen", circuit), ignore_errors=True)
    subprocess.run(["make", "-j8"], cwd=CSRC, check=True, stdout=subprocess.DEVNULL)


def measure():
    os.makedirs(OUT, exist_ok=True)
    for lib in sorted(glob.glob(os.path.join(VAR, "libr0hip_tune_*.so"))):
        tag = os.path.basename(lib)[len("libr0hip_tune_"):-3]
        env = dict(os.environ, R0HIP_LIB=lib, TMPDIR="/tmp", R0_EC_CIRCUIT=CIRCUIT)
        subprocess.run(["timeout", "-k", "10", "200", "rocprofv3", "--kernel-trace", "--stats", "-d",
                        os.path.join(OUT, tag), "-o", "run", "--output-format", "csv", "--", sys.executable,
                        os.path.join(ROOT, "tools", "bench_kernels.py"), "ec"], env=env, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        print("measured", tag, flush=True)


def kernel_times(d, circuit):
    out = {}
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
        km = re.search(r"ec_" + circuit + r"::k(\d+)<(?:false|true)>", r["Name"])
        if km:
            out[int(km.group(1))] = float(r["AverageNs"]) / 1e3
    return out


def pick(circuit):
    """Per kernel, the variant with the lowest time relative to the reference library
    measured in the same run (`ref`: the build with the committed tuning), so runs on
    different boxes (clocks differ by a few percent) compare fairly; a kernel keeps its
    committed settings unless some variant beats them. Run directories: gpurun_out/tune*
    with one subdirectory per variant (w<W>_pf<PF>) and `ref`."""
    path = os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".ectune.json")
    prev = json.load(open(path))
    best = {}  # kernel -> (ratio, waves, pf, time in its run)
    ref_us = {}
    for run in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "tune*"))):
        if not os.path.isdir(os.path.join(run, "ref")):
            print(f"skipped {run}: no ref measurement")
            continue
        ref = kernel_times(os.path.join(run, "ref"), circuit)
        for k, t in ref.items():
            ref_us.setdefault(k, []).append(t)
        for d in sorted(glob.glob(os.path.join(run, "w*_pf*"))):
            m = re.match(r"w(\d+)_pf(\d+)", os.path.basename(d))
            w, pf = int(m.group(1)), int(m.group(2))
            for k, t in kernel_times(d, circuit).items():
                r = t / ref[k]
                if r < best.get(k, (1.0,))[0]:
                    best[k] = (r, w, pf, t)
    # a variant identical to the committed setting measures within ±3-7% of the reference
    # per kernel (median ratio 1.00 in both r3g runs): adopt only clear wins
    best = {k: v for k, v in best.items() if v[0] < 1.0 - MARGIN}
    kern = {k: dict(v) for k, v in prev["kernels"].items()}
    tot_ref = tot = 0.0
    for k in sorted(int(x) for x in kern):
        base = sum(ref_us.get(k, [0])) / max(1, len(ref_us.get(k, [])))
        tot_ref += base
        if k in best:
            r, w, pf, _ = best[k]
            kern[str(k)].update(waves=w, pf=pf, us=round(base * r, 1))
            tot += base * r
            print(f"k{k:<3d} w{w} pf{pf}: {r:.3f} of the committed setting")
        else:
            tot += base
    out = dict(prev, kernels=kern, measured_total_us=round(tot, 1))
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {path}: sum of kernel means {tot_ref / 1e3:.2f} ms -> {tot / 1e3:.2f} ms (reference-relative)")


if __name__ == "__main__":
    cmd = sys.argv[1]
    c = CIRCUIT = sys.argv[2] if len(sys.argv) > 2 else "rv32im"
    {"build": lambda: build(c), "measure": measure, "pick": lambda: pick(c)}[cmd]()
