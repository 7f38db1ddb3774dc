#!/usr/bin/env python3
"""Per-kernel choice between canonical and range-analysis (lazy) arithmetic for the
generated eval_check kernels, on top of the committed (waves, prefetch) tuning.

  python tools/tune_ec_canon.py build [CIRCUIT]     # 3 variants -> risc0_amd/lib_variants/
  gpurun -- 'python tools/tune_ec_canon.py measure'  # rocprofv3 per-kernel times
  python tools/tune_ec_canon.py pick [CIRCUIT]      # adds "canon" (and "waves") to <c>.ectune.json

Variants: canonical with the tuned settings, lazy with the tuned settings, and lazy at one
wave per SIMD (twice the registers: the lazy form spills in some kernels at two). Kernel
k computes the same terms in every variant, and every value leaving a kernel is canonical,
so kernels can mix modes freely.
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
OUT = os.path.join(ROOT, "gpurun_out", "tune_canon")
CIRCUIT = "rv32im"
MARGIN = float(os.environ.get("TUNE_MARGIN", "0.05"))
VARIANTS = {"canon": {"EC_CANON_FORCE": "1"}, "lazy": {"EC_CANON_FORCE": "0"},
            "lazyw1": {"EC_CANON_FORCE": "0", "EC_WAVES_OVERRIDE": "1"}}


def build(circuit):
    os.makedirs(VAR, exist_ok=True)
    for f in glob.glob(os.path.join(VAR, "libr0hip_*.so")):
        os.remove(f)
    for name, env in VARIANTS.items():
        shutil.rmtree(os.path.join(CSRC, "gen", circuit), ignore_errors=True)
        subprocess.run(["make", "-j8"], cwd=CSRC, env=dict(os.environ, **env), check=True, stdout=subprocess.DEVNULL)
        shutil.copy(os.path.join(ROOT, "risc0_amd", "lib", "libr0hip.so"), os.path.join(VAR, f"libr0hip_{name}.so"))
        print("built", name, flush=True)
    shutil.rmtree(os.path.join(CSRC, "gen", circuit), ignore_errors=True)
    subprocess.run(["make", "-j8"], cwd=CSRC, check=True, stdout=subprocess.DEVNULL)


def measure():
    os.makedirs(OUT, exist_ok=True)
    # the committed build (copied to libr0hip_tuned.so) is measured in the same run when present
    names = list(VARIANTS) + (["tuned"] if os.path.exists(os.path.join(VAR, "libr0hip_tuned.so")) else [])
    for name in names:
        lib = os.path.join(VAR, f"libr0hip_{name}.so")
        env = dict(os.environ, R0HIP_LIB=lib, TMPDIR="/tmp", R0_EC_CIRCUIT=CIRCUIT)
        subprocess.run(["timeout", "-k", "10", "200", "rocprofv3", "--kernel-trace", "--stats", "-d",
                        os.path.join(OUT, name), "-o", "run", "--output-format", "csv", "--", sys.executable,
                        os.path.join(ROOT, "tools", "bench_kernels.py"), "ec"], env=env, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        print("measured", name, flush=True)


def pick(circuit):
    path = os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".ectune.json")
    tune = json.load(open(path))
    times = {}
    for name in VARIANTS:
        for r in csv.DictReader(open(os.path.join(OUT, name, "run_kernel_stats.csv"))):
            km = re.search(r"ec_" + circuit + r"::k(\d+)", r["Name"])
            if km:
                times.setdefault(km.group(1), {})[name] = float(r["AverageNs"]) / 1e3
    tot = {n: sum(t[n] for t in times.values()) for n in VARIANTS}
    best_tot = 0.0
    for k, t in times.items():
        kc = tune["kernels"].setdefault(k, {})
        # the committed mode stays unless another wins by more than MARGIN: one kernel of one
        # configuration measures within ±3-7% run to run (tools/tune_eval_check.py notes)
        cur = "canon" if kc.get("canon", 1) else ("lazyw1" if kc.get("waves") == 1 else "lazy")
        name = min(t, key=t.get)
        if name != cur and t[cur] - t[name] < MARGIN * t[cur]:
            name = cur
        kc["canon"] = 1 if name == "canon" else 0
        if name == "lazyw1":
            kc["waves"] = 1
        kc["us"] = round(t[name], 1)
        best_tot += t[name]
    tune["measured_total_us"] = round(best_tot, 1)
    tune["canon_variants_total_us"] = {n: round(v, 1) for n, v in tot.items()}
    with open(path, "w") as f:
        json.dump(tune, f, indent=1)
    print("totals (ms):", {n: round(v / 1e3, 3) for n, v in tot.items()}, "best per kernel:", round(best_tot / 1e3, 3))


if __name__ == "__main__":
    cmd = sys.argv[1]
    c = CIRCUIT = sys.argv[2] if len(sys.argv) > 2 else "rv32im"
    {"build": lambda: build(c), "measure": measure, "pick": lambda: pick(c)}[cmd]()
