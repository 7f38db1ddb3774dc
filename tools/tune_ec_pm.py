#!/usr/bin/env python3
"""Per-kernel choice of how the generated eval_check kernels read the poly_mix table,
measured on an MI355X, on top of the committed tuning (waves, prefetch, canon per kernel in
risc0_amd/circuits/<c>.ectune.json).

  python tools/tune_ec_pm.py build [CIRCUIT]      # variants -> risc0_amd/lib_variants/
  gpurun -- 'python tools/tune_ec_pm.py measure'  # rocprofv3 per-kernel times
  python tools/tune_ec_pm.py pick [CIRCUIT]       # "pinb" per kernel into the tune file

Variant "off" is the committed tuning as is (scalar loads the compiler hoists to the kernel
start and spills to VGPR lanes); "b<n>" pins the table pointer per batch of n poly_mix terms
(gen_eval_check.py EC_PINB). `pick` keeps, per kernel, the fastest variant. (The first
version of this tool measured EC_PMV, vector loads of the table: 1.1-9x slower per kernel.)
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
OUT = os.path.join(ROOT, "gpurun_out", "tune_pm")
BATCHES = (4, 8, 16)


def variants():
    yield "off", {}
    for n in BATCHES:
        yield f"b{n}", {"EC_PINB": str(n)}


def build(circuit):
    os.makedirs(VAR, exist_ok=True)
    for f in glob.glob(os.path.join(VAR, "libr0hip_pm_*.so")):
        os.remove(f)
    for tag, extra in variants():
        shutil.rmtree(os.path.join(CSRC, "gen", circuit), ignore_errors=True)
        env = dict(os.environ, **extra)
        subprocess.run(["make", "-j8"], cwd=CSRC, env=env, check=True, stdout=subprocess.DEVNULL)
        shutil.copy(os.path.join(ROOT, "risc0_amd", "lib", "libr0hip.so"),
                    os.path.join(VAR, f"libr0hip_pm_{tag}.so"))
        print("built", tag, flush=True)
    shutil.rmtree(os.path.join(CSRC, "gen", circuit), ignore_errors=True)
    subprocess.run(["make", "-j8"], cwd=CSRC, check=True, stdout=subprocess.DEVNULL)


def measure(circuit="rv32im"):
    os.makedirs(OUT, exist_ok=True)
    for lib in sorted(glob.glob(os.path.join(VAR, "libr0hip_pm_*.so"))):
        tag = os.path.basename(lib)[len("libr0hip_pm_"):-3]
        env = dict(os.environ, R0HIP_LIB=lib, TMPDIR="/tmp", R0_EC_CIRCUIT=circuit)
        subprocess.run(["timeout", "-k", "10", "200", "rocprofv3", "--kernel-trace", "--stats", "-d",
                        os.path.join(OUT, tag), "-o", "run", "--output-format", "csv", "--", sys.executable,
                        os.path.join(ROOT, "tools", "bench_kernels.py"), "ec"], env=env, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        print("measured", tag, flush=True)


def pick(circuit):
    times = {}
    for d in sorted(glob.glob(os.path.join(OUT, "*"))):
        tag = os.path.basename(d)
        for r in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
            km = re.search(r"ec_" + circuit + r"::k(\d+)<false>", r["Name"])
            if km:
                times.setdefault(int(km.group(1)), {})[tag] = float(r["AverageNs"]) / 1e3
    path = os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".ectune.json")
    cfg = json.load(open(path))
    tot_off = tot = 0.0
    for k, ts in sorted(times.items()):
        tag = min(ts, key=ts.get)
        kc = cfg["kernels"].setdefault(str(k), {})
        kc.pop("pinb", None)
        if tag != "off":
            kc["pinb"] = int(tag[1:])
        kc["us"] = round(ts[tag], 1)
        tot_off += ts.get("off", ts[tag])
        tot += ts[tag]
        print(f"k{k:<3d} " + " ".join(f"{t}={v:8.1f}" for t, v in sorted(ts.items())) + f"  -> {tag}")
    cfg["measured_total_us"] = round(tot, 1)
    with open(path, "w") as f:
        json.dump(cfg, f, indent=1)
    print(f"wrote {path}: sum of kernel means {tot_off / 1e3:.2f} ms without, {tot / 1e3:.2f} ms with the picks")


if __name__ == "__main__":
    cmd = sys.argv[1]
    c = sys.argv[2] if len(sys.argv) > 2 else "rv32im"
    {"build": lambda: build(c), "measure": lambda: measure(c), "pick": lambda: pick(c)}[cmd]()
