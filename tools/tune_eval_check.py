#!/usr/bin/env python3
"""Per-kernel autotuning of the generated eval_check kernels (register target and load
prefetch distance), measured on an MI355X.

  python tools/tune_eval_check.py build [CIRCUIT]     # variants -> risc0_amd/lib_variants/
  gpurun -- 'python tools/tune_eval_check.py measure'  # rocprofv3 per-kernel times
  python tools/tune_eval_check.py pick [CIRCUIT]      # -> risc0_amd/circuits/<c>.ectune.json

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


def pick(circuit):
    best = {}
    for d in sorted(glob.glob(os.path.join(OUT, "w*_pf*"))):
        m = re.match(r"w(\d+)_pf(\d+)", os.path.basename(d))
        w, pf = int(m.group(1)), int(m.group(2))
        for r in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
            km = re.search(r"ec_" + circuit + r"::k(\d+)", r["Name"])
            if not km:
                continue
            k, t = int(km.group(1)), float(r["AverageNs"]) / 1e3
            if k not in best or t < best[k][0]:
                best[k] = (t, w, pf)
    tot = sum(v[0] for v in best.values())
    path = os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".ectune.json")
    prev = json.load(open(path)) if os.path.exists(path) else {}
    kern = {str(k): dict(prev.get("kernels", {}).get(str(k), {})) for k in best}
    for k, v in best.items():  # other per-kernel fields (canon, pinb) were fixed in the variants
        kern[str(k)].update(waves=v[1], pf=v[2], us=round(v[0], 1))
    out = {"budget": BUDGET, "order": "dfs", "measured_total_us": round(tot, 1),
           "kernels": {k: kern[k] for k in sorted(kern, key=int)}}
    if prev.get("mat"):
        out["mat"] = prev["mat"]  # the partition these kernels belong to
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {path}: {len(best)} kernels, sum of best {tot / 1e3:.2f} ms")


if __name__ == "__main__":
    cmd = sys.argv[1]
    c = CIRCUIT = sys.argv[2] if len(sys.argv) > 2 else "rv32im"
    {"build": lambda: build(c), "measure": measure, "pick": lambda: pick(c)}[cmd]()
