#!/bin/bash
# NTT parity tests and per-kernel times of tools/bench_kernels.py ntt for the in-tree
# library and each risc0_amd/lib_variants/libr0hip_<name>.so (same box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ntt_var}; mkdir -p $O
for lib in tree risc0_amd/lib_variants/libr0hip_*.so; do
  v=$(basename $lib .so); v=${v#libr0hip_}
  if [ $lib = tree ]; then unset R0HIP_LIB; else export R0HIP_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "ntt or interpolate or expand or seal" > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/bench_kernels.py ntt > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, os, sys
for d in sorted(glob.glob(sys.argv[1] + "/*/")):
    fs = glob.glob(d + "*kernel_stats.csv")
    if not fs: continue
    v = os.path.basename(d.rstrip("/")); tot = 0
    for r in csv.DictReader(open(fs[0])):
        if "ntt_pass" in r["Name"]:
            tot += float(r["TotalDurationNs"])
            print(v, r["Name"][40:120], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
    print(v, "total ntt_pass ms", round(tot / 1e6, 3))
PY
