#!/bin/bash
# NTT parity tests, then per-kernel times of tools/bench_kernels.py ntt for the in-tree
# library and risc0_amd/lib_variants/libr0hip_old.so (same box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ntt_ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "ntt or interpolate or expand or bit_reverse or seal" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in new old; do
  if [ $v = old ]; then export R0HIP_LIB=$PWD/risc0_amd/lib_variants/libr0hip_old.so; else unset R0HIP_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/bench_kernels.py ntt > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys
for v in ("new", "old"):
    f = glob.glob(sys.argv[1] + f"/{v}/*kernel_stats.csv")[0]
    tot = 0
    for r in csv.DictReader(open(f)):
        if "ntt_pass" in r["Name"]:
            tot += float(r["TotalDurationNs"])
            print(v, r["Name"][40:120], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
    print(v, "total ntt_pass ms", round(tot / 1e6, 3))
PY
# the headline (trace jobs, 12 steps, no side legs), alternating builds
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export R0HIP_LIB=$PWD/risc0_amd/lib_variants/libr0hip_old.so; else unset R0HIP_LIB; fi
    timeout -k 10 300 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); print('$v', d['value'], d['ms_per_step'])"
  done
done
