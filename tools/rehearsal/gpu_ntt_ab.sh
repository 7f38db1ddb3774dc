#!/bin/bash
# NTT A/B on one box: for each variant (name=LIB, LIB "-" for the in-tree library or a suffix
# of risc0_amd/lib_variants/libr0hip_<LIB>.so) the NTT parity tests and per-kernel times of
# tools/bench_kernels.py ntt, then the pipelined headline (trace jobs, 12 steps, no side legs),
# alternating variants.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ntt_ab}; mkdir -p $O
VARIANTS=${VARIANTS:-"new=- old=old"}
sel() { local lib=${1#*=}; if [ "$lib" = "-" ]; then unset R0HIP_LIB; else export R0HIP_LIB=$PWD/risc0_amd/lib_variants/libr0hip_$lib.so; fi; }
for nm in $VARIANTS; do
  v=${nm%%=*}; sel $nm
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "ntt or interpolate or expand or bit_reverse or seal" > $O/pytest_$v.log 2>&1 || { echo "$v parity FAILED"; tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/bench_kernels.py ntt > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
done
python3 - "$O" $VARIANTS <<'PY'
import csv, glob, sys
for nm in sys.argv[2:]:
    v = nm.split("=")[0]
    f = glob.glob(sys.argv[1] + f"/{v}/*kernel_stats.csv")[0]
    tot = 0
    for r in csv.DictReader(open(f)):
        if "ntt_pass" in r["Name"]:
            tot += float(r["TotalDurationNs"])
            print(v, r["Name"][40:120], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
    print(v, "total ntt_pass ms", round(tot / 1e6, 3))
PY
for rep in $(seq 1 ${REPS:-2}); do
  for nm in $VARIANTS; do
    v=${nm%%=*}; sel $nm
    timeout -k 10 300 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); print('$v', d['value'], d['ms_per_step'], d['config']['seal_sha256_by_rank'])"
  done
done
echo done
