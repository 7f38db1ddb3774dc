#!/bin/bash
# Recursion witness generation A/B on one box: the in-tree library (new) against
# risc0_amd/lib_variants/libr0hip_rwold.so (old): recursion parity tests, per-kernel times of the
# recursion SHA-256 bench (rocprofv3 --stats: the witgen kernels), then the recursion (po2=18)
# and rv32im (po2=20) SHA-256 bench lines, alternating builds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-sha_ab}; mkdir -p $O
sel() { if [ $1 = old ]; then export R0HIP_LIB=$PWD/risc0_amd/lib_variants/libr0hip_rwold.so; else unset R0HIP_LIB; fi; }
REC="--circuit recursion --hashfn sha-256 --po2 18 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "recursion" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in new old; do
  sel $v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$v -o run -- python3 bench.py $REC --steps 8 --warmup 2 > $O/stats_$v.json 2> $O/stats_$v.err || { tail -5 $O/stats_$v.err; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys
for v in ("new", "old"):
    f = glob.glob(sys.argv[1] + f"/stats_{v}/*kernel_stats.csv")[0]
    for r in csv.DictReader(open(f)):
        if "rwg" in r["Name"] or "exec_kernel" in r["Name"]:
            print(v, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg,", round(float(r["TotalDurationNs"]) / 1e6, 2), "ms total")
PY
for rep in 1 2; do
  for v in new old; do
    sel $v
    timeout -k 10 300 python3 bench.py $REC --steps 24 --warmup 6 > $O/rec_${v}_$rep.json 2> $O/rec_${v}_$rep.err || { tail -5 $O/rec_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/rec_${v}_$rep.json')); print('recursion', '$v', d['value'], d['ms_per_step'], d['config']['seal_sha256_by_rank'])"
    timeout -k 10 300 python3 bench.py --hashfn sha-256 --steps 12 --warmup 3 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 > $O/rv_${v}_$rep.json 2> $O/rv_${v}_$rep.err || { tail -5 $O/rv_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/rv_${v}_$rep.json')); print('rv32im', '$v', d['value'], d['ms_per_step'], d['config']['seal_sha256_by_rank'])"
  done
done
echo done
