#!/bin/bash
# Poseidon2 wide Merkle layers: two nodes per lane (R0_P2_FOLD_TWO=1, default) against one
# (R0_P2_FOLD_TWO=0) on one box: hash_fold / seal parity tests with each, per-launch times of
# one po2=20 tree's layers (tools/bench_kernels.py fold), the pipelined headline, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-fold_ab}; mkdir -p $O
for v in 1 0; do
  export R0_P2_FOLD_TWO=$v
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fold or merkle or seal_identical" > $O/pytest_$v.log 2>&1 || { echo "two=$v parity FAILED"; tail -20 $O/pytest_$v.log; exit 1; }
  echo "two=$v: $(tail -1 $O/pytest_$v.log)"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$v -o run -- python3 tools/bench_kernels.py fold > $O/fold_$v.log 2>&1 || { tail -5 $O/fold_$v.log; exit 1; }
  python3 -c "import csv,glob; [print('two=$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in csv.DictReader(open(glob.glob('$O/stats_$v/*kernel_stats.csv')[0])) if 'fold' in r['Name']]"
done
for rep in $(seq 1 ${REPS:-2}); do
  for v in 1 0; do
    export R0_P2_FOLD_TWO=$v
    timeout -k 10 300 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); print('two=$v', d['value'], d['ms_per_step'], d['config']['seal_sha256_by_rank'])"
  done
done
echo done
