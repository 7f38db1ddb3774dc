#!/bin/bash
# eval_check re-split A/B on one box: the in-tree library against the
# variants in risc0_amd/lib_variants/ (built with EC_RESPLIT / EC_RESPLIT_WAVES, see
# tools/gen_eval_check.py resplit_config): eval_check parity for each, then per-kernel times
# (rocprofv3 --kernel-trace --stats over tools/bench_kernels.py ec, alternating builds), then
# the bench's trace headline per build.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ec_resplit}; mkdir -p $O
VARIANTS="base ${VARIANTS:-rs2 rs3}"
lib() { if [ $1 = base ]; then unset R0HIP_LIB; else export R0HIP_LIB=$PWD/risc0_amd/lib_variants/libr0hip_$1.so; fi; }
for v in $VARIANTS; do
  lib $v
  timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "eval_check and (rv32im or golden)" > $O/pytest_$v.log 2>&1 || { echo "$v parity FAILED"; tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2; do
  for v in $VARIANTS; do
    lib $v
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_${v}_$rep -o run -- python3 tools/bench_kernels.py ec > $O/ec_${v}_$rep.log 2>&1 || { tail -5 $O/ec_${v}_$rep.log; exit 1; }
    grep -h "eval_check" $O/ec_${v}_$rep.log | head -1
  done
done
for rep in 1 2; do
  for v in $VARIANTS; do
    lib $v
    timeout -k 10 300 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/bench_${v}_$rep.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
echo done
