#!/bin/bash
# eval_check A/B on one box over builds and tap forms. Each kernel is compiled twice (32-bit
# tap indices, or column bases from A.cp + a 32-bit byte offset); R0_EC_WIDE selects, per
# kernel, the column-base form at po2 <= 22 (mask; empty = the tuned default). A variant is
# name=LIB,MASK with LIB "-" for the in-tree library or a suffix of
# risc0_amd/lib_variants/libr0hip_<LIB>.so. For each: eval_check parity, per-kernel times and
# VALU instruction counts (tools/bench_kernels.py ec), then the pipelined trace headline,
# alternating variants. CIRCUIT=recursion runs the recursion circuit's kernels and bench
# (po2=18, SHA-256, random programs).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ec_ab}; mkdir -p $O
VARIANTS=${VARIANTS:-"base=- wide=-,0x3fffffff"}
CIRCUIT=${CIRCUIT:-rv32im}
export R0_EC_CIRCUIT=$CIRCUIT
if [ $CIRCUIT = rv32im ]; then
  KSEL="eval_check and (rv32im or golden)"
  BENCH="--steps 12 --warmup 3 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0"
else
  KSEL="eval_check and recursion"
  BENCH="--circuit recursion --hashfn sha-256 --po2 18 --steps 24 --warmup 6 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0"
fi
sel() {
  local spec=${1#*=} lib mask
  lib=${spec%%,*}; mask=${spec#*,}; [ "$mask" = "$spec" ] && mask=
  if [ "$lib" = "-" ]; then unset R0HIP_LIB; else export R0HIP_LIB=$PWD/risc0_amd/lib_variants/libr0hip_$lib.so; fi
  if [ -z "$mask" ]; then unset R0_EC_WIDE; else export R0_EC_WIDE=$mask; fi
}
for nm in $VARIANTS; do
  v=${nm%%=*}; sel $nm
  timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "$KSEL" > $O/pytest_$v.log 2>&1 || { echo "$v parity FAILED"; tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for nm in $VARIANTS; do
  v=${nm%%=*}; sel $nm
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$v -o run -- python3 tools/bench_kernels.py ec > $O/ec_$v.log 2>&1 || { tail -5 $O/ec_$v.log; exit 1; }
  grep -h "eval_check" $O/ec_$v.log | head -1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/valu_$v -o run -- python3 tools/bench_kernels.py ec > $O/valu_$v.log 2>&1 || { tail -5 $O/valu_$v.log; exit 1; }
done
for rep in $(seq 1 ${REPS:-2}); do
  for nm in $VARIANTS; do
    v=${nm%%=*}; sel $nm
    timeout -k 10 300 python3 bench.py $BENCH > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/bench_${v}_$rep.json')); print('$v', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('avg_launch_ms'), d['config']['seal_sha256_by_rank'])"
  done
done
echo done
