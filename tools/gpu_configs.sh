#!/bin/bash
# The other BASELINE.json configs on one GPU, as bench lines: configs[2] rv32im po2=24 from a
# loop-guest trace; configs[4]'s SHA-256 suite on the recursion circuit (po2=18, random
# programs proved from ctrl + preflight; lift/join programs are absent) with the CPU path's
# seal parity, and on rv32im po2=20; the recursion circuit with Poseidon2 and Poseidon254 at
# po2=18.
TAG=${1:-configs}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
run() {  # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 -u bench.py --e2e-steps 0 --accum-steps 0 --per-op-steps 0 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); c=d.get('cpu_baseline') or {}; print('$n', d['value'], d['ms_per_step'], 'seal_equal', c.get('seal_equal'))"
}
run po2_24 600 --po2 24 --steps 2 --warmup 1 --no-cpu-baseline --resident-steps 0
run sha256_recursion 400 --circuit recursion --hashfn sha-256 --po2 18 --steps 24 --warmup 6
run sha256_rv32im 300 --hashfn sha-256 --no-cpu-baseline
run recursion_p2 300 --circuit recursion --po2 18 --steps 24 --warmup 6 --no-cpu-baseline
run recursion_p254 300 --circuit recursion --hashfn poseidon_254 --po2 18 --steps 12 --warmup 6 --no-cpu-baseline
echo configs done
