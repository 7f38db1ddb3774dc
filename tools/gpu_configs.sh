#!/bin/bash
# The other BASELINE.json configs on one GPU, as bench lines (no CPU baseline, no
# end-to-end leg): configs[2] rv32im po2=24; configs[4]'s SHA-256 suite on the recursion
# circuit (po2=18; lift/join programs are absent) and on rv32im po2=20; the recursion
# circuit with Poseidon2 and Poseidon254 at po2=18.
TAG=${1:-configs}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
run() {  # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 -u bench.py --no-cpu-baseline --e2e-steps 0 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'])"
}
run po2_24 500 --po2 24 --steps 2 --warmup 1
run sha256_recursion 300 --circuit recursion --hashfn sha-256 --po2 18 --steps 12 --warmup 6
run sha256_rv32im 300 --hashfn sha-256 --steps 6 --warmup 3
run recursion_p2 300 --circuit recursion --po2 18 --steps 12 --warmup 6
run recursion_p254 300 --circuit recursion --hashfn poseidon_254 --po2 18 --steps 12 --warmup 6
echo configs done
