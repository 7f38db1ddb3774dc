#!/bin/bash
# SHA-256 suite benches: recursion po2=18 (BASELINE configs[4]) and rv32im po2=20
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sha; mkdir -p $O
for a in "recursion 18" "rv32im 20"; do set -- $a
timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-steps 0 --circuit $1 --hashfn sha-256 --po2 $2 --steps 6 --warmup 2 > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', d['value'], d['ms_per_step'], d['roofline']['kernel'])"
head -c 900 $O/$1.err; echo
done
