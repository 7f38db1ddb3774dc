#!/bin/bash
# GPU parity suite + recursion SHA-256 / Poseidon254 benches
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rec; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for h in "sha-256 2" "poseidon_254 4"; do set -- $h
timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-steps 0 --circuit recursion --hashfn $1 --po2 18 --steps 8 --warmup 2 --inflight $2 > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', d['value'], d['ms_per_step'])"
head -c 400 $O/$1.err; echo
done
