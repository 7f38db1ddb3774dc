#!/bin/bash
# Segments in flight 3 against 4 on the final library, alternating, 3 rounds (default session,
# side legs off).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z; mkdir -p $O
A="--e2e-steps 0 --accum-steps 0 --per-op-steps 0 --resident-steps 0 --no-cpu-baseline --no-prove-only"
for rep in 1 2 3; do
  for k in 3 4; do
    timeout -k 10 300 python3 -u bench.py $A --inflight $k > $O/k$k.$rep.json 2> $O/k$k.$rep.err || { tail -20 $O/k$k.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/k$k.$rep.json')); print('inflight $k run $rep', d['ms_per_step'], d['value'], d['device_memory_gb'])" | tee -a $O/ab.txt
  done
done
