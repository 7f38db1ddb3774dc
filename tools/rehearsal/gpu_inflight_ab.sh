#!/bin/bash
# Segments in flight at po2=20 (default 3) against 4, at the runtime's default 4 hardware queues
# and at 8, alternating on one box; the default 24-segment session, side legs off.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-inflight}; mkdir -p $O
A="--e2e-steps 0 --accum-steps 0 --per-op-steps 0 --resident-steps 0 --no-cpu-baseline --no-prove-only"
for rep in 1 2; do
  for v in k3 k4 k4q8 k3q8; do
    case $v in
      k3) env=""; k=3;; k4) env=""; k=4;; k4q8) env="GPU_MAX_HW_QUEUES=8"; k=4;; k3q8) env="GPU_MAX_HW_QUEUES=8"; k=3;;
    esac
    env $env timeout -k 10 300 python3 -u bench.py $A --inflight $k > $O/$v.$rep.json 2> $O/$v.$rep.err || { tail -20 $O/$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$rep.json')); print('$v', $rep, d['ms_per_step'], d['value'])"
  done
done
