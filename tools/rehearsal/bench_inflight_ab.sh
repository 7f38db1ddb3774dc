#!/bin/bash
# segments in flight A/B (ORDER, default "2 3"), alternating, 20 timed segments each (headline only)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do for k in ${ORDER:-2 3}; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --e2e-steps 0 --accum-steps 0 --resident-steps 0 --no-prove-only --inflight $k --steps 20 --warmup 4 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($k, d['value'], d['ms_per_step'])" || exit 1
done; done
