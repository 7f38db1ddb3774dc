#!/bin/bash
# runtime environment A/B for the pipelined headline and the one-segment latency: CASES is a
# list of "NAME=VALUE[,NAME=VALUE]" ("-" = nothing extra), alternating, 12 timed segments each
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-env_ab}; mkdir -p $O
i=0
for rep in $(seq 1 ${REPS:-2}); do
  for c in ${CASES:--}; do
    i=$((i + 1))
    ( [ "$c" != "-" ] && for kv in ${c//,/ }; do export "$kv"; done
      exec timeout -k 10 300 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 ) > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print('$c', d['value'], d['ms_per_step'], d['config']['seal_sha256_by_rank'], 'one', d['config'].get('ms_one_segment_unpipelined'))"
  done
done
echo done
