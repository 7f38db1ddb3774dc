#!/bin/bash
# segments in flight x HIP hardware queues (CASES "k:q ...", default "3:8 4:8 4:12 5:12"),
# alternating, 12 timed segments each, headline only
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-inflight_hwq}; mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for c in ${CASES:-3:8 4:8 4:12 5:12}; do
    k=${c%%:*}; q=${c##*:}
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --steps 12 --warmup 3 --inflight $k --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 > $O/bench_${k}_${q}_$rep.json 2> $O/bench_${k}_${q}_$rep.err || { tail -5 $O/bench_${k}_${q}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${k}_${q}_$rep.json')); print('inflight=$k hwq=$q', d['value'], d['ms_per_step'], d['config']['seal_sha256_by_rank'], d['device_memory_gb'])"
  done
done
echo done
