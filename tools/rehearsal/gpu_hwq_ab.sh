#!/bin/bash
# Hardware queues per process: the box default (GPU_MAX_HW_QUEUES=4) against more (QS, default
# "4 8") for the pipelined headline (the main thread's stream, the uploader's and three provers'
# = 5 streams), alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-hwq_ab}; mkdir -p $O
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
for rep in $(seq 1 ${REPS:-3}); do
  for q in ${QS:-4 8}; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 > $O/bench_${q}_$rep.json 2> $O/bench_${q}_$rep.err || { tail -5 $O/bench_${q}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${q}_$rep.json')); print('hwq=$q', d['value'], d['ms_per_step'], d['config']['seal_sha256_by_rank'], d['config'].get('ms_one_segment_unpipelined'))"
  done
done
echo done
