#!/bin/bash
# Round 6: the library hands each thread's idle device memory back at call end and runs one
# prover on the calling thread. GPU tests, then the default bench at the runtime's default 4
# hardware queues against 8 (same box), then po2=24 (the leg that ran out of memory in r5bb).
TAG=${1:-r6a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
L="--no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0"
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 -u bench.py $L > $O/bench_q$q.json 2> $O/bench_q$q.err || { tail -20 $O/bench_q$q.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_q$q.json')); print('queues $q', d['value'], d['ms_per_step'], d['config']['ms_one_segment_unpipelined'])"
done
timeout -k 10 600 python3 -u bench.py --po2 24 --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 --accum-steps 0 > $O/po2_24.json 2> $O/po2_24.err || { tail -20 $O/po2_24.err; exit 1; }
cat $O/po2_24.json
