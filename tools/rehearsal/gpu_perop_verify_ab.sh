#!/bin/bash
# Round 6: the per-op path tests at the BASELINE sizes, then the default bench with and without
# the pipeline's receipt check, alternating on one box (the bench line carries per_op_abi).
TAG=${1:-r6c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_per_op_path.py -v -x --timeout 300 --timeout-method thread > $O/pytest_per_op.log 2>&1 || { tail -60 $O/pytest_per_op.log; exit 1; }
tail -3 $O/pytest_per_op.log
L="--no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0"
for v in on off on off; do
  F=""; [ $v = off ] && F="--no-verify --per-op-steps 0"
  timeout -k 10 300 python3 -u bench.py $L $F > $O/bench_verify_$v.json 2> $O/bench_verify_$v.err || { tail -20 $O/bench_verify_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_verify_$v.json')); c=d['config']; p=d.get('per_op_abi') or {}; print('verify $v', d['value'], d['ms_per_step'], c['ms_one_segment_unpipelined'], c['verify_ms_per_segment'], p.get('ms_per_step'), p.get('seal_equal'), p.get('host_phases_ms'))"
done
