#!/bin/bash
# Round 6: small device-to-host copy costs (the per-op path's query phase), then the trace-job
# and per-op tests and the bench with and without the receipt check (parallel Merkle checks).
TAG=${1:-r6d}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 120 ./tools/micro/small_d2h > $O/small_d2h.txt 2>&1 || { cat $O/small_d2h.txt; exit 1; }
cat $O/small_d2h.txt
timeout -k 10 600 python -u -m pytest tests/test_rv32im_witgen_gpu.py tests/test_per_op_path.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L="--no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0"
for v in on off on; do
  F=""; [ $v = off ] && F="--no-verify --per-op-steps 0"
  timeout -k 10 300 python3 -u bench.py $L $F > $O/bench_verify_$v.json 2> $O/bench_verify_$v.err || { tail -20 $O/bench_verify_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_verify_$v.json')); c=d['config']; p=d.get('per_op_abi') or {}; print('verify $v', d['value'], d['ms_per_step'], c['ms_one_segment_unpipelined'], c['verify_ms_per_segment'], p.get('ms_per_step'), p.get('seal_equal'), (p.get('host_phases_ms') or {}).get('queries'))"
done
