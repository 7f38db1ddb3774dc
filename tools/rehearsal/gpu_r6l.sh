#!/bin/bash
# The asynchronous node-heap mirror: the copy API test, the per-op path tests and the bench's
# per_op_abi leg.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "async_mirror or pinned_host or steady_state" tests/test_per_op_path.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 -u bench.py --steps 6 --e2e-steps 0 --accum-steps 0 --resident-steps 0 --no-cpu-baseline --no-prove-only --per-op-steps 3 > $O/bench_perop.json 2> $O/bench_perop.err || { tail -30 $O/bench_perop.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_perop.json')); p=d['per_op_abi']; print('per_op', p['ms_per_step'], p['seal_equal'], p['mix_equal'], p['host_phases_ms'])"
