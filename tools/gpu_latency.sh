#!/bin/bash
# One segment's latency through the pipeline, split (config.one_segment_split), and the
# pipeline's per-job test.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-lat}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_rv32im_witgen_gpu.py -k "verification_fails" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 -u bench.py --steps 6 --e2e-steps 0 --accum-steps 0 --per-op-steps 0 --resident-steps 0 --no-cpu-baseline --no-prove-only > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['config']; print(d['ms_per_step'], c['ms_one_segment_unpipelined'], c['one_segment_split'])"
