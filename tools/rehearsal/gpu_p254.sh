#!/bin/bash
# GPU parity suite, default bench line (with the end-to-end leg), recursion/poseidon_254 bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p254b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-steps 0 --circuit recursion --hashfn poseidon_254 --po2 18 --steps 8 --warmup 2 --inflight 4 > $O/rec_p254.json 2> $O/rec_p254.err || { tail -20 $O/rec_p254.err; exit 1; }
cat $O/rec_p254.json; head -c 1200 $O/rec_p254.err
