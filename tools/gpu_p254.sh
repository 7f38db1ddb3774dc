#!/bin/bash
# Poseidon254 suite on the GPU: parity tests, then a recursion po2=18 poseidon_254 bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p254; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --circuit recursion --hashfn poseidon_254 --po2 18 --steps 3 --warmup 1 > $O/bench_rec_p254.json 2> $O/bench_rec_p254.err || { tail -20 $O/bench_rec_p254.err; exit 1; }
cat $O/bench_rec_p254.json; head -c 1500 $O/bench_rec_p254.err
