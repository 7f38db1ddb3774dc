#!/bin/bash
# rv32im accumulation on the GPU against the compiled reference (phases 1-3 and 2-3 alone).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/acc
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -k "accum" > gpurun_out/acc/p.log 2>&1; rc=$?; tail -25 gpurun_out/acc/p.log; exit $rc
