cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/acc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "accum_finalize" > gpurun_out/acc/p.log 2>&1; rc=$?; tail -15 gpurun_out/acc/p.log; exit $rc
