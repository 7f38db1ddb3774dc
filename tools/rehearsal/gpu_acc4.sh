cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/acc4
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread -k "accum or hipmalloc" > gpurun_out/acc4/p.log 2>&1 || { tail -20 gpurun_out/acc4/p.log; exit 1; }
tail -1 gpurun_out/acc4/p.log
timeout -k 10 300 python3 -u tools/micro/accum_bench.py 20
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --e2e-steps 0 --steps 5 > gpurun_out/acc4/bench.json 2> gpurun_out/acc4/bench.err || { tail -20 gpurun_out/acc4/bench.err; exit 1; }
cat gpurun_out/acc4/bench.json
