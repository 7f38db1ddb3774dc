cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1b/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u bench.py > gpurun_out/r1b/bench.json 2> gpurun_out/r1b/bench.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r1b/prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/r1b/bench_prof.json 2> gpurun_out/r1b/bench_prof.err
echo done $?
