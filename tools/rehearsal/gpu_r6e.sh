#!/bin/bash
# Round 6: FETCH_SIZE calibration on known byte counts, the whole -m gpu suite, smoke(), the
# default bench line, then configs[3]'s session leg (64 consecutive segments of one loop.s run).
TAG=${1:-r6e}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
sha256sum risc0_amd/lib/libr0hip.so | cut -c1-16 > $O/lib_sha256_16
timeout -k 10 60 ./tools/micro/fetch_calib > $O/fetch_calib.txt 2>&1 || { cat $O/fetch_calib.txt; exit 1; }
cat $O/fetch_calib.txt
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_calib_pmc -o run -- ./tools/micro/fetch_calib > $O/fetch_calib_pmc.log 2>&1 || { tail -20 $O/fetch_calib_pmc.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 900 python -u bench.py --session 64 --no-cpu-baseline --no-prove-only --per-op-steps 0 --resident-steps 0 --e2e-steps 0 --accum-steps 0 > $O/bench_session64.json 2> $O/bench_session64.err || { tail -20 $O/bench_session64.err; exit 1; }
cat $O/bench_session64.json
