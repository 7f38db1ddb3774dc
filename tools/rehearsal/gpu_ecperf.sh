#!/bin/bash
# eval_check variant check: parity (all eval_check tests), one bench line, and a
# kernel-trace stats profile of the po2=20 bench (per-kernel means for the families).
TAG=${1:-ecperf}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "eval_check" > $O/ec.log 2>&1 || { tail -30 $O/ec.log; exit 1; }
tail -1 $O/ec.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline --e2e-steps 0 --inflight 1 > $O/bench_stats.json 2> $O/bench_stats.err || { tail -20 $O/bench_stats.err; exit 1; }
python3 tools/rocprof_families.py $(find $O/stats -name "*kernel_stats.csv") 9 > $O/families.txt && cat $O/families.txt
