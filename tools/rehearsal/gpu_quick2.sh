#!/bin/bash
# Parity of the touched ops (-k filter) + a bench line + kernel stats families.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-quick2}; K=${2:-golden}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/p.log 2>&1 || { tail -30 $O/p.log; exit 1; }
tail -1 $O/p.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --e2e-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline --e2e-steps 0 --inflight 1 > $O/bs.json 2> $O/bs.err || { tail -20 $O/bs.err; exit 1; }
python3 tools/rocprof_families.py $(find $O/stats -name "*kernel_stats.csv") 9 > $O/families.txt && head -12 $O/families.txt
