#!/bin/bash
# Segment pipeline check: pipeline goldens + the bench's end-to-end leg (single segment
# latency with the witness in pinned host memory, and the pipelined rate).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-e2e2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "segments or pinned or golden" > $O/p.log 2>&1 || { tail -30 $O/p.log; exit 1; }
tail -1 $O/p.log
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['end_to_end']))"
