#!/bin/bash
# Segment pipeline: its parity tests, then single-segment latency from pinned host memory,
# plain and under a kernel + memory-copy trace (tools/timeline.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-oneseg}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "segments or pinned or golden" > $O/p.log 2>&1 || { tail -30 $O/p.log; exit 1; }
tail -1 $O/p.log
timeout -k 10 300 python3 -u tools/micro/one_segment.py > $O/plain.json 2> $O/plain.err || { tail -20 $O/plain.err; exit 1; }
cat $O/plain.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/micro/one_segment.py > $O/traced.json 2> $O/traced.err || { tail -20 $O/traced.err; exit 1; }
cat $O/traced.json
