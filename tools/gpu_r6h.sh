#!/bin/bash
# Round 6: the default bench line exactly as the driver runs it (24 segments of one loop.s
# session), then the other configs (tools/gpu_configs.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
bash tools/gpu_configs.sh r6h_configs
