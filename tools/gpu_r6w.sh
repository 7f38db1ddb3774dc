#!/bin/bash
# Round 6 final library: configs[3]'s 64 consecutive segments on one GPU, then the other
# BASELINE configs (tools/gpu_configs.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 600 python3 -u bench.py --session 64 --no-cpu-baseline --e2e-steps 0 --accum-steps 0 --per-op-steps 0 --resident-steps 0 --no-prove-only > $O/session64.json 2> $O/session64.err || { tail -30 $O/session64.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/session64.json')); print('session64', d['value'], d['ms_per_step'], d['config']['distinct_seals_rank0'], d['config']['receipts_verified'])"
bash tools/gpu_configs.sh r6w_configs
