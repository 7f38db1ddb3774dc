#!/bin/bash
# Four ranks through torch.distributed.run on a one-GPU box (all sharing GPU 0,
# R0_BENCH_SHARE_GPUS=1): one JSON line with n_gpus 4, the session's 4 x 2 consecutive
# segments split i mod 4, every receipt verified.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ranks4}; mkdir -p $O
export R0_BENCH_SHARE_GPUS=1
B="--gpus 4 --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 --accum-steps 0 --per-op-steps 0 --resident-steps 0 --no-prove-only"
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 bench.py $B > $O/trun.json 2> $O/trun.err || { tail -30 $O/trun.err; exit 1; }
cat $O/trun.json
