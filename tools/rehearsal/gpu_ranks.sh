#!/bin/bash
# Rehearsal of bench.py's multi-rank paths on a one-GPU box (the driver runs N = 1, 2, 4, 8
# on a whole node): both ranks share GPU 0 (R0_BENCH_SHARE_GPUS=1). The self-launched
# `--gpus 2` path and the torch.distributed.run path must each print one JSON line with
# n_gpus 2 and two seal digests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ranks}; mkdir -p $O
export R0_BENCH_SHARE_GPUS=1
B="--gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0"
timeout -k 10 400 python3 -u bench.py $B > $O/self.json 2> $O/self.err || { tail -30 $O/self.err; exit 1; }
cat $O/self.json
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py $B > $O/trun.json 2> $O/trun.err || { tail -30 $O/trun.err; exit 1; }
cat $O/trun.json
