#!/bin/bash
# Profile the po2=20 bench on an MI355X box (run through gpurun from the repo root):
#   kernel-trace stats (csv), then one PMC pass per counter group (never combined with
#   tracing domains), each under its own time limit; stops at the first failure.
# usage: bash tools/gpu_profile.sh TAG
set -e
TAG=${1:-prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
B="bench.py --no-cpu-baseline --e2e-steps 0 --steps 3 --warmup 1 --inflight 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline --e2e-steps 0 --inflight 1 > $O/bench_stats.json 2> $O/bench_stats.err
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/valu -o run -- python3 $B > $O/valu.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B > $O/write.log 2>&1
echo profile done
