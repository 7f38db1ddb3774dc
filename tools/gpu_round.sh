#!/bin/bash
# One GPU call for a tree worth measuring (run through gpurun from the repo root):
#   the whole -m gpu suite (including full-size eval_check parity), smoke(), the default
#   bench line (with the CPU baseline), a kernel-trace --stats profile and the PMC passes
#   (VALU group, FETCH_SIZE, WRITE_SIZE: one counter group per run, never with tracing).
# Post-process here with tools/post_round.sh TAG.
TAG=${1:-round}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
sha256sum risc0_amd/lib/libr0hip.so | cut -c1-16 > $O/lib_sha256_16
B="bench.py --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 --per-op-steps 0 --steps 3 --warmup 1 --inflight 1"
# a failing test (exit 1) still leaves the profile worth taking; a crash or time limit ends the call
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/pytest_gpu.log; exit 1; fi
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 --per-op-steps 0 --inflight 1 > $O/bench_stats.json 2> $O/bench_stats.err || { tail -20 $O/bench_stats.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/valu -o run -- python3 $B > $O/valu.log 2>&1 || { tail -20 $O/valu.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
echo round profile done
