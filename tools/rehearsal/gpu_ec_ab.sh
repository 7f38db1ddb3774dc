#!/bin/bash
# eval_check A/B on one box: eval_check parity tests for the in-tree library, then the
# per-launch eval_check time (tools/bench_kernels.py ec, HIP events, alternating builds) for
# the in-tree library and risc0_amd/lib_variants/libr0hip_old.so, plus one malloc-traced run
# of the steady-state allocation test (R0HIP_TRACE_MALLOC=1).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ec_ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "eval_check" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
R0HIP_TRACE_MALLOC=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "steady_state" > $O/steady.log 2>&1 || echo "steady-state test failed (see $O/steady.log)"
tail -1 $O/steady.log
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export R0HIP_LIB=$PWD/risc0_amd/lib_variants/libr0hip_old.so; else unset R0HIP_LIB; fi
    timeout -k 10 200 python3 tools/bench_kernels.py ec > $O/$v$rep.log 2>&1 || { tail -5 $O/$v$rep.log; exit 1; }
    grep -h "eval_check" $O/$v$rep.log | head -3
  done
done
