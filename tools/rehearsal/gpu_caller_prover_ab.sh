#!/bin/bash
# One prover on the calling thread (libr0hip.so) against k prover threads (lib_variants/
# libr0hip_base.so): the pipeline tests with the new library, then the pipelined headline at
# 4 and 8 hardware queues with each, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-caller_ab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_rv32im_witgen_gpu.py -k "prove_segments" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=risc0_amd/lib_variants/libr0hip_base.so
CASES="GPU_MAX_HW_QUEUES=4,R0_BENCH_HW_QUEUES_AS_IS=1 GPU_MAX_HW_QUEUES=4,R0_BENCH_HW_QUEUES_AS_IS=1,R0HIP_LIB=$B GPU_MAX_HW_QUEUES=8 GPU_MAX_HW_QUEUES=8,R0HIP_LIB=$B" bash tools/rehearsal/gpu_env_ab.sh ${1:-caller_ab}/bench
