#!/bin/bash
# eval_check retune (3 kernels' waves/prefetch from tools/tune_eval_check.py) against the committed
# tuning, alternating libraries on one box, 3 rounds: the pipelined headline, then eval_check alone
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_ab.sh r6aa R0HIP_LIB risc0_amd/lib_variants/libr0hip_base.so risc0_amd/lib_variants/libr0hip_tuned.so 3
