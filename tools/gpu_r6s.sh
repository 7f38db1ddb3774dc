#!/bin/bash
# r6s: same-box A/B of two library builds (risc0_amd/lib_variants/libr0hip_{base,rcs}.so,
# built by hand from the tree before and after the Poseidon2 sredc_rc change), 3 rounds; the
# GPU tests of the new build ran in the call before (profiles/r6s_p2_rc_in_redc_ab.txt).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_ab.sh r6s R0HIP_LIB risc0_amd/lib_variants/libr0hip_base.so risc0_amd/lib_variants/libr0hip_rcs.so 3
