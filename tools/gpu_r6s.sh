cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s; mkdir -p $O
true
tail -1 $O/pytest.log
bash tools/gpu_ab.sh r6s R0HIP_LIB risc0_amd/lib_variants/libr0hip_base.so risc0_amd/lib_variants/libr0hip_rcs.so 3
