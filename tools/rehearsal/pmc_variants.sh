cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcvar
for v in canon_plain lazy_plain; do
  R0HIP_LIB=$PWD/risc0_amd/lib_variants/libr0hip_tune_$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcvar/$v -o run -- python3 tools/bench_kernels.py ec > gpurun_out/pmcvar/$v.log 2>&1 || exit 1
done
echo ok
