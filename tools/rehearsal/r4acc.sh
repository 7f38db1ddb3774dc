# rv32im accumulation kernels at an occupancy target (R0_ACC_WAVES 3 / 4: amdgpu_waves_per_eu,
# some scratch) vs the compiler's own register budget (base); accum tests with each library
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4acc; mkdir -p $O
for v in w3 w4; do
  R0HIP_LIB=risc0_amd/lib/libr0hip_ab_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "accum" --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; tail -1 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in base w3 w4 base w3 w4; do
  R0HIP_LIB=risc0_amd/lib/libr0hip_ab_$v.so timeout -k 10 300 python -u tools/micro/accum_bench.py 20 > $O/acc_$v.json 2> $O/acc_$v.err || { tail -20 $O/acc_$v.err; exit 1; }
  echo "$v $(tail -1 $O/acc_$v.json)"
done
