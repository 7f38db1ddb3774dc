# rv32im witgen arm kernels: 64 / 256 threads per workgroup vs 128 (base), standalone phase
# times on the po2 20 loop guest and the po2 18 ecall-heavy guest, alternating; witgen GPU
# tests with each variant
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4thr; mkdir -p $O
for v in t64 t256; do
  R0HIP_LIB=risc0_amd/lib/libr0hip_ab_$v.so timeout -k 10 600 python -u -m pytest tests/test_rv32im_witgen_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; tail -1 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in base t64 t256 base t64 t256; do
  export R0HIP_LIB=risc0_amd/lib/libr0hip_ab_$v.so
  timeout -k 10 300 python -u tools/micro/rv32im_witgen_bench.py 20 5 --no-ref > $O/wg_$v.json 2> $O/wg_$v.err || { tail -20 $O/wg_$v.err; exit 1; }
  timeout -k 10 300 python -u tools/micro/rv32im_witgen_ecall_bench.py 18 120 3 > $O/ec_$v.json 2> $O/ec_$v.err || { tail -20 $O/ec_$v.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/wg_$v.json'))['gpu_phase_ms']; e=[json.loads(l) for l in open('$O/ec_$v.json') if l.startswith('{')][-1]['gpu_phase_ms']
print('$v loop exec', d['rv32im_witgen_exec'], 'tables', d['rv32im_witgen_tables'], '| ecall exec', e['rv32im_witgen_exec'], 'tables', e['rv32im_witgen_tables'])
"
done
