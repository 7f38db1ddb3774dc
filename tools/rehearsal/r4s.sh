# witgen: note() selects pinned in program order (no lane masks held to the kernel end) vs the
# previous header (R0HIP_LIB=risc0_amd/lib/libr0hip_ab_base.so), po2 20 loop guest and po2 18
# ecall-heavy guest, alternating on one box
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B=risc0_amd/lib/libr0hip_ab_base.so
for v in base note base note; do
  if [ $v = base ]; then export R0HIP_LIB=$B; else unset R0HIP_LIB; fi
  timeout -k 10 300 python -u tools/micro/rv32im_witgen_bench.py 20 5 --no-ref > $O/wg_$v.json 2> $O/wg_$v.err || { tail -20 $O/wg_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/wg_$v.json')); print('loop $v', d['gpu_phase_ms'])"
  timeout -k 10 300 python -u tools/micro/rv32im_witgen_ecall_bench.py 18 120 3 > $O/ec_$v.json 2> $O/ec_$v.err || { tail -20 $O/ec_$v.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$O/ec_$v.json') if l.startswith('{')][-1]; print('ecall $v', d['gpu_phase_ms'])"
done
unset R0HIP_LIB
for w in loop ec; do
  if [ $w = loop ]; then cmd="tools/micro/rv32im_witgen_bench.py 20 3 --no-ref"; else cmd="tools/micro/rv32im_witgen_ecall_bench.py 18 120 3"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_$w -o run -- python3 $cmd > $O/st_$w.log 2>&1 || { tail -20 $O/st_$w.log; exit 1; }
  python3 -c "
import csv
rows=list(csv.DictReader(open('$O/st_$w/run_kernel_stats.csv')))
print('$w', [(r['Name'].split('(')[0].split('::')[-1], round(float(r['AverageNs'])/1e3,1)) for r in sorted(rows, key=lambda r:-float(r['TotalDurationNs']))[:16]])
"
done
