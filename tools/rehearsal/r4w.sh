# witgen merge kernel: eight branch-free loads in flight per lane (new) vs one load-store round
# trip per column (base = R0HIP_LIB libr0hip_ab_base.so); both with XCD-contiguous row tiles
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then export R0HIP_LIB=risc0_amd/lib/libr0hip_ab_base.so; else unset R0HIP_LIB; fi
  timeout -k 10 300 python -u tools/micro/rv32im_witgen_bench.py 20 7 --no-ref > $O/wg_$v.json 2> $O/wg_$v.err || { tail -20 $O/wg_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/wg_$v.json')); print('$v', d['gpu_phase_ms'])"
done
unset R0HIP_LIB
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o run -- python3 bench.py --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --inflight 1 --steps 3 --warmup 1 > $O/st.log 2>&1 || { tail -20 $O/st.log; exit 1; }
python3 -c "
import csv
rows=list(csv.DictReader(open('$O/st/run_kernel_stats.csv')))
print([(r['Name'].split('(')[0].split('::')[-1], r['Calls'], round(float(r['AverageNs'])/1e3,1)) for r in rows if 'merge' in r['Name']])
"
