# witgen with notes pinned in arms 4 and 11 only (PIN_NOTES): GPU witgen tests, per-kernel
# stats, then the trace headline against the unpinned library, alternating
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in loop ec; do
  if [ $w = loop ]; then cmd="tools/micro/rv32im_witgen_bench.py 20 3 --no-ref"; else cmd="tools/micro/rv32im_witgen_ecall_bench.py 18 120 3"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_$w -o run -- python3 $cmd > $O/st_$w.log 2>&1 || { tail -20 $O/st_$w.log; exit 1; }
  python3 -c "
import csv
rows=list(csv.DictReader(open('$O/st_$w/run_kernel_stats.csv')))
print('$w pin', sorted([(r['Name'].split('(')[0].split('::')[-1], round(float(r['AverageNs'])/1e3,1)) for r in rows if 'witgen_major' in r['Name']]))
"
done
for v in base pin base pin; do
  if [ $v = base ]; then export R0HIP_LIB=risc0_amd/lib/libr0hip_ab_base.so; else unset R0HIP_LIB; fi
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --steps 12 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
