cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -20 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ec -o run -- python3 tools/micro/rv32im_witgen_ecall_bench.py 18 120 3 > $O/ec.log 2>&1 || { tail -20 $O/ec.log; exit 1; }
grep '^{' $O/ec.log
python3 -c "
import csv
rows=list(csv.DictReader(open('$O/ec/run_kernel_stats.csv')))
print([(r['Name'].split('(')[0].split('::')[-1], r['Calls'], round(float(r['AverageNs'])/1e3,1)) for r in sorted(rows, key=lambda r:-float(r['TotalDurationNs']))[:12]])
"
