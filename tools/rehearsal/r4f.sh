# witgen rework: GPU witgen tests, witgen micro-bench (sort 1 vs 2), kernel stats, default bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 400 --timeout-method thread > $O/pytest_witgen.log 2>&1
rc=$?
tail -15 $O/pytest_witgen.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for s in 1; do
  R0_RVWG_SORT=$s timeout -k 10 300 python -u tools/micro/rv32im_witgen_bench.py 20 5 > $O/witgen_sort$s.json 2> $O/witgen_sort$s.err || { tail -30 $O/witgen_sort$s.err; exit 1; }
  cat $O/witgen_sort$s.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wgstats -o run -- python3 tools/micro/rv32im_witgen_bench.py 20 3 --no-ref > $O/wgstats.log 2>&1 || { tail -20 $O/wgstats.log; exit 1; }
python3 -c "
import csv
rows=list(csv.DictReader(open('$O/wgstats/run_kernel_stats.csv')))
for r in sorted(rows, key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print(r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
timeout -k 10 900 python -u bench.py --e2e-steps 0 --accum-steps 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
