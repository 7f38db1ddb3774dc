# witgen bucket order A/B: cycle order vs minor-then-cycle order within a bin (compact stores)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rv32im_witgen_gpu.py -m gpu -q -k "matches_reference or ecalls" --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
R0_RVWG_MINOR=1 timeout -k 10 600 python -u -m pytest tests/test_rv32im_witgen_gpu.py -m gpu -q -k "matches_reference or ecalls" --timeout 400 --timeout-method thread > $O/pytest_minor.log 2>&1 || { tail -30 $O/pytest_minor.log; exit 1; }
tail -1 $O/pytest_minor.log
for m in 0 1 0 1; do
  R0_RVWG_MINOR=$m timeout -k 10 300 python -u tools/micro/rv32im_witgen_bench.py 20 5 --no-ref > $O/wg_$m.json 2> $O/wg_$m.err || { tail -20 $O/wg_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/wg_$m.json')); print('minor $m', d['gpu_phase_ms'])"
done
R0_RVWG_MINOR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats1 -o run -- python3 tools/micro/rv32im_witgen_bench.py 20 3 --no-ref > $O/stats1.log 2>&1 || exit 1
python3 -c "
import csv
rows=list(csv.DictReader(open('$O/stats1/run_kernel_stats.csv')))
print([(r['Name'].split('(')[0].split('::')[-1], round(float(r['AverageNs'])/1e3,1)) for r in sorted(rows, key=lambda r:-float(r['TotalDurationNs']))[:10]])
"
