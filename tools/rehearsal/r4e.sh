# tests for the new paths, the witgen micro-bench (sorted vs atomic buckets), the default bench,
# then a Merkle-top A/B (quads for layers <= 128 vs <= 512)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 400 --timeout-method thread > $O/pytest_witgen.log 2>&1
rc=$?
tail -15 $O/pytest_witgen.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for s in 1 2 0; do
  R0_RVWG_SORT=$s timeout -k 10 300 python -u tools/micro/rv32im_witgen_bench.py 20 5 > $O/witgen_sort$s.json 2> $O/witgen_sort$s.err || { tail -30 $O/witgen_sort$s.err; exit 1; }
  cat $O/witgen_sort$s.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wgstats -o run -- python3 tools/micro/rv32im_witgen_bench.py 20 3 --no-ref > $O/wgstats.log 2>&1 || { tail -20 $O/wgstats.log; exit 1; }
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
for q in 128 512 128 512; do
  R0_P2_TOP_QUAD_MAX=$q timeout -k 10 300 python -u bench.py --witness --no-cpu-baseline --accum-steps 0 --steps 6 > $O/top_$q.json 2> $O/top_$q.err || { tail -30 $O/top_$q.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/top_$q.json')); print('quad_max $q', d['ms_per_step'], d['end_to_end']['ms_one_segment_unpipelined'])"
done
