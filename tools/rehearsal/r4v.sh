# witgen merge kernel: XCD-contiguous row tiles (default) vs plain block order (R0_RVWG_MERGE_XCD=0)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1 0 1 0 1; do
  R0_RVWG_MERGE_XCD=$m timeout -k 10 300 python -u tools/micro/rv32im_witgen_bench.py 20 7 --no-ref > $O/wg_$m.json 2> $O/wg_$m.err || { tail -20 $O/wg_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/wg_$m.json')); print('xcd $m', d['gpu_phase_ms'])"
done
