# witgen merge: rank-grouped gathers through LDS (merge_tile_kernel<256|512|1024>) vs
# merge_kernel (R0_RVWG_MERGE_TILE=0): GPU witgen tests (default 1024), standalone phase times
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in 0 256 512 1024 0 256 512 1024; do
  R0_RVWG_MERGE_TILE=$m timeout -k 10 300 python -u tools/micro/rv32im_witgen_bench.py 20 7 --no-ref > $O/wg_$m.json 2> $O/wg_$m.err || { tail -20 $O/wg_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/wg_$m.json')); print('tile $m', d['gpu_phase_ms'])"
done
