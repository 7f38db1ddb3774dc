cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 400 --timeout-method thread > $O/pytest_witgen.log 2>&1
rc=$?
tail -15 $O/pytest_witgen.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
