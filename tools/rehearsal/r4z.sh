# the first-failure parity test per arm, then the whole witgen GPU file
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 300 --timeout-method thread -k first_failure > $O/pytest_ff.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" $O/pytest_ff.log | head -30; tail -2 $O/pytest_ff.log; [ $rc -eq 0 ] || exit $rc
