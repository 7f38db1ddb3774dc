cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -20 $O/pytest.log; exit $rc
