cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "merkle_tree_zero or seal_identical or seal_golden or hash_rows or hash_fold or full_size_seal or streamed" > $O/pytest_zero.log 2>&1 || { tail -30 $O/pytest_zero.log; exit 1; }
tail -1 $O/pytest_zero.log
EXTRA="--hashfn sha-256" SUF=_sha bash tools/gpu_ab.sh r6p R0_P2_ZERO 0 1 2 && SUF=_p2 bash tools/gpu_ab.sh r6p R0_P2_ZERO 0 1 1
