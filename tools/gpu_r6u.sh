cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_per_op_path.py -m gpu -q -x --timeout 400 --timeout-method thread -k "gather or per_op" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 --steps 6 > $O/bench_perop.json 2> $O/bench_perop.err || { tail -20 $O/bench_perop.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_perop.json')); print(json.dumps(d['per_op_abi']))"
