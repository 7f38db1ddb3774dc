cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p24; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "eval_check_full_size" > $O/ec.log 2>&1 || { tail -30 $O/ec.log; exit 1; }
tail -1 $O/ec.log
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline --e2e-steps 0 --po2 24 --steps 2 --warmup 1 > $O/po2_24.json 2> $O/po2_24.err || { tail -20 $O/po2_24.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/po2_24.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
