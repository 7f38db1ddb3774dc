# device-accumulation paths: parity tests, then a bench line with both accumulation legs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/acc5; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread -k "accum or pipeline or segments" > $O/p.log 2>&1 || { tail -30 $O/p.log; exit 1; }
tail -1 $O/p.log
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
