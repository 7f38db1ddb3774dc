#!/bin/bash
# default bench line (with the end-to-end leg) + recursion/poseidon_254 queue-depth sweep
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/e2e; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
for k in 2 4; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-steps 0 --circuit recursion --hashfn poseidon_254 --po2 18 --steps 8 --warmup 2 --inflight $k > $O/rec_p254_k$k.json 2> $O/rec_p254_k$k.err || { tail -20 $O/rec_p254_k$k.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/rec_p254_k$k.json')); print($k, d['value'], d['ms_per_step'])"
done
