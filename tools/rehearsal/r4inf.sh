# trace headline: 3 vs 4 segments in flight (po2 20), alternating, 12 timed steps each
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4inf; mkdir -p $O
for k in 3 4 3 4; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --steps 12 --inflight $k > $O/b_$k.json 2> $O/b_$k.err || { tail -20 $O/b_$k.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$k.json').read().strip().splitlines()[-1]); print('inflight $k', d['value'], d['ms_per_step'])"
done
