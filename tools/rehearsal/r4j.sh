# segments in flight for the trace headline (A/B on one box), then the round profile
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4j; mkdir -p $O
for k in 3 4 3 4 2; do
  timeout -k 10 300 python -u bench.py --inflight $k --steps 12 --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 > $O/inflight_$k.json 2> $O/inflight_$k.err || { tail -20 $O/inflight_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/inflight_$k.json')); print('inflight $k', d['value'], d['ms_per_step'])" | tee -a $O/inflight.txt
done
bash tools/gpu_round.sh r4j
