# accumulation leg under the default and under 8 hardware queues per process
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/acc7; mkdir -p $O
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 5 > $O/q$q.json 2> $O/q$q.err || { tail -20 $O/q$q.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/q$q.json')); print('queues $q', d['ms_per_step'], d['with_accumulation']['ms_per_step'], d['end_to_end']['ms_per_step'], d['end_to_end']['with_device_accumulation']['ms_per_step'])"
done
