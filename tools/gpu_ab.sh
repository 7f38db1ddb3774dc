#!/bin/bash
# Same-box A/B of an environment toggle on the default bench workload (legs other than the
# headline off): gpu_ab.sh TAG VAR VALUE_A VALUE_B [ROUNDS]. Writes gpurun_out/TAG/ab.txt.
# EXTRA (environment): more bench.py arguments, e.g. EXTRA="--hashfn sha-256"
TAG=$1; VAR=$2; A=$3; B=$4; N=${5:-2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
LEGS="$EXTRA --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 --per-op-steps 0"
for i in $(seq 1 $N); do
  for v in $A $B; do
    t=$(basename "$v")
    env $VAR=$v timeout -k 10 300 python -u bench.py $LEGS > $O/bench${SUF}_${VAR}_${t}_$i.json 2> $O/bench${SUF}_${VAR}_${t}_$i.err || { tail -20 $O/bench${SUF}_${VAR}_${t}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['config'].get('ms_one_segment_unpipelined'))" $O/bench${SUF}_${VAR}_${t}_$i.json "$SUF $VAR=$t run $i" | tee -a $O/ab.txt
  done
done
