# The A/B runs that found the slow resident accumulation leg. They used
# temporary bench.py switches (removed with the fix): R0_E2E_LEAK=1 kept the end-to-end
# leg's pinned witness buffers instead of freeing them, R0_ACC_FIRST=1 ran the accumulation
# leg before the end-to-end leg, R0_ACC_FILL=skip dropped the per-proof INVALID fill,
# R0_ACC_STAGGER_MS offset the two prover threads. This run is the after-fix check.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3accv
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 6 --accum-steps 8 > gpurun_out/r3accv/run$i.json 2> gpurun_out/r3accv/run$i.err
  python3 -c "import json; d=json.loads(open('gpurun_out/r3accv/run$i.json').read().strip().splitlines()[-1]); print(d['value'], d['with_accumulation']['ms_per_step'], d['end_to_end']['ms_per_step'])"
done
