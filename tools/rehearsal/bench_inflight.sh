cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in 1 2 3 4; do timeout -k 10 200 python -u bench.py --no-cpu-baseline --inflight $k --steps 8 --warmup 4 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($k, d['value'], d['ms_per_step'])" || exit 1; done
