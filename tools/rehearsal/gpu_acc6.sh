cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/acc6; mkdir -p $O
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --e2e-steps 0 --steps 5 > $O/a.json 2> $O/a.err || { tail -20 $O/a.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/a.json')); print(d['ms_per_step'], d['with_accumulation'])"
grep with_accumulation_proofs $O/a.err
grep phases_ms $O/a.err
