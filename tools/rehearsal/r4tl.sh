# kernel timeline of the trace headline at 3 segments in flight (GPU busy / idle gaps)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4tl; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --steps 12 --warmup 3 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
tail -c 300 $O/b.json
