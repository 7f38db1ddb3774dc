# recursion + Poseidon2 po2=18 (6 in flight): Merkle top at 64 vs 512 nodes, alternating
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4p; mkdir -p $O
for v in 64 512 64 512; do
  R0_P2_TOP_NODES=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --e2e-steps 0 --circuit recursion --po2 18 --steps 24 --warmup 6 > $O/r_$v.json 2> $O/r_$v.err || { tail -20 $O/r_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/r_$v.json')); print('top $v recursion_p2', d['value'], d['ms_per_step'])"
done
for v in 64 512; do
  R0_P2_TOP_NODES=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --e2e-steps 0 --accum-steps 0 --no-prove-only --steps 12 > $O/t_$v.json 2> $O/t_$v.err || { tail -20 $O/t_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/t_$v.json')); print('top $v rv32im trace', d['value'], d['ms_per_step'])"
done
