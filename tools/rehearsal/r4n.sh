# Merkle dataflow tree fold (R0_P2_TREE=1, default) vs per-layer launches + one-workgroup top
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_rv32im_witgen_gpu.py -m gpu -q -k "merkle or fold or golden or seal or prove" --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="bench.py --witness --no-cpu-baseline --accum-steps 0 --e2e-steps 0 --inflight 1 --steps 4 --warmup 1"
for v in 1 0; do
  R0_P2_TREE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s_$v -o run -- python3 $B > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  python3 -c "
import csv, json
rows=list(csv.DictReader(open('$O/s_$v/run_kernel_stats.csv')))
m=sum(float(r['TotalDurationNs']) for r in rows if 'fold' in r['Name'])/1e6
t=[(r['Name'].split('(')[0].split('::')[-1][:22], r['Calls'], round(float(r['AverageNs'])/1e3,1)) for r in rows if 'fold' in r['Name']]
d=json.load(open('$O/b_$v.json'))
print('tree $v: fold ms/proof', round(m/7,3), 'ms_per_step', d['ms_per_step'], 'seal', d['config']['seal_sha256_by_rank'][0], t)
"
done
for v in 1 0 1 0; do
  R0_P2_TREE=$v timeout -k 10 300 python -u bench.py --witness --no-cpu-baseline --accum-steps 0 --steps 3 > $O/e_$v.json 2> $O/e_$v.err || { tail -20 $O/e_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e_$v.json')); print('tree $v one-segment', d['end_to_end']['ms_one_segment_unpipelined'], 'e2e', d['end_to_end']['ms_per_step'], 'prove', d['ms_per_step'])"
done
