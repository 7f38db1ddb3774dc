# Merkle tree tops: where the single-workgroup top starts (R0_P2_TOP_NODES) and where quads start in
# it (R0_P2_TOP_QUAD_MAX): merkle_fold kernel time per proof (rocprof) and the one-segment latency
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "merkle or fold or golden" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="bench.py --witness --no-cpu-baseline --accum-steps 0 --e2e-steps 0 --inflight 1 --steps 4 --warmup 1"
for v in "512 128" "128 128" "64 64" "512 512"; do
  set -- $v
  R0_P2_TOP_NODES=$1 R0_P2_TOP_QUAD_MAX=$2 R0_P2_TOP_NODES_SEAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s_$1_$2 -o run -- python3 $B > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail -20 $O/b_$1_$2.err; exit 1; }
  python3 -c "
import csv, json
rows=list(csv.DictReader(open('$O/s_$1_$2/run_kernel_stats.csv')))
m=sum(float(r['TotalDurationNs']) for r in rows if 'fold' in r['Name'])/1e6
t=[(r['Name'].split('(')[0].split('::')[-1][:22], r['Calls'], round(float(r['AverageNs'])/1e3,1)) for r in rows if 'fold' in r['Name']]
d=json.load(open('$O/b_$1_$2.json'))
print('top_nodes $1 quad_max $2: fold ms/proof', round(m/7,3), 'ms_per_step', d['ms_per_step'], 'seal', d['config']['seal_sha256_by_rank'][0], t)
"
done
for v in "512 128" "128 128" "512 128" "128 128"; do
  set -- $v
  R0_P2_TOP_NODES=$1 R0_P2_TOP_QUAD_MAX=$2 timeout -k 10 300 python -u bench.py --witness --no-cpu-baseline --accum-steps 0 --steps 3 > $O/e_$1_$2.json 2> $O/e_$1_$2.err || { tail -20 $O/e_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e_$1_$2.json')); print('top $1 quad $2 one-segment', d['end_to_end']['ms_one_segment_unpipelined'], 'e2e', d['end_to_end']['ms_per_step'])"
done
