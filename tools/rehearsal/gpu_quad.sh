#!/bin/bash
# Quad-per-node Poseidon2 Merkle layers: parity (hash_fold tests + seal goldens), the
# per-layer latency of one lane vs one quad per node, and the merkle_fold family of one
# proof (single stream, HIP-event timed) with quads off / default.
TAG=${1:-quad}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "hash_fold or golden or eval_check" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 120 env R0_P2_QUAD_MAX=0 python3 -u tools/micro/fold_latency.py > $O/lat_lane.json 2>&1 || { tail -20 $O/lat_lane.json; exit 1; }
timeout -k 10 120 env R0_P2_QUAD_MAX=1000000 python3 -u tools/micro/fold_latency.py > $O/lat_quad.json 2>&1 || { tail -20 $O/lat_quad.json; exit 1; }
cat $O/lat_lane.json $O/lat_quad.json
B="bench.py --no-cpu-baseline --e2e-steps 0 --steps 3 --warmup 1"
timeout -k 10 300 env R0_P2_QUAD_MAX=0 R0_P2_TOP_QUAD_MAX=0 python3 -u $B > $O/bench_off.json 2> $O/bench_off.err || { tail -20 $O/bench_off.err; exit 1; }
timeout -k 10 300 python3 -u $B > $O/bench_on.json 2> $O/bench_on.err || { tail -20 $O/bench_on.err; exit 1; }
grep -h kernel_times_ms $O/bench_off.err $O/bench_on.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline --e2e-steps 0 --inflight 1 > $O/bench_stats.json 2> $O/bench_stats.err || { tail -20 $O/bench_stats.err; exit 1; }
python3 tools/rocprof_families.py $(find $O/stats -name "*kernel_stats.csv") 9 > $O/families.txt && cat $O/families.txt
