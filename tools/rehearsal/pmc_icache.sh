#!/bin/bash
# instruction-cache behaviour of the generated eval_check kernels (one PMC pass)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/icache
timeout -s KILL 60 rocprofv3 -L > gpurun_out/icache/avail.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU --output-format csv -d gpurun_out/icache/pmc -o run -- python3 tools/bench_kernels.py ec > gpurun_out/icache/run.log 2>&1
echo rc=$?
