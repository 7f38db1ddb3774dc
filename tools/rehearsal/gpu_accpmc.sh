#!/bin/bash
# VALU issue counters of the rv32im accumulation kernels (tools/micro/accum_bench.py, po2=20)
# for each library variant given (default: the in-tree build)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-accpmc}; shift; mkdir -p $O
libs="${@:-risc0_amd/lib/libr0hip.so}"
for f in $libs; do
  n=$(basename $f .so)
  R0HIP_LIB=$PWD/$f timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/$n -o run -- python3 tools/micro/accum_bench.py 20 > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "== $n"
  python3 tools/pmc_summary.py $(ls $O/$n/*counter_collection.csv | head -1) | grep -E "kernel|rv_accum|finalize"
done
