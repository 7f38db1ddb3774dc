#!/bin/bash
# Summaries of a tools/gpu_round.sh call into profiles/ (run here, after gpurun merged
# gpurun_out/TAG): rocprof families, per-kernel stats, PMC VALU (txt + json), HBM traffic.
set -e
TAG=$1; R=${2:-$TAG}
O=gpurun_out/$TAG
cd "$(dirname "$0")/.."
f() { find $O/$1 -name "$2" | head -1; }
# proofs per profiled run (tools/gpu_round.sh, round-5 bench): stats 18 (3 pipeline warmup + 12 timed
# trace jobs, 1 unpipelined, 2 roofline launches), PMC runs 8 (2 + 3 + 1 + 2); r5c: 11 (6-step
# default); round 4: 10 and 6
NS=${3:-18}; NP=${4:-8}
python3 tools/rocprof_families.py "$(f stats '*kernel_stats.csv')" $NS > profiles/${R}_rocprof_families.txt
cp "$(f stats '*kernel_stats.csv')" profiles/${R}_rocprof_kernel_stats.csv
python3 tools/pmc_summary.py "$(f valu '*counter_collection.csv')" profiles/${R}_pmc_valu.json > profiles/${R}_pmc_valu.txt
python3 tools/pmc_traffic.py "$(f fetch '*counter_collection.csv')" "$(f write '*counter_collection.csv')" $NP > profiles/${R}_pmc_traffic.json
# eval_check's instruction mix on this tree's objects (bench.py's roofline.eval_check_issue)
python3 tools/ec_inst_mix.py rv32im profiles/${R}_pmc_valu.json > profiles/${R}_ec_inst_mix.json
# the library the counters were taken on (bench.py compares it with the one it loads)
[ -f $O/lib_sha256_16 ] && python3 tools/pmc_stamp.py $(cat $O/lib_sha256_16) profiles/${R}_pmc_valu.json profiles/${R}_pmc_traffic.json profiles/${R}_ec_inst_mix.json
cp $O/bench.json profiles/${R}_bench.json
cp $O/pytest_gpu.log profiles/${R}_pytest_gpu.log
head -30 profiles/${R}_rocprof_families.txt
