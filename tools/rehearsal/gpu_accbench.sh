#!/bin/bash
# rv32im accumulation timing at po2=20 (HIP events) and a kernel-trace profile
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-accbench}; mkdir -p $O
timeout -k 10 300 python3 -u tools/micro/accum_bench.py 20 > $O/t.json 2> $O/t.err || { tail -20 $O/t.err; exit 1; }
cat $O/t.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 tools/micro/accum_bench.py 20 > /dev/null 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/stats/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    if "rv_accum" in r["Name"] or "scan" in r["Name"] or "finalize" in r["Name"] or "tile" in r["Name"]:
        print(f'{r["Name"][:60]:60s} {float(r["AverageNs"])/1e3:9.1f} us x{r["Calls"]}')
PY
