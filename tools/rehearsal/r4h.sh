# witgen PMC passes on the micro-bench (issue mix per arm kernel), then the full round profile
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h; mkdir -p $O
W="tools/micro/rv32im_witgen_bench.py 20 2 --no-ref"
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/valu -o run -- python3 $W > $O/valu.log 2>&1 || { tail -20 $O/valu.log; exit 1; }
python3 tools/pmc_summary.py "$(find $O/valu -name '*counter_collection.csv' | head -1)" | head -16
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES --output-format csv -d $O/mix -o run -- python3 $W > $O/mix.log 2>&1 || { tail -20 $O/mix.log; echo mix pass failed; }
python3 - <<'PY'
import csv, collections, glob, re
fs = glob.glob("gpurun_out/r4h/mix/**/*counter_collection.csv", recursive=True)
if fs:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(fs[0])):
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", ""))[-28:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAIT_INST_LDS", 0))[:12]:
        w = max(c.get("SQ_WAVES", 1), 1)
        print(k.ljust(28), {n.replace("SQ_", ""): round(v / w, 1) for n, v in sorted(c.items()) if n != "SQ_WAVES"})
PY
bash tools/gpu_round.sh r4g
