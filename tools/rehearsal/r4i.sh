# witgen: how much of each arm kernel is its data-group stores (a variant with the unchecked stores dropped)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i; mkdir -p $O
for v in base nostores; do
  L=""; [ $v = nostores ] && L="R0HIP_LIB=$GRAFT_REPO_ROOT/risc0_amd/lib_variants/libr0hip_nostores.so"
  env $L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/micro/rv32im_witgen_bench.py 20 3 --no-ref > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  tail -1 $O/$v.log
  python3 -c "
import csv
rows=list(csv.DictReader(open('$O/$v/run_kernel_stats.csv')))
print('$v', [(r['Name'].split('(')[0].split('::')[-1], round(float(r['AverageNs'])/1e3,1)) for r in sorted(rows, key=lambda r:-float(r['TotalDurationNs']))[:9]])
"
done
