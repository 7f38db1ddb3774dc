# witgen: far uses of injected loads reload the cell (R0_RVWG_REMAT) — base (no reloads),
# v1 (SHA-256 arm 11, window 400 lines), v2 (arms 9, 10, 11): per-arm kernel times
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base v1 v2 base v1 v2; do
  if [ $v = v2 ]; then unset R0HIP_LIB; else export R0HIP_LIB=risc0_amd/lib/libr0hip_ab_$v.so; fi
  for w in loop ec; do
    if [ $w = loop ]; then cmd="tools/micro/rv32im_witgen_bench.py 20 3 --no-ref"; else cmd="tools/micro/rv32im_witgen_ecall_bench.py 18 120 3"; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_${w}_$v -o run -- python3 $cmd > $O/st_${w}_$v.log 2>&1 || { tail -20 $O/st_${w}_$v.log; exit 1; }
    python3 -c "
import csv
rows=list(csv.DictReader(open('$O/st_${w}_$v/run_kernel_stats.csv')))
d={r['Name'].split('(')[0].split('_')[-1]: round(float(r['AverageNs'])/1e3,1) for r in rows if 'witgen_major' in r['Name']}
print('$w $v', {k: d[k] for k in ('4','9','10','11','12') if k in d}, 'sum', round(sum(d.values()),1))
"
  done
done
