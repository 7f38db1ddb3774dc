# per-kernel stats of the previous header (base) for the r4s A/B, same commands as r4s.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4s2; mkdir -p $O
for v in base note; do
for w in loop ec; do
  if [ $v = base ]; then export R0HIP_LIB=risc0_amd/lib/libr0hip_ab_base.so; else unset R0HIP_LIB; fi
  if [ $w = loop ]; then cmd="tools/micro/rv32im_witgen_bench.py 20 3 --no-ref"; else cmd="tools/micro/rv32im_witgen_ecall_bench.py 18 120 3"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_${w}_$v -o run -- python3 $cmd > $O/st_${w}_$v.log 2>&1 || { tail -20 $O/st_${w}_$v.log; exit 1; }
  python3 -c "
import csv
rows=list(csv.DictReader(open('$O/st_${w}_$v/run_kernel_stats.csv')))
print('$w $v', sorted([(r['Name'].split('(')[0].split('::')[-1], round(float(r['AverageNs'])/1e3,1)) for r in rows if 'witgen_major' in r['Name']]))
"
done
done
