cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6x; mkdir -p $O
R0HIP_LIB=risc0_amd/lib_variants/libr0hip_f2s.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "merkle_tree_zero or hash_fold or seal_identical or seal_golden" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
LEGS="--no-cpu-baseline --no-prove-only --e2e-steps 0 --accum-steps 0 --resident-steps 0 --per-op-steps 0"
for i in 1 2 3; do
  for v in base f2s f2n; do
    R0HIP_LIB=risc0_amd/lib_variants/libr0hip_$v.so timeout -k 10 300 python -u bench.py $LEGS > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail -20 $O/b_${v}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['config']['seal_sha256_by_rank'], d['config'].get('ms_one_segment_unpipelined'))" $O/b_${v}_$i.json "$v run $i" | tee -a $O/ab.txt
  done
done
