# pinned-source uploads: the tests that upload from host memory, then the default bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rv32im_witgen_gpu.py tests/test_gpu_parity.py -m gpu -q -k "trace or pinned or host or segments or upload" --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit 1; }
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], d['ms_per_step'], 'prove_only', d['prove_only']['ms_per_step'], 'seal_equal', (d['cpu_baseline'] or {}).get('seal_equal'))
print('e2e', d['end_to_end']['ms_per_step'], d['end_to_end']['ms_one_segment_unpipelined'])
print('e2e_trace', d['end_to_end_from_trace'])"
