# compiler scheduling strategies for the generated kernels (risc0_amd/lib/var/lib_<strategy>.so,
# built here with make EC_FLAGS="-mllvm -amdgpu-sched-strategy=<s>"): bench value, eval_check
# kernel time, accumulation step, each library in its own process
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sched; mkdir -p $O
for f in risc0_amd/lib/var/*.so; do
  n=$(basename $f .so)
  R0HIP_LIB=$PWD/$f timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --e2e-steps 0 --steps 8 --warmup 2 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  R0HIP_LIB=$PWD/$f timeout -k 10 120 python3 -u tools/micro/accum_bench.py 20 > $O/$n.acc || exit 1
  python3 - "$O/$n" <<'PY'
import json, sys
b = sys.argv[1]
d = json.load(open(b + ".json"))
kt = [json.loads(l) for l in open(b + ".err") if l.startswith('{"kernel_times_ms"')][0]["kernel_times_ms"]
acc = json.loads(open(b + ".acc").read())["ms"]
print(b.split("/")[-1], d["value"], d["ms_per_step"], "eval_check", kt.get("eval_check"),
      "with_acc", d.get("with_accumulation", {}).get("ms_per_step"), "accum_step", [v["accum_step"] for v in acc.values()])
PY
done
