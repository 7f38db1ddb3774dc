# accumulation-step variants (risc0_amd/lib/var/lib_<limit>_<inv batch>.so, built here with
# make ACC_LIMIT=.. ACC_INV_BATCH=..): po2=20 step time of each
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for f in risc0_amd/lib/var/*.so; do echo "$f"; R0HIP_LIB=$PWD/$f timeout -k 10 120 python3 -u tools/micro/accum_bench.py 20 || exit 1; done
