# Round 3: fwd32 one workgroup per CU by LDS reservation (plain streams) vs CU-masked stream pairs
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03g}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run pad2 300 env DFWFM_R32=1 DFWFM_R32_LDS=90000 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline --cu-mask none --streams 2 || exit 1
run pad2_20 300 env DFWFM_R32=1 DFWFM_R32_LDS=90000 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --cu-mask none --streams 2 || exit 1
run pad3 300 env DFWFM_R32=1 DFWFM_R32_LDS=90000 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline --cu-mask none --streams 3 || exit 1
run mask4_20b 300 env DFWFM_R32=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run base_20 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
echo done
