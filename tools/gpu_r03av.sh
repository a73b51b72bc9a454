# fwd32 per-CU K-loop token with an early hand-over (A/B, DFWFM_CU_TOKEN=1+chunks before the K loop's end)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03av}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_$name.log) $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-120)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run base 300 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
for r in 1 3 6 10; do
  run tok$r 300 env DFWFM_CU_TOKEN=$r python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
done
run base2 300 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
echo done
