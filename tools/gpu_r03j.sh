# Round 3: HBM-resident tables (--table-scale 8: 424 MB of rows, past the 256 MB Infinity Cache) and PMC traffic of
# the exact kernels the bench lines name, over the bench's own command
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03j}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run fwfm_s1 300 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run fwfm_s8 300 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline --table-scale 8 || exit 1
run fwfm_s1_20 300 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run deep_s8 300 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline --table-scale 8 || exit 1
TAG=${T}a BENCH_ARGS="" bash tools/pmc.sh > gpurun_out/${T}_pmc_deep.log 2>&1 || { cat gpurun_out/${T}_pmc_deep.log; exit 1; }
TAG=${T}b BENCH_ARGS="--config fwfm" bash tools/pmc.sh > gpurun_out/${T}_pmc_fwfm.log 2>&1 || { cat gpurun_out/${T}_pmc_fwfm.log; exit 1; }
TAG=${T}c BENCH_ARGS="--config fwfm --table-scale 8" bash tools/pmc.sh > gpurun_out/${T}_pmc_fwfm8.log 2>&1 || { cat gpurun_out/${T}_pmc_fwfm8.log; exit 1; }
TAG=${T}d BENCH_ARGS="--table-scale 8" bash tools/pmc.sh > gpurun_out/${T}_pmc_deep8.log 2>&1 || { cat gpurun_out/${T}_pmc_deep8.log; exit 1; }
TAG=${T}e BENCH_ARGS="--config fwfm" PMC_GROUPS="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" bash tools/pmc.sh > gpurun_out/${T}_pmc_fwfm_req.log 2>&1 || { cat gpurun_out/${T}_pmc_fwfm_req.log; exit 1; }
echo done
