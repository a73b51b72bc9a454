# Round 3: sparse deep tower with LDS-staged ELL entries: parity tests, bench, kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03ai}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run pytest_sparse 300 python -u -m pytest tests/test_gpu_sparse.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run bench_sparse 300 python bench.py --config pruned --sparse-mlp 0.25 --steps 400 --warmup 20 --no-cpu-baseline || exit 1
grep -o '"ms_per_step[^,]*' gpurun_out/${T}_bench_sparse.log
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --config pruned --sparse-mlp 0.25 --steps 100 --warmup 10 --no-cpu-baseline || exit 1
echo done
