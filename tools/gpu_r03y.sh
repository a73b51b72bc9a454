# Round 3: training step A/B: fork point (after the per-tile backward / after the scatter), bounded-grid Adam
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03y}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-250)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run pytest_adam 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q -k "adam or fused or split" --timeout 200 --timeout-method thread || exit 1
run train_tiles 300 python tools/bench_train.py --steps 200 --warmup 10 || exit 1
run train_spread 300 env DFWFM_TRAIN_FORK=spread python tools/bench_train.py --steps 200 --warmup 10 || exit 1
run prof_tiles 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proftiles -o run --output-format csv -- python3 tools/bench_train.py --steps 50 --warmup 10 || exit 1
export DFWFM_TRAIN_FORK=spread
run prof_spread 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profspread -o run --output-format csv -- python3 tools/bench_train.py --steps 50 --warmup 10 || exit 1
echo done
