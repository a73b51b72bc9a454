# criterion fused into the training forward: every GPU test, training step, kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03ay}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run pytest_train 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread || exit 1
run train 300 python tools/bench_train.py --steps 500 --warmup 20 || exit 1
run train_b 300 python tools/bench_train.py --steps 500 --warmup 20 || exit 1
run prof_train 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 tools/bench_train.py --steps 100 --warmup 10 || exit 1
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
echo done
