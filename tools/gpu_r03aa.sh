# Round 3: GEMM + main Adam in one launch (one-stream step graph): tests + step timing (A/B vs the forks)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03aa}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-250)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run pytest_new 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q -k "weights_adam or fused or split or adam" --timeout 200 --timeout-method thread || exit 1
run train_fused 300 python tools/bench_train.py --steps 200 --warmup 10 || exit 1
run train_tiles 300 env DFWFM_TRAIN_FORK=tiles python tools/bench_train.py --steps 200 --warmup 10 || exit 1
run prof_fused 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proffused -o run --output-format csv -- python3 tools/bench_train.py --steps 50 --warmup 10 || exit 1
run pytest_train 600 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
echo done
