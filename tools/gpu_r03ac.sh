# Round 3: dw2_kernel (b128 fragments, 16 MFMAs per two LDS reads): training tests, A/B vs dw_kernel, fork variants
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03ac}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-250)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run pytest_train 600 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
run train_dw2 300 python tools/bench_train.py --steps 200 --warmup 10 || exit 1
run train_dw1 300 env DFWFM_DW=1 python tools/bench_train.py --steps 200 --warmup 10 || exit 1
run train_dw2_none 300 env DFWFM_TRAIN_FORK=none python tools/bench_train.py --steps 200 --warmup 10 || exit 1
run prof_dw2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 tools/bench_train.py --steps 50 --warmup 10 || exit 1
echo done
