# Fresh-build check + register-direct weight-gradient GEMM (dwr_kernel) vs the LDS-staged dw_kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03an}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-220)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run train_new 300 python tools/bench_train.py --steps 300 --warmup 20 || exit 1
run train_staged 300 env DFWFM_DW_STAGED=1 python tools/bench_train.py --steps 300 --warmup 20 || exit 1
for sp in 4 10 14; do
  run train_s$sp 300 env DFWFM_DW_SPLITS=$sp python tools/bench_train.py --steps 300 --warmup 20 || exit 1
done
run prof_train 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proftrain -o run --output-format csv -- python3 tools/bench_train.py --steps 100 --warmup 10 || exit 1
run prof_train_staged 300 env DFWFM_DW_STAGED=1 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proftrain_staged -o run --output-format csv -- python3 tools/bench_train.py --steps 100 --warmup 10 --mode fused || exit 1
run bench20 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
echo done
