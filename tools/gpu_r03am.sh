# Fresh-container rebuild check: smoke, every GPU test, the driver's bench command, the training step
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03am}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run bench20 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run train 300 python tools/bench_train.py --steps 500 --warmup 20 || exit 1
echo done
