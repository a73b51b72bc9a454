# Round-3 end check of the final tree: smoke, every GPU test, the driver's bench command (+ rocprofv3 summary), FwFM-only
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03bo}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-240)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run bench20 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
run prof_bench20 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run bench2000 300 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run fwfm20 300 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run fwfm2000 300 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
echo done
