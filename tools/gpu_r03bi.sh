# Round-3 end evidence on the final code: smoke, every GPU test, the driver's bench command + its rocprofv3 summary,
# 2000-step deep / FwFM-only, QR / pruned, the training step (+ summary), the N = 2 rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03bi}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-220)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run bench20 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
run prof_bench20 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run bench2000 300 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run fwfm20 300 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run fwfm2000 300 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run qr2000 300 python bench.py --config qr --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run pruned2000 300 python bench.py --config pruned --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run train 300 python tools/bench_train.py --steps 500 --warmup 20 || exit 1
run prof_train 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proftrain -o run --output-format csv -- python3 tools/bench_train.py --steps 100 --warmup 10 || exit 1
DFWFM_BENCH_BACKEND=gloo run bench_n2 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
echo done
