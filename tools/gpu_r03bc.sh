# Batch-set evidence: smoke, every GPU test, the driver's bench command + its rocprofv3 summary, 20- and 2000-step
# deep / FwFM-only / QR / pruned configs, PMC passes of the default batch sets
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03bc}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run bench20 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
run prof_bench20 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run bench2000 300 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run fwfm20 300 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run fwfm2000 300 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run qr20 300 python bench.py --config qr --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run pruned20 300 python bench.py --config pruned --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run prof_fwfm20 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proff -o run --output-format csv -- python3 bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run fwfm20s8 300 python bench.py --config fwfm --steps 20 --warmup 5 --table-scale 8 --no-cpu-baseline || exit 1
run fwfm2000s8 300 python bench.py --config fwfm --steps 2000 --warmup 400 --table-scale 8 --no-cpu-baseline || exit 1
TAG=${T}pmc BENCH_ARGS="" bash tools/pmc.sh || exit 1
TAG=${T}pmcf BENCH_ARGS="--config fwfm" bash tools/pmc.sh || exit 1
TAG=${T}pmcf8 BENCH_ARGS="--config fwfm --table-scale 8" bash tools/pmc.sh || exit 1
echo done
