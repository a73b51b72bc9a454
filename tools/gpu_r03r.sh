# Round 3: RCCL collectives captured into the DP step graph: the RCCL tests, then the step timing
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03s}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-220)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run pytest_rccl 400 python -u -m pytest tests/test_gpu_train.py -m gpu -x -v -k "rccl" --timeout 300 --timeout-method thread || exit 1
run train_x1 300 python tools/bench_train.py --steps 100 --warmup 10 --exchange-world1 || exit 1
run prof_train_x1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proftrainx -o run --output-format csv -- python3 tools/bench_train.py --steps 50 --warmup 10 --exchange-world1 || exit 1
run pytest_train 600 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
echo done
