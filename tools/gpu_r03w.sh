# Round 3: training step host/GPU timing
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03w}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-400)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run train_1 300 python tools/bench_train.py --steps 200 --warmup 10 || exit 1
run prof_train 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proftrain -o run --output-format csv -- python3 tools/bench_train.py --steps 50 --warmup 10 || exit 1
echo done
