# Round 3: training-step fork point A/B (tiles / reduce), plus a kernel trace of each
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03af}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c150-215)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
for rep in 1 2; do
  for f in tiles reduce; do
    run train_${f}_$rep 300 env DFWFM_TRAIN_FORK=$f python tools/bench_train.py --steps 500 --warmup 20 || exit 1
  done
done
for f in tiles reduce; do
  export DFWFM_TRAIN_FORK=$f
  run prof_$f 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof$f -o run --output-format csv -- python3 tools/bench_train.py --steps 50 --warmup 10 || exit 1
done
unset DFWFM_TRAIN_FORK
run pytest_split 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q -k "split or fused" --timeout 200 --timeout-method thread || exit 1
echo done
