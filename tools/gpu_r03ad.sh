# Round 3: weight-gradient GEMM batch splits (workgroups beside the main stream's reductions / scatter / Adam)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03ad}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c150-215)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
for sp in 2 3 4 5 6 7; do
  run train_s$sp 300 env DFWFM_DW_SPLITS=$sp python tools/bench_train.py --steps 300 --warmup 10 || exit 1
done
run train_default 300 python tools/bench_train.py --steps 300 --warmup 10 || exit 1
run train_spread 300 env DFWFM_TRAIN_FORK=spread python tools/bench_train.py --steps 300 --warmup 10 || exit 1
echo done
