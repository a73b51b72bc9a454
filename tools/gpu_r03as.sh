# training step: fork placement with the register-direct GEMM
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03as}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c150-215)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
for f in tiles none spread; do
  run fork_$f 300 env DFWFM_TRAIN_FORK=$f python tools/bench_train.py --steps 500 --warmup 20 || exit 1
done
run fork_none_s6 300 env DFWFM_TRAIN_FORK=none DFWFM_DW_SPLITS=6 python tools/bench_train.py --steps 500 --warmup 20 || exit 1
run fork_tiles2 300 env DFWFM_TRAIN_FORK=tiles python tools/bench_train.py --steps 500 --warmup 20 || exit 1
echo done
