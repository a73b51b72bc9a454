# Round 3, first call: every GPU test (new: full-size QR / training parity, RCCL world-1 exchange, strict FwFM-only
# bar), the self-launching N=2 bench and training bench (gloo, both ranks on the one GPU), the driver's bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03a}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run pytest_new 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "full_size or rccl or capacity or shallow or train_step_matches_reference" || exit 1
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
run bench_n2 300 env DFWFM_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 400 --warmup 100 || exit 1
run train_n2 300 env DFWFM_BENCH_BACKEND=gloo python tools/bench_train.py --gpus 2 --steps 20 --warmup 5 || exit 1
run bench20 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
echo done
