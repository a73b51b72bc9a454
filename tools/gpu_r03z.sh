# Round 3: training step A/B: one-stream graph vs forked graph (inter-step gap)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03z}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-250)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run train_none 300 env DFWFM_TRAIN_FORK=none python tools/bench_train.py --steps 200 --warmup 10 || exit 1
export DFWFM_TRAIN_FORK=none
run prof_none 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profnone -o run --output-format csv -- python3 tools/bench_train.py --steps 50 --warmup 10 || exit 1
echo done
