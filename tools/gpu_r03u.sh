# Round 3: receive-side apply cost at world 1/2/4/8 (lists of distinct batches), standalone
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03v}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-300)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run apply 300 python tools/bench_train.py --steps 20 --warmup 5 --exchange-world1 --apply-worlds 1,2,4,8 || exit 1
echo done
