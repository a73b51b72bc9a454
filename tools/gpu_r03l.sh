# Round 3: fwd32 with both halves' FwFM chains interleaved: stamps, bit-identity tests, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03l}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run pytest_r32 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fwd32" || exit 1
run stamps 200 env DFWFM_DIAG_STAMPS=1 DFWFM_R32=1 python tools/phase_stamps.py --iters 30 || exit 1
run bench2000 300 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run bench20 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
grep -v "^W20\|^E20\|amdgpu" gpurun_out/${T}_stamps.log
