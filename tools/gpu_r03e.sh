# Round 3: the 32-sample forward (fwd32_kernel) -- bit-identity / golden tests, then the bench with and without it
# (CU-masked stream pairs), and the masked-stream microbenchmark.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03e}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-240)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run pytest_r32 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fwd32" || exit 1
run ubench 200 ./tools/ubench_m32 || exit 1
run bench_base 300 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run bench_r32_eo 300 env DFWFM_R32=1 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run bench_r32_lohi 300 env DFWFM_R32=1 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline --cu-mask lo-hi || exit 1
run bench_r32_nomask 300 env DFWFM_R32=1 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline --cu-mask none || exit 1
run bench_r32_2s 300 env DFWFM_R32=1 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline --cu-mask none --streams 2 || exit 1
run bench_r32_20 300 env DFWFM_R32=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
echo done
