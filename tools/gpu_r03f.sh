# Round 3: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) vs the CU-masked 4-stream forward
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03f}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run ubench_q16 200 env GPU_MAX_HW_QUEUES=16 ./tools/ubench_m32 || exit 1
run r32_q8 300 env GPU_MAX_HW_QUEUES=8 DFWFM_R32=1 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run r32_q8_20 300 env GPU_MAX_HW_QUEUES=8 DFWFM_R32=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run r32_q8_lohi 300 env GPU_MAX_HW_QUEUES=8 DFWFM_R32=1 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline --cu-mask lo-hi || exit 1
run base_q8 300 env GPU_MAX_HW_QUEUES=8 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run r32_q8_6s 300 env GPU_MAX_HW_QUEUES=8 DFWFM_R32=1 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline --streams 6 || exit 1
echo done
