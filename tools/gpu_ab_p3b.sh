#!/bin/bash
# Round-2 FwFM-only A/B (trimmed LDS + U' from global, eight waves; 4 workgroups per CU variant), the training
# step with the gradient zeroing on a side stream, their tests, and the FwFM-only kernel's PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02s}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run shallow 400 python -u -m pytest tests/test_gpu_shallow.py -x -q --timeout 200 --timeout-method thread || exit 1
run train_tests 900 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread || exit 1
run train 300 python tools/bench_train.py || exit 1
for i in 1 2; do
  run fwfm_s3_$i 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  DFWFM_LIB=libdfwfm_p3w8.so run fwfm_wpe8_s4_$i 200 python bench.py --config fwfm --streams 4 --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  DFWFM_LIB=libdfwfm_p3w8.so run fwfm_wpe8_s3_$i 200 python bench.py --config fwfm --streams 3 --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
done
TAG=${T}fwfm PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" BENCH_ARGS="--config fwfm" bash tools/pmc.sh || exit 1
echo done
