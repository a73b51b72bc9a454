#!/bin/bash
# Split-gather A/B: gather microbenchmark, forward parity tests on the new library, then FwFM-only and DeepFwFM
# benches alternating libdfwfm_sg0.so (one lane per row) and libdfwfm.so (split gather).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02q}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run ubench1 60 tools/ubench_gather 1 || exit 1
run ubench3 60 tools/ubench_gather 3 || exit 1
run ubench8 60 tools/ubench_gather 8 || exit 1
run parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shallow.py -x -q --timeout 200 --timeout-method thread || exit 1
for i in 1 2; do
  DFWFM_LIB=libdfwfm_sg0.so run fwfm_sg0_$i 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  run fwfm_sg1_$i 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  DFWFM_LIB=libdfwfm_sg0.so run deep_sg0_$i 200 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  run deep_sg1_$i 200 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
done
echo done
