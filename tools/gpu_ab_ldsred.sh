#!/bin/bash
# FwFM-only forward: Gram lane sums reduced through LDS (default) vs the 64-lane shuffle chain (libdfwfm_shfl.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02v}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run shallow 400 python -u -m pytest tests/test_gpu_shallow.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread || exit 1
for i in 1 2; do
  DFWFM_LIB=libdfwfm_shfl.so run fwfm_shfl_$i 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  run fwfm_lds_$i 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
done
run fwfm20 200 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run timeline 200 python tools/timeline.py --fwfm --streams 1 || exit 1
echo done
