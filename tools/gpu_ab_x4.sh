#!/bin/bash
# Gather rows as aligned dwordx4 + dwordx2 (default) vs five dwordx2 (libdfwfm_x2.so): parity, FwFM-only and deep.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02w}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run parity 600 python -u -m pytest tests/test_gpu_shallow.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread || exit 1
for i in 1 2; do
  DFWFM_LIB=libdfwfm_x2.so run fwfm_x2_$i 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  run fwfm_x4_$i 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  DFWFM_LIB=libdfwfm_x2.so run deep_x2_$i 200 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  run deep_x4_$i 200 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
done
run deep20_x4 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run timeline 200 python tools/timeline.py --fwfm --streams 1 || exit 1
echo done
