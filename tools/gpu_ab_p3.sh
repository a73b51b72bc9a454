#!/bin/bash
# FwFM-only forward: four-wave PART 3 (trimmed LDS, five workgroups per CU) vs the eight-wave form, by streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02r}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run parity 600 python -u -m pytest tests/test_gpu_shallow.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread || exit 1
for i in 1 2; do
  DFWFM_P3_NG=8 run fwfm_w8_s3_$i 200 python bench.py --config fwfm --streams 3 --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  for S in 3 4 5 6 8; do
    run fwfm_w4_s${S}_$i 200 python bench.py --config fwfm --streams $S --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  done
done
run fwfm20 200 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline || exit 1
echo done
