#!/bin/bash
# MLP-free forward with direct descriptors: eight waves (default) vs four (DFWFM_P3_NG=4) by streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02za}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
for i in 1 2; do
  run w8_s3_$i 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  for S in 3 5 6; do
    DFWFM_P3_NG=4 run w4_s${S}_$i 200 python bench.py --config fwfm --streams $S --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  done
  run w8_s4_$i 200 python bench.py --config fwfm --streams 4 --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
done
echo done
