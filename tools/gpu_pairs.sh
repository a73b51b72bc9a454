#!/bin/bash
# Pruned FwFM pair path: FwFM-only tests, then fwfm_pruned with the pair list vs the dense Gram, and fwfm.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02x}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run shallow 600 python -u -m pytest tests/test_gpu_shallow.py tests/test_gpu_parity.py tests/test_boundary.py -x -q --timeout 200 --timeout-method thread || exit 1
for i in 1 2; do
  run fwfm_pruned_pairs_$i 200 python bench.py --config fwfm_pruned --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  run fwfm_pruned_gram_$i 200 python bench.py --config fwfm_pruned --pair-max 0 --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
done
run fwfm 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run fwfm_pruned20 300 python bench.py --config fwfm_pruned --steps 20 --warmup 5 || exit 1
echo done
