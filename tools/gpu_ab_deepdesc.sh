#!/bin/bash
# Fused forward / training forward without QR: direct row descriptors (default) vs staged (libdfwfm_deepstage.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02zc}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
for i in 1 2; do
  DFWFM_LIB=libdfwfm_deepstage.so run deep_stage_$i 200 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  run deep_direct_$i 200 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  DFWFM_LIB=libdfwfm_deepstage.so run train_stage_$i 200 python tools/bench_train.py || exit 1
  run train_direct_$i 200 python tools/bench_train.py || exit 1
done
run bench20 200 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
echo done
