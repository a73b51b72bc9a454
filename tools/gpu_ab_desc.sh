#!/bin/bash
# MLP-free forward: row descriptors loaded directly (default) vs staged through LDS behind a barrier
# (libdfwfm_stage.so); then the round-end evidence set on the default library.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02y}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run shallow 600 python -u -m pytest tests/test_gpu_shallow.py -x -q --timeout 200 --timeout-method thread || exit 1
for i in 1 2 3; do
  DFWFM_LIB=libdfwfm_stage.so run fwfm_stage_$i 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
  run fwfm_direct_$i 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
done
run timeline 200 python tools/timeline.py --fwfm --streams 1 || exit 1
TAG=${T}e bash tools/gpu_round_end.sh || exit 1
echo done
