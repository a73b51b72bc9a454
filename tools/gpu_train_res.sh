#!/bin/bash
# Training step: resident-input graph sets vs copied inputs; the training GPU tests; kernel summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02t}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-220)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run train_tests 900 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread || exit 1
for i in 1 2; do
  run train_copy_$i 300 python tools/bench_train.py --copy-inputs || exit 1
  run train_res_$i 300 python tools/bench_train.py || exit 1
done
run train_res_200 300 python tools/bench_train.py --steps 200 --warmup 20 || exit 1
run prof_train 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proftrain -o run --output-format csv -- python3 tools/bench_train.py || exit 1
echo done
