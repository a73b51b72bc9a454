#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel-trace summary.
# Each step has its own time limit; a crash/abort/timeout (rc >= 124) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ "$rc" -ge 124 ]; then echo "fatal rc=$rc in $name: stopping"; exit "$rc"; fi
  return 0
}
STEPS=${STEPS:-"smoke pytest bench prof"}
for s in $STEPS; do
  case $s in
    smoke)  step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    pytestk) step pytest_k 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${PYTEST_K}" ;;
    bench20) step bench20 300 python bench.py --steps 20 --warmup 5 ;;
    benchfwfm) step benchfwfm 300 python bench.py --config fwfm --steps 400 --warmup 40 --no-cpu-baseline ;;
    benchfwfm20) step benchfwfm20 300 python bench.py --config fwfm --steps 20 --warmup 5 ;;
    benchpruned) step benchpruned 300 python bench.py --config pruned --steps 400 --warmup 40 --no-cpu-baseline ;;
    benchtrain) step benchtrain 300 python tools/bench_train.py ;;
    proffwfm) step proffwfm 400 rocprofv3 --kernel-trace --stats -d gpurun_out/proffwfm_$TAG -o run --output-format csv -- python3 bench.py --config fwfm --no-cpu-baseline --steps 400 --warmup 40 ;;
    proftrain) step proftrain 400 rocprofv3 --kernel-trace --stats -d gpurun_out/proftrain_$TAG -o run --output-format csv -- python3 tools/bench_train.py ;;
    bench)  step bench 400 python bench.py ;;
    bench_fwlw) step bench_fwlw 300 python bench.py --steps 200 --warmup 20 --first-order fwlw --no-cpu-baseline ;;
    prof)   step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline ;;
    prof1)  step prof1 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --streams 1 ;;
    pmc)    step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-graph &&
            step pmc_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-graph ;;
  esac
done
echo "== done"
