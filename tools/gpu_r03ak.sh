# Round 3: sparse pair-walk floor microbenchmark
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench_spwalk > gpurun_out/r03ak_spwalk.log 2>&1; rc=$?; cat gpurun_out/r03ak_spwalk.log; exit $rc
