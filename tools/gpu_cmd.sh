set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -5 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
STAMPS=1 VARIANTS="$(printf "X=0 2\nX=0 3\nDFWFM_DIAG_DROP_FLAGS=1 2")" ./tools/ab_real.sh > gpurun_out/ab3.log 2>&1
