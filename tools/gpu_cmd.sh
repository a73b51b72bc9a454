set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -5 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="$(printf "X=0 2\nDFWFM_PRIO=1 2\nDFWFM_PRIO=1 3\nDFWFM_NO_STATIC_K=1 2")" ./tools/ab_real.sh > gpurun_out/ab.log 2>&1
DFWFM_PRIO=1 timeout -k 10 120 python tools/timeline.py --streams 2 > gpurun_out/tl.log 2>&1
timeout -k 10 200 python tools/bench_train.py > gpurun_out/train.log 2>&1
