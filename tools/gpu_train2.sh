set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dw or weight or golden or step" > gpurun_out/tt.log 2>&1; rc=$?; tail -2 gpurun_out/tt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proftrain -o run --output-format csv -- python3 tools/bench_train.py > gpurun_out/pt.log 2>&1 || exit 1
grep -E "dw_kernel|bwd_kernel|adam_dev" gpurun_out/proftrain/run_kernel_stats.csv | cut -c1-120
timeout -k 10 200 python tools/bench_train.py > gpurun_out/bt.log 2>&1 || exit 1; echo "$(tail -1 gpurun_out/bt.log | cut -c1-200)"
