#!/bin/bash
# End-of-round GPU session: smoke, GPU tests, default bench, rocprofv3 kernel stats (bench command,
# one stream), training bench + its kernel stats.  Each step time-limited; stops at the first failure.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-final} STEPS="smoke pytest bench prof prof1" bash tools/gpu_check.sh || exit 1
grep -q "rc=0" gpurun_out/pytest_gpu.log 2>/dev/null; 
timeout -k 10 200 python tools/bench_train.py --steps 200 > gpurun_out/bench_train.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_${TAG:-final} -o run --output-format csv -- python3 tools/bench_train.py --steps 30 > gpurun_out/prof_train.log 2>&1 || exit 1
echo session done
