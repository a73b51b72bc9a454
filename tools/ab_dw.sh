#!/bin/bash
# A/B of two library builds on the training step (scratch).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; tail -5 gpurun_out/par.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 200 python tools/bench_train.py --steps 300 2>&1 | tail -1 || exit 1
DFWFM_LIB=libdfwfm_rb32.so timeout -k 10 200 python tools/bench_train.py --steps 300 2>&1 | tail -1 || exit 1
done
