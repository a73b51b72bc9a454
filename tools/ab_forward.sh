#!/bin/bash
# GPU check of one test selection, then the training step.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_train.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; tail -25 gpurun_out/par.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_train.py --steps 100 2>&1 | tail -1
