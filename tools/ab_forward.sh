#!/bin/bash
# GPU check of one test file (default: the training suite).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_train.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; tail -25 gpurun_out/par.log; exit $rc
