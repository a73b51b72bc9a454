#!/bin/bash
# GPU check of the forward parity suite (edit for A/B runs).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; tail -15 gpurun_out/par.log; exit $rc
