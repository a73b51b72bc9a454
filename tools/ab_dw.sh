#!/bin/bash
# A/B of two dw_kernel builds (libdfwfm.so vs $ALT) and batch splits on the training step (scratch).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
ALT=${ALT:-libdfwfm_alt.so}
DFWFM_LIB=$ALT timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; tail -2 gpurun_out/par.log; [ $rc -ne 0 ] && exit $rc
for v in "alt 0" "alt 0"; do
  set -- $v
  lib=libdfwfm.so; [ $1 = alt ] && lib=$ALT
  if [ $2 = 0 ]; then unset DFWFM_DW_SPLITS; else export DFWFM_DW_SPLITS=$2; fi
  echo "$1 splits=$2"
  DFWFM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dw_$1$2 -o run --output-format csv -- python3 tools/bench_train.py --steps 30 > gpurun_out/prof_dw.log 2>&1 || exit 1
  grep dw_kernel gpurun_out/prof_dw_$1$2/run_kernel_stats.csv | cut -d, -f1-4
done
