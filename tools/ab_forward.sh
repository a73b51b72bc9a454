#!/bin/bash
# A/B of forward variants on the GPU box: parity tests, then bench per (tile groups, split, streams).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; tail -3 gpurun_out/par.log; [ $rc -ne 0 ] && exit $rc
for ng in 8 4; do for sp in 0 1; do for st in 1 2; do
  out=$(DFWFM_NG=$ng DFWFM_SPLIT=$sp timeout -k 10 120 python bench.py --steps 1000 --warmup 40 --no-cpu-baseline --streams $st) || exit 1
  echo "ng=$ng split=$sp streams=$st $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"]*1000, "us", d["value"]/1e6)')"
done; done; done
