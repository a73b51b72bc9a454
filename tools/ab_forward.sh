#!/bin/bash
# dW batch-split sweep (DFWFM_DW_SPLITS, tuning only): training step time per setting.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for sp in 2 4 7 10 14; do echo "splits=$sp $(DFWFM_DW_SPLITS=$sp timeout -k 10 200 python tools/bench_train.py --steps 100 2>&1 | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" || exit 1; done
