#!/bin/bash
# Phase-cost ablation of the fused forward (diagnostic: results invalid when flags are dropped).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for ks in ${KSLIST:-1}; do
  for drop in 0 1 2 3; do
    out=$(DFWFM_KSPLIT=$ks DFWFM_DIAG_DROP_FLAGS=$drop timeout -k 10 240 python bench.py --steps 400 --warmup 40 --no-cpu-baseline)
    rc=$?; if [ $rc -ne 0 ]; then echo "ks=$ks drop=$drop rc=$rc"; exit $rc; fi
    echo "ks=$ks drop=$drop $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"]*1000, "us", d["value"])')"
  done
done
