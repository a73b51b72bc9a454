#!/bin/bash
# A/B of bench variants on the GPU box (edit the loop): prints us per batch and M samples/s.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for wu in 20 200 1000; do for steps in 200 1000; do
  out=$(timeout -k 10 120 python bench.py --steps $steps --warmup $wu --no-cpu-baseline) || exit 1
  echo "warmup=$wu steps=$steps $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"]*1000, "us", d["value"]/1e6, d["roofline"]["launch_us"])')"
done; done
