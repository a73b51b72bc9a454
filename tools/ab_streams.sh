#!/bin/bash
# A/B of streams x env at the driver's K=20 and at K=2000 (forward bench, no CPU baseline).  VARIANTS: "env streams K".
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
while read -r env st k; do
  [ -z "$k" ] && continue
  w=$([ "$k" -gt 100 ] && echo 400 || echo 5)
  out=$(env $env timeout -k 10 200 python bench.py --steps $k --warmup $w --no-cpu-baseline --streams $st)
  rc=$?; if [ $rc -ne 0 ]; then echo "$env streams=$st K=$k rc=$rc"; exit $rc; fi
  echo "$env streams=$st K=$k $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["ms_per_step"]*1000,2), "us", round(d["value"]/1e6,1), "M/s", d["roofline"]["frac"], d["streams_in_region"])')"
done <<LIST
${VARIANTS}
LIST
