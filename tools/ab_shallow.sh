#!/bin/bash
# A/B of the FwFM-only forward (bench --config fwfm): kernel variant env x streams.  VARIANTS: "env streams" lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
while read -r env st; do
  [ -z "$st" ] && continue
  out=$(env $env timeout -k 10 200 python bench.py --config fwfm --steps ${STEPS:-2000} --warmup 400 --no-cpu-baseline --streams $st)
  rc=$?; if [ $rc -ne 0 ]; then echo "$env streams=$st rc=$rc"; exit $rc; fi
  echo "$env streams=$st $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["ms_per_step"]*1000,3), "us/batch", round(d["value"]/1e6,1), "M/s frac", d["roofline"]["frac"], "launch", d["roofline"]["launch_us"])')"
done <<LIST
${VARIANTS}
LIST
