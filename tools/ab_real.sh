#!/bin/bash
# Phase-cost ablation of the fused forward at the bench's 2 / 3 streams (diagnostic: results invalid when
# flags are dropped).  VARIANTS: "env|streams" entries.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
while read -r env st; do
  [ -z "$st" ] && continue
  out=$(env $env timeout -k 10 240 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline --streams $st)
  rc=$?; if [ $rc -ne 0 ]; then echo "$env streams=$st rc=$rc"; exit $rc; fi
  echo "$env streams=$st $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["ms_per_step"]*1000,2), "us", d["value"], d["roofline"]["frac"])')"
done <<LIST
${VARIANTS:-X=0 2
X=0 3
DFWFM_DIAG=drop_flags=1 2
DFWFM_DIAG=drop_flags=33 2
DFWFM_DIAG=drop_flags=49 2}
LIST
if [ -n "${STAMPS:-}" ]; then timeout -k 10 120 python tools/phase_stamps.py; fi
