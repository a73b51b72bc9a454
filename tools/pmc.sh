#!/bin/bash
# PMC passes over bench.py's own command (hipGraph replay, its streams; rocprofv3 --pmc serialises the dispatches
# it counts), one counter group per pass, kernel-trace counters only (no sys / runtime trace).  64 steps after 64
# warmup: with the default batch sets (32) on two streams every launch holds 32 batches.
#   TAG=r03e BENCH_ARGS="--config fwfm --table-scale 8" bash tools/pmc.sh
# then: python tools/pmc_summary.py TAG gpurun_out profiles/pmc_traffic.json "$BENCH_ARGS"
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
[ -n "${BENCH_ENV:-}" ] && export ${BENCH_ENV}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $grp -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 bench.py --steps 64 --warmup 64 --settle-ms 0 --no-gate --no-cpu-baseline --no-per-call ${BENCH_ARGS:-} > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<LIST
${PMC_GROUPS:-GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum}
LIST
