#!/bin/bash
# PMC passes over the bench (one counter group per pass; kernel-trace only, no sys/runtime trace),
# eager launches, one stream.  BENCH_ENV (e.g. DFWFM_SPLIT=1) selects the forward variant, BENCH_ARGS the config.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
[ -n "${BENCH_ENV:-}" ] && export ${BENCH_ENV}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-graph --streams 1 ${BENCH_ARGS:-} > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<LIST
${PMC_GROUPS:-GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum}
LIST
