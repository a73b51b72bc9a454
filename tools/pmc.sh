#!/bin/bash
# PMC passes over the bench (one counter group per pass; kernel-trace only, no sys/runtime trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-graph --streams 1 > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done <<LIST
${PMC_GROUPS:-GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE
WRITE_SIZE
TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum}
LIST
