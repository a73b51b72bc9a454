#!/bin/bash
# A/B of two library builds (DFWFM_LIB): bench throughput and PMC FETCH/WRITE per launch.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in ${LIBS:-libdfwfm_prev.so libdfwfm.so}; do
  out=$(DFWFM_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline) || exit 1
  echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"]*1000, "us", d["value"]/1e6)')"
  DFWFM_LIB=$lib TAG=ab_$lib bash tools/pmc.sh > /dev/null || exit 1
  python tools/pmc_summary.py ab_$lib gpurun_out | python -c 'import json,sys; d=json.load(sys.stdin); [print("  ", k[:50], v.get("hbm_bytes_per_launch"), round(v.get("mfma_busy_frac",0),3), v["profiled_duration_us_median"]) for k,v in d.items()]'
done
