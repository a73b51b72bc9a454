# PMC of the training step's kernels (tools/bench_train.py, eager, fewer steps): one counter group per pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmctr_$i -o run --output-format csv -- python3 tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/pmctr_$i.log 2>&1
  rc=$?; echo "pass $i [$grp] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmctr_$i.log; exit $rc; }
  python - "$i" <<'PY'
import csv, sys, statistics as st, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f"gpurun_out/pmctr_{sys.argv[1]}/run_counter_collection.csv")):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if any(x in k for x in ("dw_kernel", "dwr_", "dw_sum", "bwd_kernel", "fwd_kernel", "ftrain", "scatter", "adam_dev")):
        d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in d.items():
    print(k[:40], {n: round(st.median(v)) for n, v in c.items()})
PY
done <<LIST
${PMC_GROUPS:-GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES
SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F32}
LIST
