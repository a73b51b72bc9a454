# PMC traffic of the final forward kernels (packed tables): deep set, FwFM-only set, FwFM-only HBM-resident
set -u
for spec in "r06deep|" "r06fwfm|--config fwfm" "r06fwfm8|--config fwfm --table-scale 8"; do
  tag=${spec%%|*}; args=${spec#*|}
  TAG=$tag BENCH_ARGS="$args" PMC_GROUPS="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
FETCH_SIZE
WRITE_SIZE" bash tools/pmc.sh || exit 1
  python tools/pmc_summary.py $tag gpurun_out gpurun_out/pmc_traffic_r06.json "$args" || exit 1
done
cat gpurun_out/pmc_traffic_r06.json | head -80
