cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=r01e STEPS="bench prof prof1 profsplit" bash tools/gpu_check.sh || exit 1
TAG=fused bash tools/pmc.sh || exit 1
TAG=split BENCH_ENV=DFWFM_SPLIT=1 bash tools/pmc.sh || exit 1
python tools/pmc_summary.py fused gpurun_out gpurun_out/pmc_fused.json > /dev/null && python tools/pmc_summary.py split gpurun_out gpurun_out/pmc_split.json > /dev/null
echo done
