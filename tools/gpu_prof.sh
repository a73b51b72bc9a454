# Round-end profile set: rocprofv3 kernel stats of the driver's bench command, PMC passes (deep and FwFM-only).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/prof_$TAG.log | cut -c1-300
TAG=$TAG bash tools/pmc.sh || exit 1
TAG=${TAG}fwfm BENCH_ARGS="--config fwfm" PMC_GROUPS="$(printf "FETCH_SIZE\nWRITE_SIZE")" bash tools/pmc.sh || exit 1
python tools/pmc_summary.py $TAG gpurun_out gpurun_out/pmc_$TAG.json > /dev/null && python tools/pmc_summary.py ${TAG}fwfm gpurun_out gpurun_out/pmc_${TAG}fwfm.json > /dev/null
cat gpurun_out/pmc_$TAG.json gpurun_out/pmc_${TAG}fwfm.json | grep -E "hbm_bytes|mfma_busy|fwd_kernel|duration"
