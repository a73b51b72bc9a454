set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline > gpurun_out/bf.log 2>&1 || exit 1; tail -1 gpurun_out/bf.log | cut -c1-120
TAG=r02fwfm8 BENCH_ARGS="--config fwfm" PMC_GROUPS="$(printf "FETCH_SIZE\nWRITE_SIZE")" bash tools/pmc.sh || exit 1
python tools/pmc_summary.py r02fwfm8 gpurun_out gpurun_out/pmc_r02fwfm8.json | grep -E "hbm|fwd"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proffwfm -o run --output-format csv -- python3 bench.py --config fwfm --steps 20 --warmup 5 > gpurun_out/pf.log 2>&1 || exit 1
grep -v "^W20\|^E20" gpurun_out/pf.log | tail -1 | cut -c1-200
