# Round 3: where the sparse deep tower's time goes (pruned config, --sparse-mlp 0.25): per-kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03ah}
timeout -k 10 300 python bench.py --config pruned --sparse-mlp 0.25 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_sparse.log 2>&1 || exit $?
grep -o '"ms_per_step[^,]*\|"launch": "[^"]*"' gpurun_out/${T}_sparse.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --config pruned --sparse-mlp 0.25 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1 || exit $?
echo done
