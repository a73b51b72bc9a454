set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
for st in 2 4; do timeout -k 10 200 python bench.py --config pruned --sparse-mlp 0.25 --steps 2000 --warmup 400 --no-cpu-baseline --streams $st > gpurun_out/bp$st.log 2>&1 || exit 1; tail -1 gpurun_out/bp$st.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1000, "us/batch", d["value"]/1e6, "M/s", d["roofline"])'; done
