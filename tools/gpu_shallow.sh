set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shallow.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -15 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/timeline.py --fwfm --streams 2 > gpurun_out/tl2.log 2>&1 || exit 1
for st in 2 4; do timeout -k 10 200 python bench.py --config fwfm --steps 400 --warmup 40 --no-cpu-baseline --streams $st > gpurun_out/bf$st.log 2>&1 || exit 1; done
DFWFM_SHALLOW=0 timeout -k 10 200 python bench.py --config fwfm --steps 400 --warmup 40 --no-cpu-baseline --streams 2 > gpurun_out/bf_old.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bf20.log 2>&1 || exit 1
cat gpurun_out/tl2.log; for f in gpurun_out/bf*.log; do echo $f; tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1000, "us/batch", d["value"]/1e6, "M/s", d["roofline"]["frac"], d["roofline"]["launch_us"])'; done
