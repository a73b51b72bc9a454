set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
s() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["ms_per_step"]*1000,3), "us/batch", round(d["value"]/1e6,1), "M/s frac", d["roofline"]["frac"], "launch", d["roofline"]["launch_us"])'; }
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g1.log 2>&1 || exit 1; echo "gate K20: $(s < gpurun_out/g1.log)"
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gate > gpurun_out/g2.log 2>&1 || exit 1; echo "nogate K20: $(s < gpurun_out/g2.log)"
timeout -k 10 120 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline > gpurun_out/g3.log 2>&1 || exit 1; echo "gate K2000: $(s < gpurun_out/g3.log)"
timeout -k 10 120 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g4.log 2>&1 || exit 1; echo "fwfm K20: $(s < gpurun_out/g4.log)"
timeout -k 10 120 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline > gpurun_out/g5.log 2>&1 || exit 1; echo "fwfm K2000: $(s < gpurun_out/g5.log)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; exit $rc
