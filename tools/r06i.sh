# full GPU suite, smoke, the driver's bench command, FwFM-only and training step (tag $1)
T=${1:-r06i}
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t-all.log 2>&1 || { tail -30 gpurun_out/${T}_t-all.log; exit 1; }; tail -2 gpurun_out/${T}_t-all.log; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -2 gpurun_out/${T}_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench20.log 2>&1 || { tail -20 gpurun_out/${T}_bench20.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/${T}_bench20.log').read().strip().splitlines()[-1])
print('bench20', d['ms_per_step']*1e3, d['roofline']['frac'], d['roofline_gather']['achieved'], d['roofline_gather']['us_per_batch'], d['per_call']['us_per_batch'], d['cpu_baseline']['value'], d['parity'])"
timeout -k 10 300 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_fwfm20.log 2>&1 || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/${T}_fwfm20.log').read().strip().splitlines()[-1])
print('fwfm20', d['ms_per_step']*1e3, d['roofline']['frac'], d['per_call']['us_per_batch'])"
timeout -k 10 300 python tools/bench_train.py > gpurun_out/${T}_train.log 2>&1 || { tail -5 gpurun_out/${T}_train.log; exit 1; }
tail -1 gpurun_out/${T}_train.log
