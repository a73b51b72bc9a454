# packed serving tables (FwFM-only) + forward_gather: tests, then benches (tag $1)
T=${1:-r06f}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batches.py tests/test_gpu_shallow.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_t-fwd.log 2>&1 || { tail -30 gpurun_out/${T}_t-fwd.log; exit 1; }
tail -2 gpurun_out/${T}_t-fwd.log
run() { # name args...
  local n=$1; shift
  timeout -k 10 250 python bench.py "$@" > gpurun_out/${T}_$n.log 2>&1 || { tail -5 gpurun_out/${T}_$n.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/${T}_$n.log').read().strip().splitlines()[-1])
print('$n', round(d['ms_per_step']*1e3,3), d['roofline']['frac'], d.get('roofline_gather', {}).get('achieved'), d.get('roofline_gather', {}).get('us_per_batch'), d.get('per_call', {}).get('us_per_batch'))"
}
run f20_pk --config fwfm --steps 20 --warmup 5 --no-cpu-baseline
run f20_plain --config fwfm --steps 20 --warmup 5 --no-cpu-baseline --no-per-call --pack-tables 0
run f2k_pk --config fwfm --steps 2000 --warmup 200 --no-cpu-baseline --no-per-call
run f2k_plain --config fwfm --steps 2000 --warmup 200 --no-cpu-baseline --no-per-call --pack-tables 0
run f20s8_pk --config fwfm --steps 20 --warmup 5 --no-cpu-baseline --no-per-call --table-scale 8
run f20s8_plain --config fwfm --steps 20 --warmup 5 --no-cpu-baseline --no-per-call --table-scale 8 --pack-tables 0
run deep20 --steps 20 --warmup 5 --no-cpu-baseline
