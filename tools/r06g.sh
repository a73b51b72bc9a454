# full GPU suite, then deep packed/plain A/B (tag $1)
T=${1:-r06g}
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t-all.log 2>&1 || { tail -30 gpurun_out/${T}_t-all.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/${T}_t-all.log
run() { # name args...
  local n=$1; shift
  timeout -k 10 250 python bench.py "$@" > gpurun_out/${T}_$n.log 2>&1 || { tail -5 gpurun_out/${T}_$n.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/${T}_$n.log').read().strip().splitlines()[-1])
g=d.get('roofline_gather', {})
print('$n', round(d['ms_per_step']*1e3,3), d['roofline']['frac'], g.get('achieved'), g.get('us_per_batch'), g.get('lone'), d.get('per_call', {}).get('us_per_batch'))"
}
run deep20_pk --steps 20 --warmup 5 --no-cpu-baseline
run deep20_plain --steps 20 --warmup 5 --no-cpu-baseline --pack-tables 0
run deep20_pk2 --steps 20 --warmup 5 --no-cpu-baseline
run deep20_plain2 --steps 20 --warmup 5 --no-cpu-baseline --pack-tables 0
run deep2k_pk --steps 2000 --warmup 200 --no-cpu-baseline --no-per-call
run deep2k_plain --steps 2000 --warmup 200 --no-cpu-baseline --no-per-call --pack-tables 0
