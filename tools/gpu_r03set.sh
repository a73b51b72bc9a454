# batch-set forward: parity, then the bench with and without sets (logs to gpurun_out/set_*)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_batches.py tests/test_gpu_parity.py -k "batch_set or fwd32" -x -v --timeout 120 --timeout-method thread > gpurun_out/set_t.log 2>&1; rc=$?; tail -3 gpurun_out/set_t.log; [ $rc -ne 0 ] && exit $rc
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --batch-set 1" "--steps 2000 --warmup 400" "--steps 20 --warmup 5 --batch-set 10 --streams 2" "--steps 20 --warmup 5 --batch-set 20 --streams 1" "--steps 2000 --warmup 400 --batch-set 1"; do
  tag=$(echo "$args" | tr -d ' -')
  timeout -k 10 200 python bench.py $args --no-cpu-baseline > gpurun_out/set_b_$tag.log 2>&1 || exit 1
  echo "$args: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step']*1e3, d['value']/1e6, r['frac'], r['launch_us'], d['streams_in_region'])" gpurun_out/set_b_$tag.log)"
done
for args in "--config fwfm --steps 20 --warmup 5" "--config fwfm --steps 20 --warmup 5 --batch-set 1" "--config fwfm --steps 2000 --warmup 400" "--config fwfm --steps 2000 --warmup 400 --batch-set 1"; do
  tag=$(echo "$args" | tr -d ' -')
  timeout -k 10 200 python bench.py $args --no-cpu-baseline > gpurun_out/set_b_$tag.log 2>&1 || exit 1
  echo "$args: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step']*1e3, d['value']/1e6, r['frac'], r['launch_us'], d['streams_in_region'])" gpurun_out/set_b_$tag.log)"
done
