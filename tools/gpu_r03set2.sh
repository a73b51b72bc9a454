# batch-set forward: stream / set-size sweep, PMC passes and the rocprofv3 summary of the driver's command
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step']*1e3,3), round(d['value']/1e6,1), r['frac'], r['launch_us'], r.get('traffic'), d['streams_in_region'])" $1; }
for args in "--config fwfm --steps 20 --warmup 5 --streams 1" "--config fwfm --steps 20 --warmup 5 --streams 3" "--config fwfm --steps 2000 --warmup 400 --streams 1" "--config fwfm --steps 2000 --warmup 400 --streams 3" "--config fwfm --steps 2000 --warmup 400 --batch-set 32" "--steps 2000 --warmup 400 --batch-set 32" "--steps 2000 --warmup 400 --streams 3"; do
  tag=$(echo "$args" | tr -d ' -')
  timeout -k 10 200 python bench.py $args --no-cpu-baseline > gpurun_out/set2_b_$tag.log 2>&1 || exit 1
  echo "$args: $(summ gpurun_out/set2_b_$tag.log)"
done
TAG=r03set BENCH_ARGS="" bash tools/pmc.sh || exit 1
python tools/pmc_summary.py r03set gpurun_out gpurun_out/pmc_traffic_new.json "" | grep -E "hbm_bytes|mfma_busy|kernel"
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_base.json
python tools/pmc_summary.py r03set gpurun_out gpurun_out/pmc_traffic_base.json "" > /dev/null
TAG=r03setf BENCH_ARGS="--config fwfm" bash tools/pmc.sh || exit 1
python tools/pmc_summary.py r03setf gpurun_out gpurun_out/pmc_traffic_base.json "--config fwfm" | grep -E "hbm_bytes|kernel"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_set20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_set20.log 2>&1 || exit 1
grep -v "^W20\|^E20" gpurun_out/prof_set20.log | tail -1 | cut -c1-300
