# does an idle gap before the timed region change the 20-step number (clock drop)?
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r03bn
summ() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(d.get('idle_before_region_us'), d['n_gpus'], round(d['ms_per_step']*1e3,3), round(d['value']/1e6,1), r['frac'], r['launch_us'])" $1; }
for rep in 1 2 3 4; do
for idle in 0 2; do
  DFWFM_BENCH_IDLE_MS=$idle timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_i${idle}_$rep.log 2>&1 || exit 1
  echo "IDLE=$idle: $(summ gpurun_out/${T}_i${idle}_$rep.log)"
done
done
