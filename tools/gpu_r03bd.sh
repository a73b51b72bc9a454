# A/B in batch-set mode: gather / shallow priority raise (DFWFM_PRIO=0 off), and the N = 2 rehearsal (gloo, both ranks on the one GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r03bd
summ() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(d['n_gpus'], round(d['ms_per_step']*1e3,3), round(d['value']/1e6,1), r['frac'], r['launch_us'])" $1; }
for rep in 1 2; do
for pr in 1 0; do
  for args in "--steps 2000 --warmup 400" "--steps 20 --warmup 5" "--config fwfm --steps 2000 --warmup 400"; do
    tag=p${pr}_$(echo "$args" | tr -d ' -')_$rep
    DFWFM_PRIO=$pr timeout -k 10 200 python bench.py $args --no-cpu-baseline > gpurun_out/${T}_$tag.log 2>&1 || exit 1
    echo "PRIO=$pr $args: $(summ gpurun_out/${T}_$tag.log)"
  done
done
done
DFWFM_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_n2.log 2>&1 || exit 1
echo "n2: $(summ gpurun_out/${T}_n2.log)"
