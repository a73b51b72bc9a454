# A/B: fwd32 first-round stagger (DFWFM_STAGGER=n sleeps of ~8k cycles for the second workgroup of each CU)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r03bl
summ() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(d['n_gpus'], round(d['ms_per_step']*1e3,3), round(d['value']/1e6,1), r['frac'], r['launch_us'])" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_batches.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_t.log 2>&1 || { tail -20 gpurun_out/${T}_t.log; exit 1; }; tail -1 gpurun_out/${T}_t.log
for rep in 1 2 3; do
for sg in 0 1 2 3; do
  DFWFM_STAGGER=$sg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_s${sg}_$rep.log 2>&1 || exit 1
  echo "STAGGER=$sg: $(summ gpurun_out/${T}_s${sg}_$rep.log)"
done
done
