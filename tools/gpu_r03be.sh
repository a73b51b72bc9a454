# A/B in batch-set mode: fwd32 epilogue priority (DFWFM_PRIO_EPI=1); FwFM-only on four-wave workgroups (DFWFM_P3_NG=4)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r03be
timeout -k 10 300 python -u -m pytest tests/test_gpu_batches.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_t.log 2>&1 || { tail -20 gpurun_out/${T}_t.log; exit 1; }; tail -1 gpurun_out/${T}_t.log
summ() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(d['n_gpus'], round(d['ms_per_step']*1e3,3), round(d['value']/1e6,1), r['frac'], r['launch_us'])" $1; }
for rep in 1 2; do
for env in "DFWFM_PRIO_EPI=0" "DFWFM_PRIO_EPI=1" "DFWFM_DEFER_TAIL=1" "DFWFM_DEFER_TAIL=1 DFWFM_PRIO_EPI=1"; do
  for args in "--steps 2000 --warmup 400" "--steps 20 --warmup 5"; do
    tag=$(echo "$env$args" | tr -d ' -=')_$rep
    env $env timeout -k 10 200 python bench.py $args --no-cpu-baseline > gpurun_out/${T}_$tag.log 2>&1 || exit 1
    echo "$env $args: $(summ gpurun_out/${T}_$tag.log)"
  done
done
for env in "DFWFM_P3_NG=8" "DFWFM_P3_NG=4"; do
  for args in "--config fwfm --steps 2000 --warmup 400" "--config fwfm --steps 20 --warmup 5"; do
    tag=$(echo "$env$args" | tr -d ' -=')_$rep
    env $env timeout -k 10 200 python bench.py $args --no-cpu-baseline > gpurun_out/${T}_$tag.log 2>&1 || exit 1
    echo "$env $args: $(summ gpurun_out/${T}_$tag.log)"
  done
done
done
