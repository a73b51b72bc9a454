# FwFM-only batch sets: parity of the LDS-DMA forward, then A/B benches (tag $1)
T=${1:-r06b}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batches.py tests/test_gpu_shallow.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fwfm or shallow or pair" > gpurun_out/${T}_t-fwfm.log 2>&1 || { tail -30 gpurun_out/${T}_t-fwfm.log; exit 1; }
tail -2 gpurun_out/${T}_t-fwfm.log
run() { # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config fwfm --no-cpu-baseline --no-per-call $BARGS > gpurun_out/${T}_$n.log 2>&1 || { tail -5 gpurun_out/${T}_$n.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${T}_$n.log').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step']*1e3,3), d['roofline']['frac'])"
}
BARGS="--steps 20 --warmup 5" run f20_dma DFWFM_P3_DMA=1
BARGS="--steps 20 --warmup 5" run f20_old DFWFM_P3_DMA=0
BARGS="--steps 2000 --warmup 200" run f2k_dma DFWFM_P3_DMA=1
BARGS="--steps 2000 --warmup 200" run f2k_old DFWFM_P3_DMA=0
BARGS="--steps 2000 --warmup 200" run f2k_nofwfm DFWFM_DIAG_DMA=1
BARGS="--steps 2000 --warmup 200" run f2k_norows DFWFM_DIAG_DMA=2
BARGS="--steps 2000 --warmup 200" run f2k_none DFWFM_DIAG_DMA=3
