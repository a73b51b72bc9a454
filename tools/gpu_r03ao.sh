# weight-gradient GEMM alone (tools/ubench_dw: dwr vs staged by splits); fwd32 with the per-CU K-loop token (A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03ao}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-220)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
run ubench_dw 120 ./tools/ubench_dw 4096 200 || exit 1
run tok_parity 300 env DFWFM_CU_TOKEN=1 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fwd32 or golden" --timeout 200 --timeout-method thread || exit 1
run bench2000_tok 300 env DFWFM_CU_TOKEN=1 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run bench2000 300 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run bench20_tok 300 env DFWFM_CU_TOKEN=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run bench20 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
echo done
