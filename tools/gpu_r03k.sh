# Round 3: per-phase cycles of fwd32_kernel and fwd_kernel (one workgroup per CU, eager, one stream)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03k}
timeout -k 10 200 env DFWFM_DIAG_STAMPS=1 DFWFM_R32=1 python tools/phase_stamps.py --iters 30 > gpurun_out/${T}_stamps_r32.log 2>&1 || exit 1
timeout -k 10 200 env DFWFM_DIAG_STAMPS=1 DFWFM_R32=0 python tools/phase_stamps.py --iters 30 > gpurun_out/${T}_stamps_r16.log 2>&1 || exit 1
cat gpurun_out/${T}_stamps_r32.log gpurun_out/${T}_stamps_r16.log | grep -v "^W20\|^E20\|amdgpu"
