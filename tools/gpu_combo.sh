set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_train2.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_shallow.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tp.log 2>&1; rc=$?; tail -2 gpurun_out/tp.log; [ $rc -ne 0 ] && exit $rc
STEPS=2000 VARIANTS="$(printf "DFWFM_NO_PART3=1 3\nX=0 3\nX=0 4\nX=0 5\nX=0 6\nDFWFM_PART3_NG8=1 2\nDFWFM_PART3_NG8=1 3\nDFWFM_PART3_NG8=1 4")" bash tools/ab_shallow.sh 2>&1 | grep -v amdgpu.ids
