#!/bin/bash
# Round-2 end extras: the N = 2 bench path (gloo, both ranks on the one GPU), Zipf-skewed indices for the deep
# and FwFM-only forwards, and the training step over two gloo ranks (sparse touched-row exchange).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r02z}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-200)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
DFWFM_BENCH_BACKEND=gloo run bench_n2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 400 --warmup 100 || exit 1
DFWFM_BENCH_BACKEND=gloo run fwfm_n2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --config fwfm --gpus 2 --steps 400 --warmup 100 || exit 1
run zipf 200 python bench.py --inputs zipf --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
run fwfm_zipf 200 python bench.py --config fwfm --inputs zipf --steps 2000 --warmup 400 --no-cpu-baseline || exit 1
echo done
