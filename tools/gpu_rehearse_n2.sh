cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
DFWFM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 400 --warmup 100 > gpurun_out/bench_n2_rehearsal.log 2>&1 || { tail -30 gpurun_out/bench_n2_rehearsal.log; exit 1; }
tail -1 gpurun_out/bench_n2_rehearsal.log
timeout -k 10 300 python bench.py --inputs zipf --no-cpu-baseline > gpurun_out/bench_zipf.log 2>&1 || exit 1
tail -1 gpurun_out/bench_zipf.log
timeout -k 10 300 python bench.py --first-order fwlw --no-cpu-baseline > gpurun_out/bench_fwlw.log 2>&1 || exit 1
tail -1 gpurun_out/bench_fwlw.log
