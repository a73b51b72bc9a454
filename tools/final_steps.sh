#!/bin/bash
# Round-end evidence on the gpurun box (tools/gpu_steps.sh steps; TAG = $1): the GPU test suite, smoke(), the
# driver's bench command under rocprofv3 (kernel trace + stats) and plain, the steady-state and per-config lines,
# the training step (deterministic default, float-atomic, several steps per graph, under rocprofv3, phase stamps), the single-call
# latency table.
T=${1:-final}
bash tools/gpu_steps.sh "$T" \
 't-tests|1100|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
 'smoke|300|python -c "import __graft_entry__ as g; g.smoke()"' \
 'bench|300|python bench.py' \
 'bench20|200|python bench.py --steps 20 --warmup 5' \
 "prof20|300|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5" \
 'bench2000|300|python bench.py --steps 2000 --warmup 400 --no-cpu-baseline' \
 'fwfm20|200|python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline' \
 "proffwfm20|300|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proffwfm20 -o run --output-format csv -- python3 bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline" \
 'fwfm2000|300|python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline --no-per-call' \
 'fwfm8-20|200|python bench.py --config fwfm --table-scale 8 --steps 20 --warmup 5 --no-cpu-baseline' \
 'qr20|200|python bench.py --config qr --steps 20 --warmup 5 --no-cpu-baseline' \
 'pruned20|200|python bench.py --config pruned --steps 20 --warmup 5 --no-cpu-baseline' \
 'train|200|python tools/bench_train.py --steps 500 --warmup 20' \
 'train4|200|python tools/bench_train.py --steps 500 --warmup 20 --steps-per-graph 4' \
 'trainatomic|200|python tools/bench_train.py --steps 500 --warmup 20 --atomic' \
 'train0|200|DFWFM_DIAG=ftrain=0 python tools/bench_train.py --steps 500 --warmup 20' \
 "proftrain|200|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proftrain -o run --output-format csv -- python3 tools/bench_train.py --steps 50" \
 'st-train|120|python tools/phase_stamps.py --train --batch 4096 --iters 10' \
 'latency|300|python tools/latency.py --calls 300'
