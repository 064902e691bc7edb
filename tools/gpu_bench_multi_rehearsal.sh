#!/bin/bash
# The N>1 bench path rehearsed on one GPU: 2 ranks share the device, tiles gathered over gloo
# (RCCL refuses two ranks on one device). Checks the multi-rank control flow, not its speed.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CRT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { echo "N=2 rehearsal FAILED"; tail -20 gpurun_out/bench_n2_gloo.err; exit 1; }
cat gpurun_out/bench_n2_gloo.json
