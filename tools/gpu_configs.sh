#!/bin/bash
# Bench lines for the other BASELINE configs (one frame each, no CPU baseline): config 3 (Cornell,
# 600x600, 1000 spp, depth 1000) and config 4 (millions of spheres, 1920x1080, 256 spp, depth 50).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --scene cornell --width 600 --height 600 --spp 1000 --depth 1000 --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/bench_config3.json 2> gpurun_out/bench_config3.err &&
echo "config3: $(cat gpurun_out/bench_config3.json)" &&
timeout -k 10 600 python bench.py --scene millions --seed 42 --width 1920 --height 1080 --spp 256 --depth 50 --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/bench_config4.json 2> gpurun_out/bench_config4.err &&
echo "config4: $(cat gpurun_out/bench_config4.json)"
