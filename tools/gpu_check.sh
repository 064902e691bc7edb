#!/bin/bash
# The round's quick check session: every GPU test, then bench lines of configs 2-4 (3 steps, no CPU
# baseline) with their frame digests. Each GPU step has its own time limit; stops at the first
# failure.   usage: bash tools/gpu_check.sh <outdir under gpurun_out> [configs, default "2 3 4"]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/$1
CFGS=${2:-"2 3 4"}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { echo "pytest FAILED"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
echo "pytest gpu: $(tail -1 "$OUT/pytest_gpu.log")"
for c in $CFGS; do
  case $c in
    2) a="" ;;
    3) a="--scene cornell --width 600 --height 600 --spp 1000 --depth 1000" ;;
    4) a="--scene millions --seed 42 --width 1920 --height 1080 --spp 256 --depth 50" ;;
    5) a="--scene rtow_final --seed 42 --width 3840 --height 2160 --spp 10000 --depth 50" ;;
  esac
  steps=3; [ "$c" = 5 ] && steps=1
  timeout -k 10 600 python bench.py --steps $steps --warmup 1 --no-cpu-baseline $a > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" \
    || { echo "bench c$c FAILED"; tail -5 "$OUT/bench_c$c.err"; exit 1; }
  python -c "import json; j=json.load(open('$OUT/bench_c$c.json')); print('c$c', j['ms_per_step'], 'ms', j['roofline']['kernel_ms'], 'kernel ms', j['frame_check']['frame_digest'], j['config']['workload'])"
done
