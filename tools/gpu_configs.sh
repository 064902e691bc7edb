#!/bin/bash
# Bench lines for the other BASELINE configs (no CPU baseline), each step time-limited and chained:
#   config 3: Cornell, 600x600, 1000 spp, depth 1000
#   config 4: millions of spheres (seed 42), 1920x1080, 256 spp, depth 50
#   config 5: rtow_final (seed 42) at 3840x2160, 10000 spp, depth 50 -- the 8-GPU config, run on ONE
#             GPU here (82.9 G samples, ~15 s a frame; 37.6 GB of partial sums -> 10 bands)
# CONFIGS selects (default "3 4 5").
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-2}
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" --no-cpu-baseline > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err &&
  echo "$n: $(cat gpurun_out/bench_$n.json)"
}
rc=0
for c in ${CONFIGS:-3 4 5}; do
  case $c in
    3) run config3 600 --scene cornell --width 600 --height 600 --spp 1000 --depth 1000 --steps $STEPS --warmup 1 || { rc=1; break; } ;;
    4) run config4 600 --scene millions --seed 42 --width 1920 --height 1080 --spp 256 --depth 50 --steps $STEPS --warmup 1 || { rc=1; break; } ;;
    5) run config5 900 --scene rtow_final --seed 42 --width 3840 --height 2160 --spp 10000 --depth 50 --steps 1 --warmup 0 || { rc=1; break; } ;;
  esac
done
exit $rc
