#!/bin/bash
# PC sampling of one bench workload (rocprofv3 beta): which instructions the render kernel's waves
# sit on. usage: tools/gpu_pcsample.sh <outdir under gpurun_out> [bench.py args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for m in "stochastic cycles 1048576" "host_trap time 100"; do
  set -- $m
  timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $1 --pc-sampling-unit $2 \
    --pc-sampling-interval $3 --output-format csv -d "$OUT/$1" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 \
    --no-cpu-baseline "$@" > "$OUT/$1.json" 2> "$OUT/$1.err" && { echo "pc sampling ($1) ok"; exit 0; }
  echo "pc sampling ($1) failed: $(tail -2 $OUT/$1.err)"
done
exit 1
