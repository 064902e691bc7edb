#!/bin/bash
# Bench variants that differ only in environment knobs read by the library at render time.
# usage: bash tools/gpu_env_variants.sh name1 "VAR=val ..." name2 "VAR=val ..." ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-}
run() { n=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $ARGS > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err || { echo "bench $n FAILED"; tail -5 gpurun_out/bench_$n.err; exit 1; }
  python -c "import json; j=json.load(open('gpurun_out/bench_$n.json')); print('$n', j['value'], j['ms_per_step'], j.get('wave_time_share'), j.get('lane_utilization'))"; }
while [ $# -ge 2 ]; do run "$1" $2 || exit 1; shift 2; done
