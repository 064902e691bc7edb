#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { n=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err || { echo "bench $n FAILED"; tail -5 gpurun_out/bench_$n.err; exit 1; }
  python -c "import json; j=json.load(open('gpurun_out/bench_$n.json')); print('$n', j['value'], j['ms_per_step'], j.get('wave_time_share'), j.get('lane_utilization'))"; }
run default A=1 && run nolds CRT_NO_LDS_SCENE=1
