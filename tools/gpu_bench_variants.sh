#!/bin/bash
# Bench only (no tests): the product build and each variant .so given as arguments.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in default "$@"; do
  if [ "$v" = default ]; then unset CRT_LIB; else export CRT_LIB=$GRAFT_REPO_ROOT/$v; fi
  n=$(basename $v .so)
  timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err || { echo "bench $v FAILED"; tail -5 gpurun_out/bench_$n.err; exit 1; }
  python -c "import json; j=json.load(open('gpurun_out/bench_$n.json')); print('$n', j['value'], 'Msamples/s', j['ms_per_step'], 'ms', j.get('wave_time_share'), j.get('lane_utilization'))"
  grep "crt counters" gpurun_out/bench_$n.err || true
done
