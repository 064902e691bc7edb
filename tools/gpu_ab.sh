#!/bin/bash
# A/B: GPU parity tests on the product build, then config-2 bench lines alternating the product
# build and the variant .so files given as arguments (CRT_LIB), REPS rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
for r in $(seq ${REPS:-2}); do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset CRT_LIB; else export CRT_LIB=$GRAFT_REPO_ROOT/$v; fi
    n=$(basename $v .so)
    timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "bench $v FAILED"; tail -5 gpurun_out/ab_$n.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['wave_time_share'])"
  done
done
