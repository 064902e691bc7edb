#!/bin/bash
# GPU parity tests + a short bench (no profiler). Each step time-limited, chained with &&.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-3}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err && echo "bench ok"
rc=$?
cat gpurun_out/bench.json 2>/dev/null
tail -15 gpurun_out/pytest_gpu.log
tail -3 gpurun_out/bench.err
exit $rc
