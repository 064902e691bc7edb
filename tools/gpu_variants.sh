#!/bin/bash
# Parity tests on the product build, then the bench for the product build and each variant .so
# given as arguments (paths relative to the repo). Each step time-limited; stops on failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest FAILED"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo "pytest gpu ok: $(tail -1 gpurun_out/pytest_gpu.log)"
for v in default "$@"; do
  if [ "$v" = default ]; then unset CRT_LIB; else export CRT_LIB=$GRAFT_REPO_ROOT/$v; fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_$(basename $v .so).json 2> gpurun_out/bench_$(basename $v .so).err || { echo "bench $v FAILED"; tail -5 gpurun_out/bench_$(basename $v .so).err; exit 1; }
  python -c "import json,sys; j=json.load(open('gpurun_out/bench_$(basename $v .so).json')); print('$v', j['value'], 'Msamples/s', j['ms_per_step'], 'ms')"
done
