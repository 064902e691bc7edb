#!/bin/bash
# GPU parity tests on the product build, then bench of the product build and each variant .so
# (paths relative to the repo) on BASELINE configs 2 and 3. Each step time-limited; stops on failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest FAILED"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo "pytest gpu ok: $(tail -1 gpurun_out/pytest_gpu.log)"
for cfg in "c2:" "c3:--scene cornell --width 600 --height 600 --spp 1000 --depth 1000"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  for v in default "$@"; do
    if [ "$v" = default ]; then unset CRT_LIB; else export CRT_LIB=$GRAFT_REPO_ROOT/$v; fi
    n=${tag}_$(basename $v .so)
    timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline $args > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err || { echo "bench $n FAILED"; tail -5 gpurun_out/bench_$n.err; exit 1; }
    python -c "import json; j=json.load(open('gpurun_out/bench_$n.json')); print('$n', j['value'], 'Msamples/s', j['ms_per_step'], 'ms')"
  done
done
