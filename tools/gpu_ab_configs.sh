#!/bin/bash
# GPU parity tests on the product build, then bench of the product build and each variant .so
# (paths relative to the repo) on BASELINE configs 2 and 3 (CFGS="2 3 4" adds config 4). Each step
# time-limited; stops on failure. SKIP_TESTS=1 skips the tests; REPS repeats the bench rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest FAILED"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  echo "pytest gpu ok: $(tail -1 gpurun_out/pytest_gpu.log)"
fi
cfgs=()
for c in ${CFGS:-2 3}; do
  case $c in
    2) cfgs+=("c2:") ;;
    3) cfgs+=("c3:--scene cornell --width 600 --height 600 --spp 1000 --depth 1000") ;;
    4) cfgs+=("c4:--scene millions --seed 42 --width 1920 --height 1080 --spp 256 --depth 50") ;;
  esac
done
for r in $(seq ${REPS:-1}); do
for cfg in "${cfgs[@]}"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  for v in default "$@"; do
    if [ "$v" = default ]; then unset CRT_LIB; else export CRT_LIB=$GRAFT_REPO_ROOT/$v; fi
    n=${tag}_$(basename $v .so)
    timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline $args > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err || { echo "bench $n FAILED"; tail -5 gpurun_out/bench_$n.err; exit 1; }
    python -c "import json; j=json.load(open('gpurun_out/bench_$n.json')); print('$n', j['value'], 'Msamples/s', j['ms_per_step'], 'ms', j.get('wave_time_share'))"
  done
done
done
