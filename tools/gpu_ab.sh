#!/bin/bash
# A/B of kernel variants on the BASELINE configs, alternating rounds on one box (the product
# build first in every round). A variant is a library .so (path relative to the repo, loaded
# through CRT_LIB) or an environment-knob set "name:VAR=val,VAR2=val" read by the library at run
# time. Every step has its own time limit; the script stops at the first failure.
#   TESTS=all|subset|none (default none): the GPU parity tests on the product build (all), or the
#         parity subset on each .so variant (subset: render goldens, sample means, linear mode,
#         five-wave / flat-box / HBM-scene instances, GPU-vs-oracle)
#   CFGS="2 3 4 5" (default "2"), REPS (rounds, default 1), STEPS (bench steps, default 3)
# usage: bash tools/gpu_ab.sh cpp_raytracer_amd/lib/variants/x.so "noxcd:CRT_XCD_QUEUES=0" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
SUBSET="render_matches or sample_means or linear_world or five_wave or flat_box or hbm_scene or vs_oracle and not tall"
if [ "${TESTS:-none}" = all ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
    || { echo "pytest FAILED"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  echo "pytest gpu ok: $(tail -1 gpurun_out/pytest_gpu.log)"
fi
if [ "${TESTS:-none}" = subset ]; then
  for v in "$@"; do
    case $v in *.so) ;; *) continue ;; esac
    n=$(basename $v .so)
    CRT_LIB=$R/$v timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "$SUBSET" \
      > gpurun_out/pytest_$n.log 2>&1 || { echo "pytest $n FAILED"; tail -30 gpurun_out/pytest_$n.log; exit 1; }
    echo "pytest $n ok: $(tail -1 gpurun_out/pytest_$n.log)"
  done
fi
args_of() {
  case $1 in
    2) echo "" ;;
    3) echo "--scene cornell --width 600 --height 600 --spp 1000 --depth 1000" ;;
    4) echo "--scene millions --seed 42 --width 1920 --height 1080 --spp 256 --depth 50" ;;
    5) echo "--scene rtow_final --seed 42 --width 3840 --height 2160 --spp 10000 --depth 50" ;;
  esac
}
for r in $(seq ${REPS:-1}); do
  for c in ${CFGS:-2}; do
    args=$(args_of $c)
    steps=${STEPS:-3}; [ "$c" = 5 ] && steps=1
    for v in default "$@"; do
      envs=(); n=default
      case $v in
        default) ;;
        *.so) envs=("CRT_LIB=$R/$v"); n=$(basename $v .so) ;;
        *:*) n=${v%%:*}; IFS=, read -ra envs <<< "${v#*:}" ;;
      esac
      tag=c${c}_${n}_r$r
      env "${envs[@]}" timeout -k 10 900 python bench.py --steps $steps --warmup 1 --no-cpu-baseline $args \
        > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { echo "bench $tag FAILED"; tail -5 gpurun_out/bench_$tag.err; exit 1; }
      python -c "import json; j=json.load(open('gpurun_out/bench_$tag.json')); print('$tag', j['value'], 'Msamples/s', j['ms_per_step'], 'ms', j['roofline']['kernel_ms'], 'kernel ms')"
    done
  done
done
