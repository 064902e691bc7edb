#!/bin/bash
# Parity subset of the GPU tests on each variant library (CRT_LIB), then the config A/B of
# tools/gpu_ab_configs.sh. usage: tools/gpu_variant_check.sh lib/variants/x.so ...  (paths relative
# to cpp_raytracer_amd/); CFGS / REPS / STEPS as in gpu_ab_configs.sh.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
vs=()
for v in "$@"; do
  vs+=("cpp_raytracer_amd/$v")
  n=$(basename $v .so)
  CRT_LIB=$R/cpp_raytracer_amd/$v timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    -k "render_matches or sample_means or linear_world or five_wave or flat_box or hbm_scene or vs_oracle and not tall" > gpurun_out/pytest_$n.log 2>&1 \
    || { echo "pytest $n FAILED"; tail -30 gpurun_out/pytest_$n.log; exit 1; }
  echo "pytest $n ok: $(tail -1 gpurun_out/pytest_$n.log)"
done
SKIP_TESTS=1 bash tools/gpu_ab_configs.sh "${vs[@]}"
