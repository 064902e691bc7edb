#!/bin/bash
# One measurement session on the GPU box, every GPU step under its own time limit and chained with
# && (nothing runs after a failure):
#   1. GPU parity tests (pytest -m gpu)                 -> gpurun_out/pytest_gpu.log
#   2. smoke()                                          -> gpurun_out/smoke.log
#   3. bench.py (config 2, CPU baseline)                 -> gpurun_out/bench.json
#   4. rocprofv3 --kernel-trace --stats of the bench     -> gpurun_out/prof/run_kernel_stats.csv
#   5. PMC passes of config 2 (tools/gpu_pmc.sh)         -> gpurun_out/pmc_c2/summary.json (= pmc_latest.json)
#   6. bench.py again, reading that summary              -> gpurun_out/bench_traffic.json
#   7. PMC passes of configs 3 and 4 (PMC_CONFIGS=1)     -> gpurun_out/pmc_c3, pmc_c4
#   8. VALU issue-cost microbenchmark (VALU_RATE=1)      -> gpurun_out/valu_rate.json
#   9. bench lines of BASELINE configs 3, 4, 5 on one GPU (CONFIGS="3 4 5"), each with its CPU baseline
#      at reduced spp, extrapolated               -> gpurun_out/bench_config<c>.json
# SKIP_TESTS=1 skips 1-2; SKIP_BENCH=1 skips 3-4; SKIP_PMC=1 skips 5-6; STEPS sets the bench steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
C3="--scene cornell --width 600 --height 600 --spp 1000 --depth 1000"
C4="--scene millions --width 1920 --height 1080 --spp 256 --depth 50"
step_tests() {
  [ -n "$SKIP_TESTS" ] && return 0
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
  echo "pytest gpu ok: $(tail -1 gpurun_out/pytest_gpu.log)" &&
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok"
}
step_configs() {
  [ -n "$PMC_CONFIGS" ] || return 0
  bash tools/gpu_pmc.sh gpurun_out/pmc_c3 $C3 && bash tools/gpu_pmc.sh gpurun_out/pmc_c4 $C4
}
step_bench_configs() {
  for c in $CONFIGS; do
    case $c in
      # CPU baselines at reduced spp, extrapolated linearly in samples (BASELINE.md §3 Coverage)
      3) a="$C3 --steps 2 --warmup 1 --cpu-spp 100" ;;
      4) a="$C4 --seed 42 --steps 2 --warmup 1 --cpu-spp 16" ;;
      5) a="--scene rtow_final --seed 42 --width 3840 --height 2160 --spp 10000 --depth 50 --steps 1 --warmup 0 --cpu-spp 16" ;;
      *) continue ;;
    esac
    timeout -k 10 900 python bench.py $a > gpurun_out/bench_config$c.json 2> gpurun_out/bench_config$c.err &&
    echo "config $c: $(cat gpurun_out/bench_config$c.json | head -c 300)" || return 1
  done
}
step_pmc() {
  [ -n "$SKIP_PMC" ] && return 0
  bash tools/gpu_pmc.sh gpurun_out/pmc_c2 && cp gpurun_out/pmc_c2/summary.json gpurun_out/pmc_latest.json &&
  timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --pmc-json gpurun_out/pmc_latest.json > gpurun_out/bench_traffic.json 2> gpurun_out/bench_traffic.err && echo "bench (traffic) ok"
}
step_valu() {
  [ -n "$VALU_RATE" ] || return 0
  timeout -k 10 120 tools/build/valu_rate > gpurun_out/valu_rate.json && echo "valu_rate ok"
}
step_bench() {
  [ -n "$SKIP_BENCH" ] && return 0
  timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo "bench ok" &&
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps $STEPS --warmup 2 --no-cpu-baseline > "$R/gpurun_out/bench_prof.json" 2> "$R/gpurun_out/bench_prof.err") && echo "rocprof ok"
}
step_tests && step_bench && step_pmc && step_configs && step_valu && step_bench_configs
rc=$?
cat gpurun_out/bench.json 2>/dev/null
grep -h "render_kernel\|resolve" gpurun_out/prof/*kernel_stats.csv 2>/dev/null | head -4
exit $rc
