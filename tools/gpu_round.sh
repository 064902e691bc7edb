#!/bin/bash
# One measurement session on the GPU box, every GPU step under its own time limit and chained with
# && (nothing runs after a failure):
#   1. GPU parity tests (pytest -m gpu)          -> gpurun_out/pytest_gpu.log
#   2. smoke()                                   -> gpurun_out/smoke.log
#   3. bench.py (config 2, CPU baseline)          -> gpurun_out/bench.json
#   4. rocprofv3 --kernel-trace --stats of bench  -> gpurun_out/prof/run_kernel_stats.csv
#   5. three PMC passes (FETCH_SIZE; WRITE_SIZE; 8 SQ counters), each its own rocprofv3 run, summarised into
#      gpurun_out/pmc_latest.json (tools/pmc_summary.py: the guide's gfx950 FETCH_SIZE x2, VALU issue)
#   6. bench.py again, reading that summary for roofline.traffic -> gpurun_out/bench_traffic.json
# SKIP_TESTS=1 skips 1-2; STEPS sets the bench steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
STEPS=${STEPS:-10}
W="rtow_final seed 42, 1200x800, 500 spp, max_depth 50 (BASELINE config 2)"
step_tests() {
  [ -n "$SKIP_TESTS" ] && return 0
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
  echo "pytest gpu ok: $(tail -1 gpurun_out/pytest_gpu.log)" &&
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok"
}
step_tests &&
timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo "bench ok" &&
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps $STEPS --warmup 2 --no-cpu-baseline > "$R/gpurun_out/bench_prof.json" 2> "$R/gpurun_out/bench_prof.err") && echo "rocprof ok" &&
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/p1" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc/bench_p1.json" 2> "$R/gpurun_out/pmc/bench_p1.err") && echo "pmc FETCH_SIZE ok" &&
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/p2" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc/bench_p2.json" 2> "$R/gpurun_out/pmc/bench_p2.err") && echo "pmc WRITE_SIZE ok" &&
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/p3" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc/bench_p3.json" 2> "$R/gpurun_out/pmc/bench_p3.err") && echo "pmc SQ ok" &&
python tools/pmc_summary.py gpurun_out/pmc "$W" gpurun_out/pmc_latest.json > /dev/null && echo "pmc summary ok" &&
timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --pmc-json gpurun_out/pmc_latest.json > gpurun_out/bench_traffic.json 2> gpurun_out/bench_traffic.err && echo "bench (traffic) ok"
rc=$?
cat gpurun_out/bench.json 2>/dev/null
grep -h "render_kernel\|resolve" gpurun_out/prof/*kernel_stats.csv 2>/dev/null | head -4
exit $rc
