#!/bin/bash
# Experiment-time counters (not the bench's roofline source: tools/gpu_pmc.sh is): two rocprofv3
# --pmc passes of one bench workload, VALU / issue and vector-memory groups, each under its own time
# limit, summarised by tools/quick_pmc.py. Environment knobs pass through (A/B of run-time switches).
#   tools/gpu_quick_pmc.sh <outdir under gpurun_out> [bench.py args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
shift
ARGS="--steps 1 --warmup 0 --no-cpu-baseline $*"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
Q1="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE"
Q2="TA_TA_BUSY_sum TD_TD_BUSY_sum TD_TC_STALL_sum SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
i=0
for grp in "$Q1" "$Q2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/q$i" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/bench_q$i.json" 2> "$OUT/bench_q$i.err" || { echo "quick pmc pass $i failed"; tail -5 "$OUT/bench_q$i.err"; exit 1; }
done
cd "$R" && python tools/quick_pmc.py "$OUT"
