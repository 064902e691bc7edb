#!/bin/bash
# Vector-memory pipeline counters (TA / TD / TCP) of one bench workload, one rocprofv3 --pmc pass
# each group (at most 2 TA, 2 TD, 4 TCP a pass), each under its own time limit.
#   tools/gpu_mem_pmc.sh <outdir under gpurun_out> [bench.py args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
shift
ARGS="--steps 1 --warmup 0 --no-cpu-baseline $*"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
M1="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES"
M2="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VMEM"
i=0
for grp in "$M1" "$M2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/m$i" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/bench_m$i.json" 2> "$OUT/bench_m$i.err" || { echo "mem pass $i failed"; tail -5 "$OUT/bench_m$i.err"; exit 1; }
  echo "mem pass $i ok: $grp"
done
