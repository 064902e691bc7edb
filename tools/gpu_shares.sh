#!/bin/bash
# Multi-GPU evidence on one GPU, every step time-limited and chained:
#   1. per-rank shares (tools/tile_timing.py --all: every rank of N = 1, 2, 4, 8 rendered alone,
#      packed, plus a rank's setup) for the configs in CFGS (default "2 4 5")
#      -> gpurun_out/shares/config<c>.txt
#   2. per-phase costs of the instrumented pass, walking like the timed kernel (CRT_COUNT_SPEC=1,
#      CRT_ROUND_COUNTERS=1; tools/phase_costs.py) for PHASES (default "config2")
#      -> gpurun_out/shares/phases_<c>.txt
#   3. bench.py's N-rank pipeline with 2 ranks sharing the device over gloo (REHEARSE=1)
# Item-size knobs for sweeps: CRT_ITEM_CHUNKS / CRT_TAIL_CHUNKS in the environment.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/shares
export TMPDIR=/tmp
for c in ${CFGS:-2 4 5}; do
  steps=3; [ "$c" = 5 ] && steps=1
  timeout -k 10 900 python -u tools/tile_timing.py --config $c --steps $steps --all > gpurun_out/shares/config$c.txt 2>&1 \
    || { echo "tile_timing config $c FAILED"; tail -5 gpurun_out/shares/config$c.txt; exit 1; }
  cat gpurun_out/shares/config$c.txt
done
for p in ${PHASES:-config2}; do
  CRT_COUNT_SPEC=1 CRT_ROUND_COUNTERS=1 CRT_DEBUG_COUNTERS=1 timeout -k 10 300 python -u tools/phase_costs.py $p \
    > gpurun_out/shares/phases_$p.txt 2>&1 || { echo "phases $p FAILED"; exit 1; }
  cat gpurun_out/shares/phases_$p.txt
done
if [ -n "$REHEARSE" ]; then
  CRT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/shares/bench_n2_gloo.json \
    2> gpurun_out/shares/bench_n2_gloo.err || { echo "N=2 rehearsal FAILED"; tail -20 gpurun_out/shares/bench_n2_gloo.err; exit 1; }
  cat gpurun_out/shares/bench_n2_gloo.json
fi
