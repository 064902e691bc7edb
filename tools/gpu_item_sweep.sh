#!/bin/bash
# Work-queue item size sweep on the per-rank shares of config 2 (tools/tile_timing.py, every rank
# of N = 1, 2, 4, 8 rendered alone on one GPU). Frames never change with these knobs.
# CFGS entries are K:T = CRT_ITEM_CHUNKS:CRT_TAIL_CHUNKS (measured in round 2: DESIGN.md §6).
# Each step time-limited; stops on the first failure.
set -o pipefail
for cfg in ${CFGS:-"1:0" "2:30" "3:30" "4:30" "4:60"}; do
  IFS=: read -r k t <<< "$cfg"
  echo "== CRT_ITEM_CHUNKS=$k CRT_TAIL_CHUNKS=$t"
  CRT_ITEM_CHUNKS=$k CRT_TAIL_CHUNKS=$t timeout -k 10 200 python tools/tile_timing.py 3 all 2>&1 | grep "N=" || exit 1
done
