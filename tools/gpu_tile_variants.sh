#!/bin/bash
# tools/tile_timing.py under environment knob variants: bash tools/gpu_tile_variants.sh "VAR=v ..." ...
set -o pipefail
for v in "$@"; do
  echo "== $v"; env $v timeout -k 10 300 python tools/tile_timing.py 2 2>&1 | grep -v amdgpu.ids || exit 1
done
