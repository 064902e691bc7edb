#!/bin/bash
# Per-phase costs (tools/phase_costs.py) of the product build and each variant .so given as an
# argument, on the configs in CFGS (default "config2"), with CRT_DEBUG_COUNTERS=1 (round counters
# print when the variant was built with CRT_ROUND_COUNTERS=1). Each step time-limited; stops on failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp CRT_DEBUG_COUNTERS=1
for c in ${CFGS:-config2}; do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset CRT_LIB; else export CRT_LIB=$GRAFT_REPO_ROOT/$v; fi
    echo "== $c $(basename $v .so)"
    timeout -k 10 300 python tools/phase_costs.py $c 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
