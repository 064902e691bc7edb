#!/bin/bash
# Counter collection: one rocprofv3 pass per counter group (no --pmc mixed with tracing options).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
ARGS=${PMC_BENCH_ARGS:---steps 1 --warmup 0 --no-cpu-baseline}
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/bench_p$i.json 2> $R/gpurun_out/pmc/bench_p$i.err || { echo "pmc pass $i ($grp) failed"; tail -5 $R/gpurun_out/pmc/bench_p$i.err; exit 1; }
  echo "pass $i ok: $grp"
done
