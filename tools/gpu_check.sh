#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel trace. Each GPU step has its
# own time limit and the steps are chained with && (nothing runs after a failure).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-3}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo "bench ok" &&
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps $STEPS --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_prof.err) && echo "rocprof ok"
rc=$?
cat gpurun_out/bench.json 2>/dev/null
tail -5 gpurun_out/pytest_gpu.log
exit $rc
