#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok: $(tail -1 gpurun_out/pytest_gpu.log)" &&
CRT_DEBUG_COUNTERS=1 timeout -k 10 300 python tools/phase_costs.py config2 > gpurun_out/phase_c2.txt 2>&1 && cat gpurun_out/phase_c2.txt | grep -v amdgpu.ids &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err && python -c "import json; d=json.load(open('gpurun_out/bench_q.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
