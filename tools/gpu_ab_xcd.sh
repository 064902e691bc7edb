export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for q in 1 0 1 0; do
  CRT_XCD_QUEUES=$q timeout -k 10 300 python bench.py --scene millions --seed 42 --width 1920 --height 1080 --spp 256 --depth 50 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab4_$q.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab4_$q.json')); print('c4 xcd=$q', d['value'], d['roofline']['kernel_ms'])"
  CRT_XCD_QUEUES=$q timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab2_$q.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab2_$q.json')); print('c2 xcd=$q', d['value'], d['roofline']['kernel_ms'])"
done
