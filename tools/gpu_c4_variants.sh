#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for v in default cpp_raytracer_amd/lib/variants/NOTOP.so; do
  if [ "$v" = default ]; then unset CRT_LIB; else export CRT_LIB=$GRAFT_REPO_ROOT/$v; fi
  n=$(basename $v .so)
  timeout -k 10 600 python bench.py --scene millions --seed 42 --width 1920 --height 1080 --spp 256 --depth 50 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4_$n.json 2> gpurun_out/c4_$n.err || exit 1
  python -c "import json; j=json.load(open('gpurun_out/c4_$n.json')); print('$n', j['value'], j['wave_time_share'])"
done
