set -o pipefail
mkdir -p gpurun_out/sched
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sched/c2_default.json 2>/dev/null && echo "default $(python -c "import json;j=json.load(open('gpurun_out/sched/c2_default.json'));print(j['ms_per_step'])")" &&
CRT_ITEM_CHUNKS=3 CRT_TAIL_CHUNKS=81 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sched/c2_k3t81.json 2>/dev/null && echo "K3 tail81 $(python -c "import json;j=json.load(open('gpurun_out/sched/c2_k3t81.json'));print(j['ms_per_step'])")" &&
CRT_ITEM_CHUNKS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sched/c2_k1.json 2>/dev/null && echo "K1 $(python -c "import json;j=json.load(open('gpurun_out/sched/c2_k1.json'));print(j['ms_per_step'])")" &&
timeout -k 10 300 python -u tools/tile_timing.py --config 2 --ns 8 --all > gpurun_out/sched/n8_default.txt 2>&1 && tail -1 gpurun_out/sched/n8_default.txt &&
CRT_ITEM_CHUNKS=7 CRT_TAIL_CHUNKS=13 timeout -k 10 300 python -u tools/tile_timing.py --config 2 --ns 8 --all > gpurun_out/sched/n8_k7t13.txt 2>&1 && tail -1 gpurun_out/sched/n8_k7t13.txt &&
CRT_ITEM_CHUNKS=7 CRT_TAIL_CHUNKS=40 timeout -k 10 300 python -u tools/tile_timing.py --config 2 --ns 8 --all > gpurun_out/sched/n8_k7t40.txt 2>&1 && tail -1 gpurun_out/sched/n8_k7t40.txt &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --width 64 --height 16 --spp 4 --no-cpu-baseline > gpurun_out/sched/tiny.json 2>/dev/null && echo "tiny $(python -c "import json;j=json.load(open('gpurun_out/sched/tiny.json'));print(j['ms_per_step'], j['roofline']['kernel_ms'])")"
