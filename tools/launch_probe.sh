# Per-frame fixed cost: kernel trace of a tiny frame (64x16, 4 spp) through bench.py's render path
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/launch
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/launch/tiny -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --width 64 --height 16 --spp 4 --no-cpu-baseline > $R/gpurun_out/launch/tiny.json 2> $R/gpurun_out/launch/tiny.err && echo "tiny ok"
