#!/bin/bash
# Builds the render library of a git revision as an A/B variant for tools/gpu_ab.sh:
#   bash tools/build_variant.sh <rev> <name>   -> cpp_raytracer_amd/lib/variants/<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" archive "$1" cpp_raytracer_amd include | tar -x -C "$T"
mkdir -p "$R/cpp_raytracer_amd/lib/variants"
make -s -C "$T/cpp_raytracer_amd" OUT="$R/cpp_raytracer_amd/lib/variants/$2.so" OBJDIR="$T/build" -j 3
rm -rf "$T"
echo "$R/cpp_raytracer_amd/lib/variants/$2.so"
