#!/bin/bash
# Build a variant of libdat.so with extra compile flags into build_var/libdat_<name>.so (CPU side, for
# tools/ab_bench.sh on the GPU box).   tools/build_var.sh <name> [flags...]
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/build_var
name=$1; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" $R/distributed_aerial_transportation_amd/csrc/dat.hip \
  -o $R/build_var/libdat_$name.so
echo "built build_var/libdat_$name.so ($*)"
