#!/bin/bash
# Build a variant of libdat.so with extra compile flags on dat.hip into build_var/libdat_<name>.so (CPU
# side, for tools/ab_bench.sh on the GPU box); the centralized kernel's object is compiled once into
# build_var/dat_cent.o.
#   tools/build_var.sh <name> [flags...]
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/build_var
name=$1; shift
P=$R/distributed_aerial_transportation_amd
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=on"
[ -f $R/build_var/dat_cent.o ] || hipcc $F -c $P/csrc/dat_cent.hip -o $R/build_var/dat_cent.o
[ -f $R/build_var/dat_comm.o ] || hipcc $F -c $P/csrc/dat_comm.hip -o $R/build_var/dat_comm.o
hipcc $F "$@" -c $P/csrc/dat.hip -o $R/build_var/dat_$name.o
hipcc $F -shared $R/build_var/dat_$name.o $R/build_var/dat_cent.o $R/build_var/dat_comm.o -lrccl -o $R/build_var/libdat_$name.so
rm -f $R/build_var/dat_$name.o
echo "built build_var/libdat_$name.so ($*)"
