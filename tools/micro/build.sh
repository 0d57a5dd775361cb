#!/bin/bash
# Build the IPM microbenchmark variants into tools/micro/bin (gfx950).
set -e
D=$(cd "$(dirname "$0")" && pwd)
C=$D/../../distributed_aerial_transportation_amd/csrc
mkdir -p $D/bin
b() { name=$1; shift; hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$C -DVARIANT="\"$name\"" "$@" $D/ipm_micro.hip -o $D/bin/$name; }
b r13 &
b r3 -DDAT_IPM_NROW=3 &
b r5 -DDAT_IPM_NROW=5 &
b r13minreg -mllvm -amdgpu-sched-strategy=iterative-minreg &
wait
ls -la $D/bin
