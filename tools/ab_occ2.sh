#!/bin/bash
# Occupancy A/B: the base build at 4 resident k_cadmm wavefronts per CU vs a build whose k_cadmm is
# held to 256 registers (amdgpu_waves_per_eu(2), more scratch) at 8 per CU; C4 and C5.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
for cfg in "C4" "C5"; do
  for w in 4 8; do
    DAT_WAVES_PER_CU=$w VARIANTS="${VARIANTS:-base wpe2}" BENCH_ARGS="--config $cfg" TESTS=0 bash tools/ab_bench.sh | sed "s/^/$cfg w=$w /" || exit 11
  done
done
echo done
