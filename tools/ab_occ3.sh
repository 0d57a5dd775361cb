#!/bin/bash
# Occupancy A/B without a forest (class-0 LDS carve only): base (512 registers) vs wpe2 (256
# registers, more scratch) at 4 / 8 resident k_cadmm wavefronts per CU; C5 and C2.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
for cfg in ${CFGS:-C5 C2}; do
  for w in ${WAVES:-4 8}; do
    DAT_WAVES_PER_CU=$w VARIANTS="${VARIANTS:-base wpe2}" BENCH_ARGS="--config $cfg" bash tools/ab_bench.sh | sed "s/^/$cfg w=$w /" || exit 11
  done
done
echo done
