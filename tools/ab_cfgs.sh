#!/bin/bash
# A/B of build_var/ variants over bench configurations (gpurun): CFGS (default "C4 C2 C3 C5"), VARIANTS.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
for cfg in ${CFGS:-C4 C2 C3 C5}; do
  BENCH_ARGS="--config $cfg ${EXTRA:-}" bash tools/ab_bench.sh | sed "s/^/$cfg /" || exit 11
done
