#!/bin/bash
# C2 small-batch A/B of the C-ADMM slots per wavefront (DAT_SLOT_BLOCKS target blocks).
set -u
for sb in 1024 256 128 64 32; do
  echo "slot blocks $sb"
  DAT_SLOT_BLOCKS=$sb VARIANTS="slots" BENCH_ARGS="--config C2 --fixed-work" TESTS=0 bash tools/gpu_ab.sh || exit 11
  DAT_SLOT_BLOCKS=$sb VARIANTS="slots" BENCH_ARGS="--config C2" TESTS=0 bash tools/gpu_ab.sh || exit 12
done
