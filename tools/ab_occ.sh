set -u
VARIANTS="base dd ddocc" BENCH_ARGS="--config C3" TESTS=0 bash tools/gpu_ab.sh || exit 11
for w in 4 3 2; do
  echo "C4 waves/CU=$w"
  DAT_WAVES_PER_CU=$w VARIANTS="dd" TESTS=0 bash tools/gpu_ab.sh || exit 12
done
