#!/bin/bash
# Round-5 GPU call: parity suite + smoke of the in-tree build, C4 A/B of build variants, the 10 s C4 loop.
#   TESTS=0|1 VARIANTS="base new" LONG=0|1 bash tools/r05_gpu.sh
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 11; }
  tail -1 gpurun_out/gpu_tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 12; }
  tail -1 gpurun_out/smoke.log
fi
if [ -n "${VARIANTS:-}" ]; then
  VARIANTS="$VARIANTS" STEPS=${STEPS:-20} WARMUP=${WARMUP:-5} bash tools/ab_bench.sh || exit 13
fi
if [ "${LONG:-0}" = "1" ]; then
  timeout -k 10 400 python -u tools/c4_long_run.py 1000 100 gpurun_out/c4_long_run_r05.json > gpurun_out/c4_long_run_r05.log 2>&1 || { tail -20 gpurun_out/c4_long_run_r05.log; exit 14; }
  tail -12 gpurun_out/c4_long_run_r05.log
fi
echo done
