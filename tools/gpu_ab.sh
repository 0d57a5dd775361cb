#!/bin/bash
# Development round trip on the GPU box: parity tests of the in-tree build, then an A/B of the
# build_var/ variants on the C4 bench (tools/ab_bench.sh).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 11; }
  tail -1 gpurun_out/gpu_tests.log
fi
bash tools/ab_bench.sh
