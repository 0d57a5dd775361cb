#!/bin/bash
# Development round trip on the GPU box: parity tests, then the bench at both C4 start modes.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 11; }
  tail -1 gpurun_out/gpu_tests.log
fi
timeout -k 10 200 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/occ_path.log 2>&1 || { tail -20 gpurun_out/occ_path.log; exit 12; }
timeout -k 10 200 python -u bench.py --no-cpu-baseline --start edge ${BENCH_ARGS:-} > gpurun_out/occ_edge.log 2>&1 || { tail -20 gpurun_out/occ_edge.log; exit 13; }
echo done
