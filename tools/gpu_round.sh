#!/bin/bash
# GPU round trip (gpurun): parity suite of the in-tree build, smoke, then optional A/B scripts given
# as arguments (each run with bash, chained: the first failure ends the call).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 11; }
  tail -1 gpurun_out/gpu_tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 12; }
  tail -1 gpurun_out/smoke.log
fi
for s in "$@"; do
  bash -c "$s" || { echo "step failed: $s"; exit 13; }
done
echo done
