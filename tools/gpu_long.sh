#!/bin/bash
# Long-horizon parity tests alone on the GPU box, with a heartbeat (the C-ADMM 100 s loop prints only
# at its end) and per-test durations.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
( while sleep 30; do echo "hb $(date +%T)"; done ) & HB=$!
timeout -k 10 900 python -u -m pytest tests/test_gpu_long.py -x -v -s --durations=0 --timeout 900 --timeout-method thread > gpurun_out/gpu_long.log 2>&1
rc=$?
kill $HB
tail -25 gpurun_out/gpu_long.log
exit $rc
