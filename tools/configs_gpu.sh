#!/bin/bash
# GPU round trip for the SURVEY.md 8(d) QP-level configs: parity tests, then one bench line per config.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 11; }
  tail -3 gpurun_out/gpu_tests.log
fi
for c in C2 C3 C5; do
  timeout -k 10 240 python -u bench.py --config $c --cpu-sample-s ${CPU_S:-10} > gpurun_out/bench_$c.log 2>&1 || { tail -20 gpurun_out/bench_$c.log; exit 12; }
  grep '^{' gpurun_out/bench_$c.log
done
for c in C2 C5; do
  timeout -k 10 240 python -u bench.py --config $c --fixed-work --no-cpu-baseline > gpurun_out/bench_${c}_fw.log 2>&1 || { tail -20 gpurun_out/bench_${c}_fw.log; exit 13; }
  grep '^{' gpurun_out/bench_${c}_fw.log
done
echo done
