#!/bin/bash
# Round-6 GPU call.  Steps (each under its own time limit, chained: the first failure ends the call):
#   TESTS=1   parity suite (-m gpu) + smoke of the in-tree build
#   STALL=1   stall-stretch latency (tools/stall_fixture.py) + its kernel trace
#   BENCH=1   the default bench line (C4, 10 s sustained loop, CPU baseline) -> gpurun_out/bench_r06.json
#   TAG=...   suffix of the output names
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-a}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$T.log; exit 11; }
  tail -1 gpurun_out/gpu_tests_$T.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { cat gpurun_out/smoke_$T.log; exit 12; }
  tail -1 gpurun_out/smoke_$T.log
fi
if [ "${STALL:-1}" = "1" ]; then
  timeout -k 10 300 python -u tools/stall_fixture.py gpurun_out/stall_$T.json > gpurun_out/stall_$T.log 2>&1 || { tail -20 gpurun_out/stall_$T.log; exit 13; }
  grep scenario gpurun_out/stall_$T.log | grep -v '"scenario"'
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/stall_kt_$T -o run --output-format csv -- python3 $R/tools/stall_fixture.py > $R/gpurun_out/stall_kt_$T.log 2>&1) || { tail -20 gpurun_out/stall_kt_$T.log; exit 14; }
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { tail -20 gpurun_out/bench_$T.err; exit 15; }
  python tools/show_bench.py gpurun_out/bench_$T.json || true
fi
for s in "$@"; do
  bash -c "$s" || { echo "step failed: $s"; exit 16; }
done
echo done
