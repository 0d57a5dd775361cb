#!/bin/bash
# GPU round trip used during development (run on the GPU box via gpurun):
#   parity tests -> smoke -> default bench -> kernel-trace profile of a short bench.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=$R/gpurun_out
mkdir -p $O/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 11; }
echo "tests ok"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 12; }
echo "smoke ok"
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 13; }
grep '^{' $O/bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof/kt -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof/kt.log 2>&1 || { echo "profile failed"; tail -20 $O/prof/kt.log; exit 14; }
  cat $O/prof/kt/run_kernel_stats.csv
fi
echo done
