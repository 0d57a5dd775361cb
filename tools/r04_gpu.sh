#!/bin/bash
# Round-4 GPU round trip: gpu tests, smoke, C4 bench, QP-level config benches (no CPU legs).
#   TESTS=0 to skip the tests; CONFIGS="C2 C3 C5" to choose the config lines.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
O=gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1080 python -u -m pytest tests -m gpu --maxfail=${MAXFAIL:-1} -v --timeout 300 --timeout-method thread ${PYARGS:-} > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 11; }
  tail -3 $O/gpu_tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 12; }
  tail -1 $O/smoke.log
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_c4.log 2>&1 || { tail -30 $O/bench_c4.log; exit 13; }
python tools/show_bench.py $O/bench_c4.log; grep "^{" $O/bench_c4.log | cut -c1-600
for c in ${CONFIGS:-C1 C2 C3 C5}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || { tail -30 $O/bench_$c.log; exit 14; }
  python tools/show_bench.py $O/bench_$c.log; grep -o "\"inband[^,]*,[^,]*" $O/bench_$c.log
done
for c in ${FUSED:-}; do
  timeout -k 10 300 python -u bench.py --config $c --fused --steps ${FSTEPS:-10} --no-cpu-baseline > $O/bench_${c}_fused.log 2>&1 || { tail -30 $O/bench_${c}_fused.log; exit 15; }
  python tools/show_bench.py $O/bench_${c}_fused.log; grep -o "\"inband[^,]*,[^,]*" $O/bench_${c}_fused.log
done
echo done
