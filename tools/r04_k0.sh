#!/bin/bash
# k_cadmm0 (class-0 drain for forestless launches): gpu tests, smoke, bench lines; C4 with a larger
# runtime scratch limit
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/k0
O=gpurun_out/k0
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=3 -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | cut -c1-300 | tail -30; exit 11; }
  tail -1 $O/gpu_tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 12; }
  tail -1 $O/smoke.log
fi
for c in C4 C2 C5 C1 C3; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 13; }
  echo "$c: $(python tools/show_bench.py $O/bench_$c.log | head -1 | cut -c30-150) $(grep -o '"inband_beyond[^,}]*' $O/bench_$c.log)"
done
HSA_SCRATCH_SINGLE_LIMIT=4294967296 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_C4_sl.log 2>&1 || { tail -20 $O/bench_C4_sl.log; exit 14; }
echo "C4 scratch limit 4 GB: $(python tools/show_bench.py $O/bench_C4_sl.log | head -1 | cut -c30-150)"
echo done
