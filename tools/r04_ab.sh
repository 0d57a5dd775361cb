#!/bin/bash
# Round-4 A/B on the GPU box: drain tests, then C4 at several sub-batch counts, then fused QP-level lines.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
O=gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_drain.py -v --timeout 300 --timeout-method thread > $O/drain_tests.log 2>&1 || { grep -E "PASS|FAIL|Error" $O/drain_tests.log | cut -c1-300 | tail -20; exit 11; }
  grep -cE "PASSED" $O/drain_tests.log
fi
for sb in ${SUBS:-1 2 3}; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --sub-batches $sb --steps ${STEPS:-20} > $O/c4_sub$sb.log 2>&1 || { tail -20 $O/c4_sub$sb.log; exit 12; }
  python tools/show_bench.py $O/c4_sub$sb.log | head -1
done
for c in ${FUSED:-}; do
  timeout -k 10 300 python -u bench.py --config $c --fused --steps ${FSTEPS:-20} --no-cpu-baseline > $O/bench_${c}_fused.log 2>&1 || { tail -30 $O/bench_${c}_fused.log; exit 15; }
  python tools/show_bench.py $O/bench_${c}_fused.log | head -1; grep -o "\"inband[^,]*,[^,]*" $O/bench_${c}_fused.log
done
echo done
