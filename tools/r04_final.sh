#!/bin/bash
# Final-tree round trip: gpu tests, smoke, the default bench line with its CPU baseline leg
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/final
O=gpurun_out/final
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=${MAXFAIL:-3} -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 11; }
tail -3 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 12; }
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 13; }
python tools/show_bench.py $O/bench.log | head -1
echo done
