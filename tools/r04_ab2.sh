#!/bin/bash
# A/B of two libdat builds on the C4 bench (interleaved, same box): $BASE (DAT_LIB_PATH) vs the in-tree build.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
O=gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/ab2_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/ab2_tests.log | cut -c1-300 | tail -20; exit 11; }
  tail -1 $O/ab2_tests.log
fi
for rep in 1 2; do
  for v in base new; do
    for B in ${BATCHES:-65536}; do
      if [ "$v" = "base" ]; then export DAT_LIB_PATH=$R/${BASE:-build_var/libdat_base.so}; else unset DAT_LIB_PATH; fi
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch $B --steps ${STEPS:-20} ${EXTRA:-} > $O/ab2_${v}_${B}_$rep.log 2>&1 || { tail -20 $O/ab2_${v}_${B}_$rep.log; exit 12; }
      echo "$v B=$B rep $rep: $(python tools/show_bench.py $O/ab2_${v}_${B}_$rep.log | head -1 | cut -c1-200)"
    done
  done
done
unset DAT_LIB_PATH
echo done
