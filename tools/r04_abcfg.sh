#!/bin/bash
# A/B of two libdat builds over bench configs, interleaved: LIBS="name=path ...", CFGS="C4 C5 ..."
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
O=gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/abc_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/abc_tests.log | cut -c1-300 | tail -20; exit 11; }
  tail -1 $O/abc_tests.log
fi
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $LIBS; do
    name=${spec%%=*}; path=${spec#*=}
    if [ -n "$path" ]; then export DAT_LIB_PATH=$R/$path; else unset DAT_LIB_PATH; fi
    for c in ${CFGS:-C4}; do
      timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline ${EXTRA:-} > $O/abc_${name}_${c}_$rep.log 2>&1 || { tail -20 $O/abc_${name}_${c}_$rep.log; exit 12; }
      echo "$name $c rep $rep: $(python tools/show_bench.py $O/abc_${name}_${c}_$rep.log | head -1 | cut -c30-150) $(grep -o '"inband_beyond[^,}]*' $O/abc_${name}_${c}_$rep.log)"
    done
  done
done
unset DAT_LIB_PATH
echo done
