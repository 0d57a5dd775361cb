#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
O=gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_hard_stretch.py tests/test_gpu_dropin.py -q -x --timeout 300 --timeout-method thread > $O/retry_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/retry_tests.log | cut -c1-300 | tail -20; exit 11; }
tail -1 $O/retry_tests.log
for rep in 1 2; do
for spec in prev=build_var/libdat_lds4.so new=; do
  name=${spec%%=*}; path=${spec#*=}
  if [ -n "$path" ]; then export DAT_LIB_PATH=$R/$path; else unset DAT_LIB_PATH; fi
  for c in C4 C1 C3; do
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/retry_${name}_$c.log 2>&1 || { tail -30 $O/retry_${name}_$c.log; exit 14; }
    echo "$name $c: $(python tools/show_bench.py $O/retry_${name}_$c.log | head -1 | cut -c20-140) $(grep -o '"inband_beyond[^,}]*' $O/retry_${name}_$c.log)"
  done
done
done
unset DAT_LIB_PATH
timeout -k 10 300 python -u bench.py --config C5 --no-cpu-baseline > $O/retry_C5.log 2>&1 || { tail -30 $O/retry_C5.log; exit 15; }
echo "new C5: $(python tools/show_bench.py $O/retry_C5.log | head -1 | cut -c20-140) $(grep -o '"inband_beyond[^,}]*' $O/retry_C5.log)"
