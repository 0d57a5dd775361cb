#!/bin/bash
# A/B of build variants (build_var/libdat_<v>.so) on the stall fixture and the C4 stall parity test.
#   VARIANTS="a b" bash tools/r06_stall_ab.sh
set -u
for v in ${VARIANTS:-base}; do
  DAT_LIB_PATH=$PWD/build_var/libdat_$v.so timeout -k 10 200 python -u tools/stall_fixture.py > gpurun_out/abst_$v.log 2>&1 || exit 11
  DAT_LIB_PATH=$PWD/build_var/libdat_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_c4_hard.py -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/abt_$v.log 2>&1; t=$?
  echo "$v: $(grep '^scenario' gpurun_out/abst_$v.log | tr '\n' ' ') tests rc $t"
done
