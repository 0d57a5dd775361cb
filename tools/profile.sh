#!/bin/bash
# Profiling recipe used for profiles/ (run on the GPU box via gpurun).
# Pass 1: kernel trace + stats. Passes 2-4: PMC counters, one block per pass (no sys/runtime trace).
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
B=${B:-65536}
ARGS="$R/bench.py --steps 5 --warmup 1 --batch $B --no-cpu-baseline"
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $ARGS > $OUT/kt.log 2>&1 || exit 11
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_VALU --kernel-trace -d $OUT/pmc1 -o run --output-format csv -- python3 $ARGS > $OUT/pmc1.log 2>&1 || exit 12
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc2 -o run --output-format csv -- python3 $ARGS > $OUT/pmc2.log 2>&1 || exit 13
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc3 -o run --output-format csv -- python3 $ARGS > $OUT/pmc3.log 2>&1 || exit 14
echo done
