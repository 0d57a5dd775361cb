#!/bin/bash
# Kernel trace of one bench configuration + an LDS conflict pass (gpurun):  CFG=C3 bash tools/quick_prof.sh
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
CFG=${CFG:-C4}
OUT=$R/gpurun_out/qp_$CFG
mkdir -p $OUT
ARGS="$R/bench.py --config $CFG --steps ${STEPS:-3} --warmup ${WARMUP:-2} --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $ARGS > $OUT/kt.log 2>&1 || exit 11
cat $OUT/kt/run_kernel_stats.csv | cut -d, -f1-4
if [ "${LDS:-0}" = "1" ]; then
  timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAVES --kernel-trace -d $OUT/pmcl -o run --output-format csv -- python3 $ARGS > $OUT/pmcl.log 2>&1 || exit 12
fi
