#!/bin/bash
# Counters of the lone-wave stall case (tools/stall_latency.py): instruction mix and wait cycles per IPM iteration.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/stallprof
mkdir -p $OUT
ARGS="$R/tools/stall_latency.py $R/scratch/c4_stall_states.npz 0 3"
timeout -k 10 120 python3 $ARGS > $OUT/plain.log 2>&1 || exit 11
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $ARGS > $OUT/kt.log 2>&1 || exit 12
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --kernel-trace -d $OUT/pmc1 -o run --output-format csv -- python3 $ARGS > $OUT/pmc1.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --kernel-trace -d $OUT/pmc2 -o run --output-format csv -- python3 $ARGS > $OUT/pmc2.log 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_EXP --kernel-trace -d $OUT/pmc3 -o run --output-format csv -- python3 $ARGS > $OUT/pmc3.log 2>&1 || echo "pmc3 failed"
echo done
