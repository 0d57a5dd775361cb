#!/bin/bash
# Counters of the lone-wave stall case (tools/stall_fixture.py: the two C4 stall stretches, each scenario alone):
# kernel trace, then instruction mix and wait cycles of k_cadmm_tail / k_cadmm per dispatch (one PMC pass each).
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/stallprof${TAG:-}
mkdir -p $OUT
ARGS="$R/tools/stall_fixture.py"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $ARGS > $OUT/kt.log 2>&1 || exit 12
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --kernel-trace -d $OUT/pmc1 -o run --output-format csv -- python3 $ARGS > $OUT/pmc1.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --kernel-trace -d $OUT/pmc2 -o run --output-format csv -- python3 $ARGS > $OUT/pmc2.log 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU --kernel-trace -d $OUT/pmc3 -o run --output-format csv -- python3 $ARGS > $OUT/pmc3.log 2>&1 || echo "pmc3 failed"
echo done
