#!/bin/bash
# Kernel trace + PMC passes of one QP-level bench configuration (gpurun):
#   CFG=C3 B=16384 bash tools/profile_cfg.sh   -> gpurun_out/prof_<CFG>/{kt,pmc1..5} (tools/summarize_prof.py)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
CFG=${CFG:-C3}
OUT=$R/gpurun_out/prof_$CFG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --config $CFG --batch ${B:-16384} --steps ${STEPS:-4} --warmup ${WARMUP:-2} --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $ARGS > $OUT/kt.log 2>&1 || exit 11
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d $OUT/pmc1 -o run --output-format csv -- python3 $ARGS > $OUT/pmc1.log 2>&1 || exit 12
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc2 -o run --output-format csv -- python3 $ARGS > $OUT/pmc2.log 2>&1 || exit 13
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc3 -o run --output-format csv -- python3 $ARGS > $OUT/pmc3.log 2>&1 || exit 14
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc4 -o run --output-format csv -- python3 $ARGS > $OUT/pmc4.log 2>&1 || exit 15
timeout -s KILL 240 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --kernel-trace -d $OUT/pmc5 -o run --output-format csv -- python3 $ARGS > $OUT/pmc5.log 2>&1 || exit 16
echo "profile_cfg $CFG done"
