#!/bin/bash
# Profiling recipe used for profiles/ (run on the GPU box via gpurun).
# Pass 1: kernel trace + stats.  Passes 2-5: PMC counters, one counter block per pass, no
# sys/runtime trace (MI355X_MICROARCH.md "rocprofv3 PMC slots").
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=${OUT:-$R/gpurun_out/prof}
mkdir -p $OUT
B=${B:-65536}
# B=default: the bench's own default workload (65,536 scenarios, strong split), whose workload string
# profiles/traffic.json is keyed on
BATCH_ARG="--batch $B"; [ "$B" = "default" ] && BATCH_ARG=""
ARGS="$R/bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-2} $BATCH_ARG --no-cpu-baseline --sustained-steps 0 ${EXTRA:-}"
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $ARGS > $OUT/kt.log 2>&1 || exit 11
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d $OUT/pmc1 -o run --output-format csv -- python3 $ARGS > $OUT/pmc1.log 2>&1 || exit 12
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc2 -o run --output-format csv -- python3 $ARGS > $OUT/pmc2.log 2>&1 || exit 13
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc3 -o run --output-format csv -- python3 $ARGS > $OUT/pmc3.log 2>&1 || exit 14
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc4 -o run --output-format csv -- python3 $ARGS > $OUT/pmc4.log 2>&1 || exit 15
# pass 6 (optional): LDS / vector-memory instruction mix (scratch spills are VMEM); names checked against -L
if grep -q "SQ_INSTS_VMEM_RD" $OUT/counters_list.txt 2>/dev/null; then
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU --kernel-trace -d $OUT/pmc5 -o run --output-format csv -- python3 $ARGS > $OUT/pmc5.log 2>&1 || echo "pass 6 failed"
fi
echo done
