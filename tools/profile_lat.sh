#!/bin/bash
# Latency / issue PMC passes (gpurun): LDS and vector-memory latency (SQ_INST_LEVEL_x / SQ_INSTS_x),
# issue-busy cycles by unit and lane-level VALU cycles, one counter block per pass.
#   CFG=C4|C2|C3|C5 bash tools/profile_lat.sh   -> gpurun_out/prof_lat_<CFG>/pmc{a,b}
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
CFG=${CFG:-C4}
OUT=$R/gpurun_out/prof_lat_$CFG
mkdir -p $OUT
ARGS="$R/bench.py --config $CFG --steps ${STEPS:-3} --warmup ${WARMUP:-2} --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --kernel-trace -d $OUT/pmca -o run --output-format csv -- python3 $ARGS > $OUT/pmca.log 2>&1 || exit 11
timeout -s KILL 240 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY --kernel-trace -d $OUT/pmcb -o run --output-format csv -- python3 $ARGS > $OUT/pmcb.log 2>&1 || exit 12
echo "profile_lat $CFG done"
