#!/bin/bash
# PMC A/B of build variants (build_var/libdat_<v>.so) on the C4 bench (run on the GPU box): instruction mix,
# waits and instruction-cache counters of k_cadmm per variant.  VARIANTS="base new" bash tools/pmc_ab.sh
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmcab
mkdir -p $OUT
for v in ${VARIANTS:-base}; do
  export DAT_LIB_PATH=$R/build_var/libdat_$v.so
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace -d $OUT/${v}_a -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/${v}_a.log 2>&1 || exit 11
  timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_BUSY_CYCLES --kernel-trace -d $OUT/${v}_b -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/${v}_b.log 2>&1 || exit 12
done
echo done
