#!/bin/bash
# Instruction-cache counters of k_cadmm (run on the GPU box): C4 and C2 at two slot packings.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pic
mkdir -p $OUT
run() {  # tag, bench args
  local tag=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ --kernel-trace -d $OUT/${tag}_a -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > $OUT/${tag}_a.log 2>&1 || return 1
  timeout -s KILL 200 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace -d $OUT/${tag}_b -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > $OUT/${tag}_b.log 2>&1 || return 1
}
run c4 || exit 11
run c2 --config C2 --fixed-work || exit 12
DAT_SLOT_BLOCKS=1024 run c2s --config C2 --fixed-work || exit 13
echo done
