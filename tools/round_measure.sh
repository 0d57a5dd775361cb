#!/bin/bash
# End-of-milestone measurement on the GPU box: default bench (C4, with the CPU baseline), the
# SURVEY 8(d) config lines, then the profiling recipe (kernel trace + PMC passes, tools/profile.sh).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_C4.log 2>&1 || { tail -20 gpurun_out/bench_C4.log; exit 11; }
grep '^{' gpurun_out/bench_C4.log
# the 8,192-scenario shard a rank of BASELINE configs[3] (65,536 across 8 GPUs) runs
timeout -k 10 200 python -u bench.py --batch 8192 --no-cpu-baseline > gpurun_out/bench_C4_8192.log 2>&1 || { tail -20 gpurun_out/bench_C4_8192.log; exit 14; }
grep '^{' gpurun_out/bench_C4_8192.log
TESTS=0 CPU_S=${CPU_S:-8} bash tools/configs_gpu.sh || exit 12
bash tools/profile.sh || exit 13
echo done
