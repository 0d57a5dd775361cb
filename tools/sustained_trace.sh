#!/bin/bash
# Kernel trace of the bench's 10 s sustained loop (per-step composition of the late regime: k_cadmm, the
# concurrent tail launch, the hand-over tail launch).  Output under gpurun_out/sust_kt.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/sust_kt -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 > $R/gpurun_out/sust_kt.log 2>&1 || exit 12
echo done
