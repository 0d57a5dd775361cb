#!/bin/bash
# Small-batch diagnosis (run on the GPU box): kernel trace + cycle counters of the C2 fixed-work
# bench at B = 1024 and at B = 16384 (same code path, 16x the wavefronts).
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/psmall
mkdir -p $OUT
for B in 1024 16384; do
  ARGS="$R/bench.py --config C2 --fixed-work --no-cpu-baseline --steps 4 --warmup 1 --batch $B"
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/b$B -o run --output-format csv -- python3 $ARGS > $OUT/b$B.log 2>&1 || exit 11
  grep '^{' $OUT/b$B.log | cut -c1-400
done
echo done
