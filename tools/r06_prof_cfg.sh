#!/bin/bash
# Round-6 kernel trace + PMC of the critical-path lines (tools/profile.sh per config) and of the stall fixture's
# tail kernel (kernel trace + one PMC pass), under gpurun_out/prof_<name>.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
for c in C2 C3; do
  OUT=$R/gpurun_out/prof_$c B=default EXTRA="--config $c" bash tools/profile.sh || exit 11
done
O=$R/gpurun_out/prof_stall
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/tools/stall_fixture.py > $O/kt.log 2>&1) || exit 12
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc4 -o run --output-format csv -- python3 $R/tools/stall_fixture.py > $O/pmc4.log 2>&1) || exit 13
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU --kernel-trace -d $O/pmc5 -o run --output-format csv -- python3 $R/tools/stall_fixture.py > $O/pmc5.log 2>&1) || exit 14
echo done
