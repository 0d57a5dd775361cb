#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
O=gpurun_out
export PYTHONUNBUFFERED=1
for sb in 0 512 1024; do
  if [ "$sb" = "0" ]; then unset DAT_SLOT_BLOCKS; else export DAT_SLOT_BLOCKS=$sb; fi
  timeout -k 10 300 python -u bench.py --config C2 --fused --steps 10 --no-cpu-baseline > $O/c2f_$sb.log 2>&1 || { tail -20 $O/c2f_$sb.log; exit 12; }
  echo "C2 fused slot_blocks=$sb: $(python tools/show_bench.py $O/c2f_$sb.log | head -1 | cut -c20-140)"
done
unset DAT_SLOT_BLOCKS
timeout -k 10 400 python -u tools/c4_long_run.py 1000 100 > $O/c4_long.log 2>&1 || { tail -20 $O/c4_long.log; exit 13; }
tail -3 $O/c4_long.log
