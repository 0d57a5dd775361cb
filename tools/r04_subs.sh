#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
O=gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2; do
for B in ${BATCHES:-65536 8192}; do
  for sb in ${SUBS:-1 2 3}; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch $B --sub-batches $sb --steps ${STEPS:-20} > $O/subs_${B}_$sb.log 2>&1 || { tail -20 $O/subs_${B}_$sb.log; exit 12; }
    echo "B=$B sub=$sb rep $rep: $(python tools/show_bench.py $O/subs_${B}_$sb.log | head -1 | cut -c30-120)"
  done
done
done
