#!/bin/bash
# A/B/C of libdat builds on the C4 bench, interleaved on one box: LIBS="name=path ..." (path "" = in-tree)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
O=gpurun_out
export PYTHONUNBUFFERED=1
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $LIBS; do
    name=${spec%%=*}; path=${spec#*=}
    if [ -n "$path" ]; then export DAT_LIB_PATH=$R/$path; else unset DAT_LIB_PATH; fi
    for B in ${BATCHES:-65536}; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch $B --steps ${STEPS:-20} ${EXTRA:-} > $O/ab3_${name}_${B}_$rep.log 2>&1 || { tail -20 $O/ab3_${name}_${B}_$rep.log; exit 12; }
      echo "$name B=$B rep $rep: $(python tools/show_bench.py $O/ab3_${name}_${B}_$rep.log | head -1 | cut -c1-170)"
    done
  done
done
unset DAT_LIB_PATH
echo done
