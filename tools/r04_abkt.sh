#!/bin/bash
# A/B of libdat builds by kernel trace: per build, rocprofv3 --kernel-trace --stats over the default bench;
# prints each kernel's mean and the bench's ms/step.  LIBS="name=path ...", REPS
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/abkt
O=$R/gpurun_out/abkt
export PYTHONUNBUFFERED=1
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $LIBS; do
    name=${spec%%=*}; path=${spec#*=}
    if [ -n "$path" ]; then export DAT_LIB_PATH=$R/$path; else unset DAT_LIB_PATH; fi
    d=$O/${name}_$rep
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline ${EXTRA:-} > $d.log 2>&1) || { tail -5 $d.log; exit 12; }
    echo "$name rep $rep: $(python tools/show_bench.py $d.log | head -1 | cut -c40-120)"
    python3 -c "
import csv,sys
for r in csv.DictReader(open('$d/run_kernel_stats.csv')):
    n=r['Name']
    if any(k in n for k in ('k_env_class','k_cadmm','k_rollout','k_bucket','k_dd')): print('   ', n.split('(')[0].split('::')[-1], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['MinNs'])/1e3,1), 'min')
"
  done
done
unset DAT_LIB_PATH
echo done
