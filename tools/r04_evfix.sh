#!/bin/bash
# bench lines with the metrics step outside the k_cadmm event time, and a kernel trace of the same command
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/evf
O=$R/gpurun_out/evf
export PYTHONUNBUFFERED=1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || { tail -5 $O/bench_$i.log; exit 11; }
  python tools/show_bench.py $O/bench_$i.log | head -1
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/kt.log 2>&1) || { tail -5 $O/kt.log; exit 12; }
python tools/trace_vs_events.py $O/kt/run_kernel_trace.csv $O/kt.log
