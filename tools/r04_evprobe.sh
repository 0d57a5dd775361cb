#!/bin/bash
# HIP-event vs device-clock vs kernel-trace timing (tools/event_probe.hip), and the bench with the
# runtime's scratch reclaim off
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/evp
O=$R/gpurun_out/evp
export PYTHONUNBUFFERED=1
timeout -k 10 60 ./tools/event_probe > $O/probe.log 2>&1 || { cat $O/probe.log; exit 11; }
cat $O/probe.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- $R/tools/event_probe > $O/probe_kt.log 2>&1) || { tail -5 $O/probe_kt.log; exit 12; }
for v in base noreclaim base noreclaim; do
  if [ $v = noreclaim ]; then export HSA_NO_SCRATCH_RECLAIM=1; else unset HSA_NO_SCRATCH_RECLAIM; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; exit 13; }
  echo "$v: $(python tools/show_bench.py $O/bench_$v.log | head -1 | cut -c1-160)"
done
