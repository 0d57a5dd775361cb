#!/bin/bash
# Round-6 final measurement on the GPU box, two calls:
#   PART=A  parity suite (-m gpu) + smoke, the default bench line (C4, 10 s sustained loop, CPU baseline), the
#           8,192-scenario shard, the stall-stretch latency + its kernel trace
#   PART=B  the QP-level config lines (C2, C3, C5) and the profiling recipe (tools/profile.sh: kernel trace + PMC)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${PART:-A}" = "A" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=10 --timeout 300 --timeout-method thread > gpurun_out/f_gpu_tests.log 2>&1 || { tail -30 gpurun_out/f_gpu_tests.log; exit 11; }
  tail -1 gpurun_out/f_gpu_tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1 || { cat gpurun_out/f_smoke.log; exit 12; }
  tail -1 gpurun_out/f_smoke.log
  timeout -k 10 400 python -u bench.py > gpurun_out/f_bench.json 2> gpurun_out/f_bench.err || { tail -20 gpurun_out/f_bench.err; exit 13; }
  python tools/show_bench.py gpurun_out/f_bench.json || true
  timeout -k 10 200 python -u bench.py --batch 8192 --no-cpu-baseline --sustained-steps 0 --steps 20 > gpurun_out/f_shard.json 2> gpurun_out/f_shard.err || { tail -20 gpurun_out/f_shard.err; exit 14; }
  timeout -k 10 200 python -u tools/stall_fixture.py gpurun_out/f_stall.json > gpurun_out/f_stall.log 2>&1 || { tail -20 gpurun_out/f_stall.log; exit 15; }
  grep '^scenario' gpurun_out/f_stall.log
else
  TESTS=0 CPU_S=${CPU_S:-8} bash tools/configs_gpu.sh || exit 21
  bash tools/profile.sh || exit 22
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f_stall_kt -o run --output-format csv -- python3 $R/tools/stall_fixture.py > $R/gpurun_out/f_stall_kt.log 2>&1) || exit 23
fi
echo done
