set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 13; }
grep '^{' gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/kt -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof/kt.log 2>&1 || { echo "profile failed"; tail -20 $R/gpurun_out/prof/kt.log; exit 14; }
cat $R/gpurun_out/prof/kt/run_kernel_stats.csv
