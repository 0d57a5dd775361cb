set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4_hard.py tests/test_gpu_c4.py tests/test_gpu_drain.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_t2.log 2>&1 || { tail -30 gpurun_out/gpu_tests_t2.log; exit 11; }
tail -1 gpurun_out/gpu_tests_t2.log
timeout -k 10 300 python -u tools/stall_fixture.py gpurun_out/stall_t2.json > gpurun_out/stall_t2.log 2>&1 || { tail -20 gpurun_out/stall_t2.log; exit 13; }
grep "^scenario" gpurun_out/stall_t2.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_t2.json 2> gpurun_out/bench_t2.err || { tail -20 gpurun_out/bench_t2.err; exit 15; }
DAT_LIB_PATH=$R/build_var/libdat_notail.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_notail.json 2> gpurun_out/bench_notail.err || { tail -20 gpurun_out/bench_notail.err; exit 16; }
echo done
