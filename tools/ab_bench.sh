#!/bin/bash
# A/B timing of differently compiled builds of libdat.so (build_var/libdat_<name>.so) on the C4
# bench (run on the GPU box via gpurun): one short bench per variant, JSON line per variant.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-base}; do
  DAT_LIB_PATH=$R/build_var/libdat_$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps ${STEPS:-6} --warmup ${WARMUP:-2} ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v.log; exit 11; }
  python - "$v" gpurun_out/ab_$v.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith('{')][-1]
j = json.loads(line)
print(f"{sys.argv[1]:>12}: {j['ms_per_step']:.3f} ms/step  k_cadmm {j['roofline']['launch_ms']:.3f} ms  {j['value']/1e6:.1f} M QP/s  ipm/qp {j['stats']['mean_ipm_iters_per_qp']:.2f}")
PY
done
