#!/bin/bash
# A/B of build variants (build_var/libdat_<v>.so) on the two tail measures: the stall stretches alone
# (tools/stall_fixture.py) and the bench's 10 s sustained loop (no CPU baseline).   VARIANTS="a b" bash tools/r06_ab.sh
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-base}; do
  DAT_LIB_PATH=$R/build_var/libdat_$v.so timeout -k 10 200 python -u tools/stall_fixture.py > gpurun_out/abst_$v.log 2>&1 || { echo "$v stall failed"; tail -5 gpurun_out/abst_$v.log; exit 11; }
  echo "$v: $(grep '^scenario' gpurun_out/abst_$v.log | tr '\n' ' ')"
  DAT_LIB_PATH=$R/build_var/libdat_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 > gpurun_out/abb_$v.json 2> gpurun_out/abb_$v.err || { echo "$v bench failed"; tail -5 gpurun_out/abb_$v.err; exit 12; }
  python - "$v" gpurun_out/abb_$v.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
s = d["stats"]["sustained"]
print(f"{sys.argv[1]:>8}: {d['ms_per_step']:.3f} ms/step, sustained {s['ms_per_step']:.1f} avg / {s['slowest_block_ms_per_step']:.1f} slowest,"
      f" blocks {[round(b['ms_per_step'], 1) for b in s['blocks']]}, loose {s['inband_beyond_clarabel_tol']}")
PY
done
