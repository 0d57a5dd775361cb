#!/bin/bash
# Slot-count sweep (dat_set_persistent_blocks: more resident workgroups hold fewer scenario slots each) on the
# critical-path-bound lines: C2, C3 and the 8,192-scenario C4 shard (one rank's share of configs[3] on 8 GPUs).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
O=gpurun_out/slots.jsonl
: > $O
for pb in ${PBS:-0 2048 4096}; do
  for c in ${CFGS:-C2 C3 C4s}; do
    if [ $c = C4s ]; then a="--batch 8192"; else a="--config $c"; fi
    timeout -k 10 200 python -u bench.py $a --persistent-blocks $pb --no-cpu-baseline --sustained-steps 0 --steps ${STEPS:-10} > gpurun_out/slots_${c}_${pb}.log 2>&1 || { tail -5 gpurun_out/slots_${c}_${pb}.log; exit 11; }
    grep '^{' gpurun_out/slots_${c}_${pb}.log >> $O
    python - "$c" "$pb" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/slots.jsonl").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>4} pb {sys.argv[2]:>5}: {d['ms_per_step']:.3f} ms/step (p50 {d.get('ms_per_step_p50')})")
PY
  done
done
