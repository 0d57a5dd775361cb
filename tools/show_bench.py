"""Print the headline numbers and per-class stats of bench logs (development helper)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    except Exception as e:  # noqa: BLE001
        print(f, "no result:", e)
        continue
    r = d["roofline"]
    print(f"{f}: value {d['value']:.4g} ms/step {d['ms_per_step']:.3f} kernel {r['kernel']} {r['launch_ms']:.3f} ms "
          f"frac {r['frac']:.4f} ipm/qp {d['stats']['mean_ipm_iters_per_qp']:.3f}")
    for k, v in (d["stats"].get("env_classes") or {}).items():
        print("   ", k, {a: (round(b, 3) if isinstance(b, float) else b) for a, b in v.items()})
