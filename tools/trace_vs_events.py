"""The bench's HIP-event k_cadmm time next to rocprofv3's kernel trace of the same run.

    python tools/trace_vs_events.py <run_kernel_trace.csv> <bench log> [kernel]

The bench runs `warmup` launches, then the `steps` timed ones, then one metrics-only step; the timed
launches are therefore trace launches [warmup, warmup + steps) of the kernel.
"""
import csv
import json
import sys

trace, log = sys.argv[1], sys.argv[2]
kernel = sys.argv[3] if len(sys.argv) > 3 else "k_cadmm"
d = json.loads([ln for ln in open(log) if ln.startswith("{")][-1])
rows = sorted((r for r in csv.DictReader(open(trace)) if kernel in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
per = d["roofline"].get("launches_per_step", 1)
w, k = d["warmup"] * per, d["steps"] * per
timed = dur[w:w + k]
print(json.dumps({"launches_in_trace": len(dur), "timed_launches": len(timed),
                  "trace_mean_ms": sum(timed) / max(len(timed), 1), "event_launch_ms": d["roofline"]["launch_ms"],
                  "ms_per_step": d["ms_per_step"], "all_launches_ms": [round(x, 3) for x in dur]}))
