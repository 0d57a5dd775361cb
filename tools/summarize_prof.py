"""Summarise a tools/profile.sh output directory (gpurun_out/prof) into profiles/<tag>_*.

    python tools/summarize_prof.py gpurun_out/prof r01_v3 ["<bench workload string>"]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats of the kernel-trace pass, verbatim
  profiles/<tag>_pmc.md             per-kernel counter sums and per-dispatch means, the gfx950
                                    FETCH_SIZE x2 correction of MI355X_MICROARCH.md in its own
                                    column, and per-dispatch medians (the median drops the cold
                                    first control step of the closed loop, which runs many more
                                    ADMM iterations than the steady-state steps the bench times)
  profiles/traffic.json             (with a workload string) HBM bytes per launch of each kernel,
                                    median over dispatches of 2 x FETCH_SIZE + WRITE_SIZE, read by
                                    bench.py for roofline.traffic
"""

import collections
import csv
import json
import os
import shutil
import statistics
import sys


def kname(raw: str) -> str:
    if "anonymous namespace" in raw:
        return raw.split("::")[1].split("(")[0]
    return raw.split("(")[0]


def main():
    src, tag = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else None
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "profiles")
    os.makedirs(dst, exist_ok=True)
    ks = os.path.join(src, "kt", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    lines = [f"# PMC summary {tag}", "",
             "Counters per kernel over all dispatches of the profiled `bench.py` run (recipe: `tools/profile.sh`). "
             "FETCH_SIZE / WRITE_SIZE in KB as rocprofv3 reports them; `FETCH_SIZE x2` applies the gfx950 "
             "correction (MI355X_MICROARCH.md, HBM section). SQ_* cycle counters are in quad-cycles.", "",
             "| kernel | counter | dispatches | sum | mean / dispatch | median / dispatch |",
             "|---|---|---|---|---|---|"]
    med = {}
    meta = {}
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not p.startswith("pmc") or not os.path.exists(f):
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k.startswith("__amd_rocclr"):
                continue
            per[(k, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
            meta[k] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
        for (k, c), d in sorted(per.items()):
            vals = list(d.values())
            s, m = sum(vals), statistics.median(vals)
            med[(k, c)] = m
            lines.append(f"| {k} | {c} | {len(vals)} | {s:.6g} | {s / len(vals):.6g} | {m:.6g} |")
            if c == "FETCH_SIZE":
                lines.append(f"| {k} | FETCH_SIZE x2 | {len(vals)} | {2 * s:.6g} | {2 * s / len(vals):.6g} | {2 * m:.6g} |")
    # durations from the kernel-trace pass
    tr = os.path.join(src, "kt", "run_kernel_trace.csv")
    dur = collections.defaultdict(list)
    if os.path.exists(tr):
        for r in csv.DictReader(open(tr)):
            dur[kname(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    # bench.py launches each per-step kernel once per step: warmup launches, then the timed ones
    w0, nk = int(os.environ.get("WARMUP", "2")), int(os.environ.get("STEPS", "5"))
    lines += ["", f"Durations from the kernel-trace pass; `timed mean` = mean over launches {w0}..{w0 + nk - 1} "
                  f"(the bench's timed steps with --warmup {w0} --steps {nk}; compare with the bench line's "
                  "roofline.launch_ms).", "",
              "| kernel | dispatches | mean ms | timed mean ms | median ms | min ms | max ms |",
              "|---|---|---|---|---|---|---|"]
    for k, v in sorted(dur.items()):
        if k.startswith("__amd_rocclr"):
            continue
        tv = v[w0:w0 + nk] or v
        lines.append(f"| {k} | {len(v)} | {statistics.mean(v):.4f} | {statistics.mean(tv):.4f} | "
                     f"{statistics.median(v):.4f} | {min(v):.4f} | {max(v):.4f} |")
    lines += ["", "| kernel | VGPR | AGPR | SGPR | LDS | scratch |", "|---|---|---|---|---|---|"]
    for k, m in sorted(meta.items()):
        lines.append(f"| {k} | " + " | ".join(m) + " |")
    traffic = {}
    for k in sorted({k for k, _ in med}):
        if (k, "FETCH_SIZE") in med and (k, "WRITE_SIZE") in med:
            b = (2.0 * med[(k, "FETCH_SIZE")] + med[(k, "WRITE_SIZE")]) * 1024.0
            traffic[k] = {"bytes_per_launch": b, "median_ms": statistics.median(dur[k]) if dur.get(k) else None}
    if traffic:
        lines += ["", "HBM bytes per launch (median over dispatches of 2 x FETCH_SIZE + WRITE_SIZE):", ""]
        for k, t in traffic.items():
            lines.append(f"- {k}: {t['bytes_per_launch'] / 1e6:.2f} MB")
    open(os.path.join(dst, f"{tag}_pmc.md"), "w").write("\n".join(lines) + "\n")
    if workload and traffic:
        out = {k: dict(t, workload=workload, source=f"profiles/{tag}_pmc.md") for k, t in traffic.items()}
        with open(os.path.join(dst, "traffic.json"), "w") as f:
            json.dump(out, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
