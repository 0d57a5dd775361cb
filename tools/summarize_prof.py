"""Summarise a tools/profile.sh output directory (gpurun_out/prof) into profiles/<tag>_*.

    python tools/summarize_prof.py gpurun_out/prof r01_v1

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim) and profiles/<tag>_pmc.md
(per-kernel counter sums and per-dispatch means, with the gfx950 FETCH_SIZE x2 correction of
MI355X_MICROARCH.md applied in a separate column).
"""

import collections
import csv
import os
import shutil
import sys


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "profiles")
    os.makedirs(dst, exist_ok=True)
    ks = os.path.join(src, "kt", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    lines = [f"# PMC summary {tag}", "",
             "Sums over all dispatches of each kernel in the profiled `bench.py` run; FETCH_SIZE/WRITE_SIZE in KB "
             "as rocprofv3 reports them; `FETCH_SIZE x2` applies the gfx950 correction (MI355X_MICROARCH.md).", "",
             "| kernel | counter | dispatches | sum | mean / dispatch |", "|---|---|---|---|---|"]
    res = {}
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not p.startswith("pmc") or not os.path.exists(f):
            continue
        agg = collections.defaultdict(float)
        cnt = collections.defaultdict(set)
        meta = {}
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")
            if "anonymous" in r["Kernel_Name"]:
                k = r["Kernel_Name"].split("::")[1].split("(")[0]
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            cnt[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
            meta[k] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
        for (k, c), v in sorted(agg.items()):
            nd = len(cnt[(k, c)])
            lines.append(f"| {k} | {c} | {nd} | {v:.6g} | {v / nd:.6g} |")
            res[(k, c)] = (v, nd)
            if c == "FETCH_SIZE":
                lines.append(f"| {k} | FETCH_SIZE x2 | {nd} | {2 * v:.6g} | {2 * v / nd:.6g} |")
    lines += ["", "| kernel | VGPR | AGPR | SGPR | LDS | scratch |", "|---|---|---|---|---|---|"]
    for k, m in sorted(meta.items()):
        lines.append(f"| {k} | " + " | ".join(m) + " |")
    open(os.path.join(dst, f"{tag}_pmc.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
