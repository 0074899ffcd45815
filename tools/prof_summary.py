#!/usr/bin/env python3
"""Summarise a tools/profile.sh output dir into profiles/<tag>_summary.md and update
profiles/pmc_summary.json (HBM bytes per k_match launch; a record, bench.py measures live)."""
import collections
import csv
import glob
import json
import os
import sys

tag, src = sys.argv[1], sys.argv[2]
key = sys.argv[3] if len(sys.argv) > 3 else "1920x1080_D128_w9_sad"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lines = [f"# rocprofv3 summary — {tag}", "", f"workload key: `{key}`", ""]
stats = glob.glob(f"{src}/trace/*kernel_stats.csv")
if stats:
    lines += ["## Kernel trace (`rocprofv3 --kernel-trace --stats`)", "",
              "| kernel | calls | avg µs | min µs | max µs | % |", "|---|---|---|---|---|---|"]
    for r in csv.DictReader(open(stats[0])):
        lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                     f"{float(r['MinNs'])/1e3:.2f} | {float(r['MaxNs'])/1e3:.2f} | {float(r['Percentage']):.1f} |")
    lines.append("")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for name in ("fetch", "write", "sq", "sq2", "lds"):
    for f in glob.glob(f"{src}/{name}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
if agg:
    lines += ["## PMC counters (separate `--pmc` passes; mean per dispatch)", "",
              "FETCH_SIZE / WRITE_SIZE are KiB per dispatch as reported (uncorrected).", ""]
    for k, d in agg.items():
        lines.append(f"### `{k}`")
        for c, v in sorted(d.items()):
            lines.append(f"- {c}: {sum(v)/len(v):,.1f} (n={len(v)})")
        lines.append("")
    pmc_path = os.path.join(root, "profiles", "pmc_summary.json")
    pmc = json.load(open(pmc_path)) if os.path.exists(pmc_path) else {}
    for k, d in agg.items():
        if "k_match" in k and "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            fetch = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) * 1024
            write = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) * 1024
            valu = d.get("SQ_INSTS_VALU")
            pmc[key] = {"hbm_bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch),
                        "write_bytes": round(write), "tag": tag,
                        "valu_insts_per_launch": round(sum(valu) / len(valu)) if valu else None,
                        "note": "FETCH_SIZE+WRITE_SIZE KiB x 1024, uncorrected: the x2 gfx950 read correction "
                                "applies to 16-B/lane streams; k_match reads dwords (uncalibrated, DESIGN.md)"}
    json.dump(pmc, open(pmc_path, "w"), indent=1)
out = os.path.join(root, "profiles", f"{tag}_summary.md")
open(out, "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
