"""Summarise rocprofv3 PMC passes (scripts/gpu_profile.sh output) per kernel.

    python scripts/pmc_summary.py gpurun_out/prof > profiles/<round>/pmc_<workload>.json

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch;
on gfx950 FETCH_SIZE counts half the bytes of 128-B line fills
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section), so hbm_bytes applies
the x2 correction to FETCH_SIZE and none to WRITE_SIZE.
"""
import collections
import csv
import glob
import json
import os
import sys


def summarise(root):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            per[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, d in per.items():
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        e = {"dispatches": max(len(v) for v in d.values()), "avg": avg}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["hbm_bytes_per_dispatch"] = 2 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024
        out[k] = e
    return out


if __name__ == "__main__":
    print(json.dumps(summarise(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"), indent=1, sort_keys=True))
