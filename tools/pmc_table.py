"""Per-kernel sums of rocprofv3 --pmc counter CSVs (one directory per pass).
Usage: python tools/pmc_table.py gpurun_out/pmc_<tag>  -> JSON {kernel: {counter: sum, 'dispatches': n}}"""
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"(k_[a-z_0-9]+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def table(root):
    out = {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        seen = {}
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            d = out.setdefault(k, {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            seen.setdefault(k, set()).add(r["Dispatch_Id"])
        for k, s in seen.items():
            out[k]["dispatches"] = max(out[k].get("dispatches", 0), len(s))
    return out


if __name__ == "__main__":
    t = table(sys.argv[1])
    keys = sys.argv[2:] or None
    for k, d in sorted(t.items()):
        if keys and not any(x in k for x in keys):
            continue
        print(k, json.dumps({c: round(v, 3) for c, v in sorted(d.items())}))
