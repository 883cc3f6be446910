"""Summarise rocprofv3 --pmc CSVs per kernel (tools/profile.sh output).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half
the bytes of wide coalesced streams on gfx950, so read bytes = 2 x
FETCH_SIZE x 1024 (an upper bound for narrower gathers); WRITE_SIZE x 1024.
FETCH_SIZE and WRITE_SIZE come from separate passes.

Kernels are keyed by their full template instantiation (k_extend<true, false, 0>
is the production extension kernel, k_extend<true, true, 0> the work-counting
one that bench.py's counted step runs): a summary never averages the two.

Lanes per VALU instruction = SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU (both
count the cycles of multi-cycle instructions; the round-4 quotient by
SQ_INSTS_VALU read 66 for kernels whose every lane is active). Calibration:
k_generate, k_accumulate and k_samp_reset read 64.00 with it (gpurun_out/prof_r04).
"""
import collections
import csv
import glob
import os
import re
import sys


def kernel_key(name):
    """'void wpt::(anonymous namespace)::k_extend<true, false, 0>(...)' ->
    'k_extend<true, false, 0>'; plain kernels -> their name."""
    m = re.search(r"(k_[a-z0-9_]+)(<[^<>()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else None


def load(prof_dir):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(int))
    for f in sorted(glob.glob(os.path.join(prof_dir, "pmc*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            if not k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k][r["Counter_Name"]] += 1
    return agg, disp


def bytes_per_launch(path_or_dir, kernel):
    d = path_or_dir if os.path.isdir(path_or_dir) else os.path.dirname(os.path.dirname(path_or_dir))
    agg, disp = load(d)
    a, n = agg[kernel], disp[kernel]
    if not n.get("FETCH_SIZE") or not n.get("WRITE_SIZE"):
        return None
    rd = 2.0 * a["FETCH_SIZE"] * 1024 / n["FETCH_SIZE"]
    wr = a["WRITE_SIZE"] * 1024 / n["WRITE_SIZE"]
    return rd + wr


def standalone_ms(prof_dir):
    """Per kernel: summed dispatch durations (ms) of the first counter pass,
    where rocprofv3 runs every dispatch alone."""
    out = collections.defaultdict(float)
    files = sorted(glob.glob(os.path.join(prof_dir, "pmc1", "*counter_collection.csv")))
    seen = set()
    for f in files[:1]:
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            if not k or (r["Dispatch_Id"], k) in seen:
                continue
            seen.add((r["Dispatch_Id"], k))
            out[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return dict(out)


def summary(prof_dir):
    agg, disp = load(prof_dir)
    out = {}
    for k, a in agg.items():
        n = disp[k]
        row = {"dispatches": max(n.values())}
        if a.get("SQ_INSTS_VALU"):
            row["valu_insts"] = a["SQ_INSTS_VALU"]
            row["salu_per_valu"] = a.get("SQ_INSTS_SALU", 0) / a["SQ_INSTS_VALU"]
        if a.get("SQ_THREAD_CYCLES_VALU") and a.get("SQ_ACTIVE_INST_VALU"):
            row["active_lanes_per_valu"] = a["SQ_THREAD_CYCLES_VALU"] / a["SQ_ACTIVE_INST_VALU"]
        if a.get("SQ_WAVE_CYCLES"):
            row["wait_frac"] = a.get("SQ_WAIT_ANY", 0) / a["SQ_WAVE_CYCLES"]
            row["active_frac"] = a.get("SQ_ACTIVE_INST_ANY", 0) / a["SQ_WAVE_CYCLES"] if a.get("SQ_ACTIVE_INST_ANY") else None
        if a.get("TCC_HIT_sum") is not None and (a.get("TCC_HIT_sum", 0) + a.get("TCC_MISS_sum", 0)) > 0:
            row["l2_hit"] = a["TCC_HIT_sum"] / (a["TCC_HIT_sum"] + a["TCC_MISS_sum"])
        if n.get("FETCH_SIZE"):
            row["hbm_read_bytes_per_launch"] = 2.0 * a["FETCH_SIZE"] * 1024 / n["FETCH_SIZE"]
        if n.get("WRITE_SIZE"):
            row["hbm_write_bytes_per_launch"] = a["WRITE_SIZE"] * 1024 / n["WRITE_SIZE"]
        out[k] = row
    return out


def raw(prof_dir):
    """Every counter per kernel: total and per-dispatch mean."""
    agg, disp = load(prof_dir)
    return {k: {c: {"total": v, "per_dispatch": v / max(disp[k][c], 1)} for c, v in a.items()} for k, a in agg.items()}


if __name__ == "__main__":
    import json
    if len(sys.argv) > 2 and sys.argv[2] == "raw":
        print(json.dumps(raw(sys.argv[1]), indent=1))
    else:
        print(json.dumps(summary(sys.argv[1]), indent=1))
