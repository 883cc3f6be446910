"""Copy a tools/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>/ and
write profiles/traffic_<config>.json, the per-launch HBM bytes bench.py reports
as roofline.traffic for the same workload.

Usage: python tools/collect_profile.py gpurun_out/prof_r01 r01 [config] [batch] [spp] [traversal] [lanes]
(hbm_bytes_per_launch is per DISPATCH; bench.py scales it by the lanes of a logical launch;
kernels are keyed by full instantiation, so the counting build's dispatches stay apart)
"""
import glob
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, tag = sys.argv[1], sys.argv[2]
    config = sys.argv[3] if len(sys.argv) > 3 else "c3"
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 27
    spp = int(sys.argv[5]) if len(sys.argv) > 5 else 64
    trav = sys.argv[6] if len(sys.argv) > 6 else "bvh2"
    lanes = int(sys.argv[7]) if len(sys.argv) > 7 else 4
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dst, f"{config}_kernel_stats.csv"))
    for f in ("trace.log", "args.txt"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f"{config}_{f}"))
    summ = pmc.summary(src)
    # counter passes serialise the dispatches: their durations are each
    # kernel's standalone time (one step + the counted step of bench.py)
    for k, ms in pmc.standalone_ms(src).items():
        if k in summ:
            summ[k]["standalone_ms_per_pass"] = ms
    json.dump(summ, open(os.path.join(dst, f"{config}_pmc_summary.json"), "w"), indent=1)
    kernels = {}
    for k, row in summ.items():
        if "hbm_read_bytes_per_launch" in row and "hbm_write_bytes_per_launch" in row:
            kernels[k] = {"hbm_bytes_per_launch": row["hbm_read_bytes_per_launch"] + row["hbm_write_bytes_per_launch"],
                          "read": row["hbm_read_bytes_per_launch"], "write": row["hbm_write_bytes_per_launch"]}
            if row.get("valu_insts") and row.get("active_lanes_per_valu"):
                # SQ_INSTS_VALU per dispatch and SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU (one pass)
                kernels[k]["valu_insts_per_launch"] = row["valu_insts"] / row["dispatches"]
                kernels[k]["active_lanes_per_valu"] = row["active_lanes_per_valu"]
    meta = {"config": config, "batch": batch, "spp": spp, "gpus": 1, "traversal": trav, "lanes": lanes,
            "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, profiles/{tag}/", "kernels": kernels}
    json.dump(meta, open(os.path.join(ROOT, "profiles", f"traffic_{config}.json"), "w"), indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
