"""Device memory left after each of R init/compute/shutdown cycles of a
session_rate.py session (a leak across shutdown shows as a falling `free`).
usage: python tools/mem_cycle.py [session] [--reps 10] [--spp 2]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import session_rate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("session", nargs="?", default="init")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--spp", type=int, default=2)
    a = ap.parse_args()
    import torch
    pkg = session_rate.wpt_loader.load()
    itf = pkg.interface
    itf.set_device(0)
    cloud = pkg.scenes.triangle_cloud(100000)
    for k in range(a.reps):
        t = time.perf_counter()
        r = session_rate.run(itf, pkg, cloud, a.session, [], a.spp)
        free, total = torch.cuda.mem_get_info(0)
        print(json.dumps({"cycle": k, "s": round(time.perf_counter() - t, 3), "window_s": r["s"],
                          "free_GiB": round(free / 2**30, 2), "total_GiB": round(total / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
