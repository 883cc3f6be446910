"""One warm-up and N production steps of a bench config, nothing else (a
short program for rocprofv3 PC sampling / counter passes).
Usage: python tools/one_step.py [c3|c5|museum|c2] [steps] [lanes]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (CONFIGS only)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    lanes = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    import wpt_loader

    pkg = wpt_loader.load()
    itf = pkg.interface
    cfg = bench.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    itf.init(W, H, cfg["scene"], *pkg.scenes.scene_camera(cfg["scene"]))
    if cfg["mesh"]:
        itf.store_mesh(1, pkg.scenes.triangle_cloud(cfg["mesh"]))
    ad = cfg.get("adaptive", 0)
    itf.update_settings(cfg["nee"], cfg["nee"], ad, ad, 0)
    itf.set_render_options(cfg["depth"], 0xBABABEBE, 1 << 27)
    if lanes:
        itf.set_lanes(lanes)
    n = W * H * cfg["spp"]
    itf.compute(n)
    itf.sync()
    itf.clear_stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        itf.compute(n)
    itf.sync()
    dt = time.perf_counter() - t0
    st = itf.stats()
    print(f"{name} lanes={itf.get_option('lanes')} {steps} steps {dt * 1e3 / steps:.2f} ms/step "
          f"{(st['rays'] + st['shadow_rays']) / dt / 1e6:.1f} Mray/s")
    itf.shutdown()


if __name__ == "__main__":
    main()
