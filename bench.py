"""Benchmark: Mray/s (primary + shadow + bounce) of the path-tracing core.

Workload (BASELINE.json configs[2], "C3"): bunny scene (scene id 2) with mesh
slot 1 = seeded 100k-triangle cloud (stand-in for the missing bunny2.obj,
SURVEY §0 F2), 1920x1080, 64 spp per GPU share, depth cap 8, NormalNEE.
One step = one pass of the path loop over the step's paths with inputs
resident in HBM: generate -> [extend -> shade -> shadow] x8 -> accumulate.

Multi-GPU (one process per GPU: under torchrun, or `--gpus N` alone, which
spawns its N ranks itself, launch_ranks): the frame is tile-partitioned
(16x16 tiles, tile t -> rank t % N); every rank traces
64*N spp over its own tiles, so per-GPU work is fixed (weak scaling) and the
N-GPU job renders the 1080p frame at 64*N spp. The partitions are gathered to
rank 0 over RCCL (torch.distributed, backend nccl) at the end of every step.

value = rays traced by all ranks / max-over-ranks wall time of the K steps.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: scene, W, H, spp per GPU share, depth, render type
    "c3": dict(name="bunny scene", scene=2, W=1920, H=1080, spp=64, depth=8, nee=1, mesh=100000),
    "c2": dict(name="sphere+plane scene, no BVH", scene=101, W=1920, H=1080, spp=64, depth=4, nee=1, mesh=0),
    "c1": dict(name="Cornell box", scene=100, W=256, H=256, spp=1, depth=1, nee=1, mesh=0),
    # C5: PNEE (300k-photon octree) + adaptive sampling on both halves, 1024
    # spp budget; on N GPUs the ranks exchange the frame at round boundaries
    # and split each global round by tiles (strong scaling)
    "c5": dict(name="bunny scene PNEE + adaptive", scene=2, W=1920, H=1080, spp=1024, depth=8, nee=2, mesh=100000,
               adaptive=1),
    # the reference's default scene (index.ts:42): 27 tori (f64 quartic), 108 lights
    "museum": dict(name="museum scene", scene=0, W=1920, H=1080, spp=64, depth=8, nee=1, mesh=0),
    "c4": dict(name="bunny scene 4K", scene=2, W=3840, H=2160, spp=256, depth=8, nee=1, mesh=100000),
}
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
# wpt_get_option(WPT_OPT_SCENE_TRAVERSAL): what the session's scene runs
TRAVERSAL_NAMES = {0: "bvh2", 1: "bvh4", 2: "linear"}
PEAK_VALU_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 256 CU x 4 SIMD32 x 2.4 GHz lane-ops (78.6 T/s)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _host_threads():
    """The host cores this job may use: OMP_NUM_THREADS when the launcher sets
    it (the GPU box: 16 of a larger machine), else the CPU affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(pkg, cfg, cloud, threads, t1_s=8.0, tall_s=15.0):
    """Oracle (C++ restatement, recursive BVH2, AoS) on the host over bounded
    samples of the same frame, full spp and depth: every k-th row, k sized
    from a one-row pilot. Once on 1 thread (the reference's own execution
    model: one WASM instance) for ~t1_s, once on `threads` threads with a
    pixel-row partition (README.md:87's intent) for ~tall_s. Returns the
    baseline record and the all-threads sample (rows, acc) for the parity check."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import pyoracle

    sc = pyoracle.OracleScene(cfg["scene"], cloud)
    cam = pkg.scenes.scene_camera(cfg["scene"])
    W, H = cfg["W"], cfg["H"]
    acc = np.zeros((H, W, 3), np.float32)
    nee = cfg["nee"]

    def run(stride, nthreads, y0=0):
        acc[:] = 0
        t0 = time.time()
        _, st = sc.render(W, H, cam, nee, nee, cfg["depth"], 0xBABABEBE, 0, cfg["spp"], region=(0, y0, W, H),
                          row_step=stride, threads=nthreads, acc=acc)
        return time.time() - t0, st["rays"]

    # pilot: one row in the middle of the frame, one thread
    dt, _ = run(H, 1, y0=H // 2)
    per_row = max(dt, 1e-3)
    s1 = max(1, int(H / max(1.0, t1_s / per_row)))
    dt1, rays1 = run(s1, 1)
    sa = max(1, int(H / max(1.0, tall_s * threads / per_row)))
    dta, raysa = run(sa, threads)
    rows = np.arange(0, H, sa)
    rec = {"value": raysa / dta / 1e6, "unit": "Mray/s", "cores": threads, "kind": "port",
           "threads_1": rays1 / dt1 / 1e6, "threads_all": raysa / dta / 1e6, "nproc": os.cpu_count(),
           "job_cpus": threads,
           "cpu_model": _cpu_model(),
           "sample": f"{len(rows)} rows (every {sa}th) x {W} px x {cfg['spp']} spp of the {W}x{H} frame, depth "
                     f"{cfg['depth']}: {raysa} rays in {dta:.1f} s on {threads} threads; 1 thread: "
                     f"{len(range(0, H, s1))} rows (every {s1}th), {rays1} rays in {dt1:.1f} s (oracle/ C++ "
                     f"restatement; the Rust reference cannot be built here)"}
    return rec, rows, acc[rows].copy()


def parity(gpu_acc, rows, ref_rows):
    """Relative L2 and bit-exact pixel share of the GPU frame's rows against
    the oracle's (north_star: <= 1e-4 relative L2)."""
    import numpy as np

    g = gpu_acc[rows]
    d = np.linalg.norm((g - ref_rows).astype(np.float64).ravel())
    n = max(np.linalg.norm(ref_rows.astype(np.float64).ravel()), 1e-30)
    exact = float(np.mean(np.all(g.view(np.uint32) == ref_rows.view(np.uint32), axis=2)))
    return {"rel_l2": float(d / n), "bit_exact_frac": exact, "pixels": int(g.shape[0] * g.shape[1]),
            "tolerance": 1e-4, "reference": "oracle/ C++ restatement, same per-path seeds (cpu_baseline sample rows)"}


def _rows_parity(gpu_acc, ref_acc, rows):
    """Bit-exact share and relative L2 of the GPU frame's rows against the oracle's."""
    import numpy as np

    g, r = gpu_acc[rows], ref_acc[rows]
    d = np.linalg.norm((g - r).astype(np.float64).ravel())
    n = max(np.linalg.norm(r.astype(np.float64).ravel()), 1e-30)
    return {"rel_l2": float(d / n), "bit_exact_frac": float(np.mean(np.all(g.view(np.uint32) == r.view(np.uint32), axis=2))),
            "pixels": int(g.shape[0] * g.shape[1])}


def secondary(pkg, threads):
    """The other configs of BASELINE.json and the reference's init-default
    session, one bounded measurement each (single GPU, same process), with an
    oracle parity check: full-size row bands where the frame is a fixed spp
    (C2, museum), or a reduced viewport of the same session where the sample
    plan is adaptive (C5, init defaults: the CPU cannot replay 1080p x 1024
    spp adaptive rounds in seconds)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    itf = pkg.interface
    cloud = pkg.scenes.triangle_cloud(100000)
    out = {}

    def start(scene, W, H, types, adaptive, depth, mesh):
        itf.init(W, H, scene, *pkg.scenes.scene_camera(scene))
        if mesh is not None:
            itf.store_mesh(1, mesh)
        if types is not None:
            itf.update_settings(types[0], types[1], adaptive[0], adaptive[1], 0)
        itf.set_render_options(depth, 0xBABABEBE, 0)

    def timed(n, calls=1):
        itf.sync()
        itf.clear_stats()
        t0 = time.perf_counter()
        for _ in range(calls):
            itf.compute(n)
        itf.sync()
        dt = time.perf_counter() - t0
        st = itf.stats()
        return dt, st["rays"] + st["shadow_rays"]

    # fixed-spp configs: `steps` timed full steps (each after a reset, so
    # every step traces samples 0..spp-1), then oracle row bands of the last
    # step's frame; the value is the median step's rate, with min and max
    steps = 5
    for name in ("c2", "museum"):
        cfg = CONFIGS[name]
        W, H = cfg["W"], cfg["H"]
        start(cfg["scene"], W, H, (cfg["nee"], cfg["nee"]), (0, 0), cfg["depth"], None)
        itf.compute(W * H * cfg["spp"])  # warm-up: one full step (sizes the path buffers)
        rates, times = [], []
        for _ in range(steps):
            itf.set_render_options(cfg["depth"], 0xBABABEBE, 0)  # reset: samples 0..spp-1 below
            dt, rays = timed(W * H * cfg["spp"])
            rates.append(rays / dt / 1e6)
            times.append(dt * 1e3)
        acc = itf.read_radiance(W, H)[0]
        trav = itf.get_option("scene_traversal")
        itf.shutdown()
        rows = np.array([0, 1, H // 2, H // 2 + 1, H - 1])
        ref = np.zeros_like(acc)
        sc = pyoracle.OracleScene(cfg["scene"])
        for y in rows:
            sc.render(W, H, pkg.scenes.scene_camera(cfg["scene"]), cfg["nee"], cfg["nee"], cfg["depth"], 0xBABABEBE, 0,
                      cfg["spp"], region=(0, int(y), W, int(y) + 1), threads=threads, acc=ref)
        order = sorted(range(steps), key=lambda i: rates[i])
        med = order[steps // 2]
        out[name] = {"workload": f"{name.upper()} {cfg['name']} (scene {cfg['scene']}), {W}x{H}, {cfg['spp']} spp, "
                                 f"depth {cfg['depth']}", "value": rates[med], "unit": "Mray/s",
                     "ms_per_step": times[med], "steps": steps, "statistic": "median step",
                     "min": min(rates), "max": max(rates), "all": [round(r, 1) for r in rates],
                     "traversal": TRAVERSAL_NAMES.get(trav, str(trav)),
                     "parity": dict(_rows_parity(acc, ref, rows), check=f"rows {rows.tolist()} of the last timed frame")}

    # adaptive sessions: timed at full size, parity on a reduced viewport
    sessions = {
        "c5": dict(types=(2, 2), adaptive=(1, 1), depth=8, W=1920, H=1080, n=1920 * 1080 * 1024, calls=1,
                   warm=1920 * 1080 * 1024, what="C5 bunny scene PNEE + adaptive (both halves), 1920x1080, "
                                             "1024 spp budget, depth 8"),
        "init_defaults": dict(types=None, adaptive=None, depth=0, W=1920, H=1080, n=1920 * 1080 * 16, calls=3,
                              warm=1920 * 1080 * 16,
                              what="the reference's init defaults (left NormalNEE random, right PNEE adaptive, "
                                   "unbounded RR), bunny scene 1920x1080, compute(W*H*16) x 3"),
    }
    for name, c in sessions.items():
        start(2, c["W"], c["H"], c["types"], c["adaptive"], c["depth"], cloud)
        itf.compute(c["warm"])  # photons, the first rounds, path buffers sized for the timed call
        # the timed calls start from an empty sample stock (re-setting the
        # option drops it): every sample they add was traced inside the window
        itf.set_option("stock", itf.get_option("stock"))
        dt, rays = timed(c["n"], c["calls"])
        st = itf.stats()
        itf.shutdown()
        w, h, chunks = 64, 48, (64 * 48 * 6, 64 * 48 * 5 + 17, 64 * 48 * 9)
        types = c["types"] or (1, 2)
        adaptive = c["adaptive"] or (0, 1)
        start(2, w, h, c["types"], c["adaptive"], c["depth"], cloud)
        for n in chunks:
            itf.compute(n)
        acc, cnt = itf.read_radiance(w, h)
        itf.shutdown()
        ref = pyoracle.OracleScene(2, cloud).adaptive(w, h, pkg.scenes.scene_camera(2), types, adaptive, c["depth"])
        for n in chunks:
            ref.compute(n, threads=threads)
        acc_r, cnt_r, _ = ref.read()
        par = _rows_parity(acc, acc_r, np.arange(h))
        par["counts_equal"] = bool(np.array_equal(cnt, cnt_r))
        par["check"] = f"the same session at {w}x{h}, compute{chunks}, against the oracle's session"
        out[name] = {"workload": c["what"], "value": rays / dt / 1e6, "unit": "Mray/s",
                     "ms_per_step": dt * 1e3 / c["calls"], "steps": c["calls"], "parity": par,
                     # the adaptive halves' sample stock over the window: samples traced into it
                     # (refills + round deficits) and taken by the rounds, rays traced into it
                     "stock": {k: st[k] for k in ("stock_traced", "stock_consumed", "stock_deficit", "stock_waits",
                                                  "stock_rays")},
                     "rays_counted": "per sample when a round adds it (the stock starts empty at the window)"}
    return out


def strong_c4(pkg, rank, world, backend, own_comm, threads, frames=2):
    """N > 1: BASELINE configs[3] as strong scaling -- the one fixed C4 frame
    (3840x2160, 256 spp, depth 8, NormalNEE, the 100k stand-in) split over the
    N ranks by 16x16 tiles. Per frame: render (max over ranks) and gather to
    rank 0; rank 0 checks oracle rows 0, 15, 16, H/2 and H-1 of the gathered
    frame bit for bit (README.md:87, wasm_interface.rs:78,90-94)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    itf = pkg.interface
    cfg = CONFIGS["c4"]
    W, H, spp = cfg["W"], cfg["H"], cfg["spp"]
    cloud = pkg.scenes.triangle_cloud(cfg["mesh"])
    cam = pkg.scenes.scene_camera(cfg["scene"])
    itf.init(W, H, cfg["scene"], *cam)
    itf.store_mesh(1, cloud)
    itf.update_settings(cfg["nee"], cfg["nee"], 0, 0, 0)
    itf.set_render_options(cfg["depth"], 0xBABABEBE, 0)
    gather = None
    if own_comm:
        box = [itf.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        itf.set_comm(rank, world, 16, box[0])
    else:
        itf.set_partition(rank, world, 16)
        from wasm_pathtracer_amd import multigpu
        gather = multigpu.FrameGather(W, H, rank, world, 16, device="cuda")
    npart = len(itf.partition_pixels())
    rdev = "cuda" if backend == "nccl" else "cpu"

    def frame():
        itf.set_render_options(cfg["depth"], 0xBABABEBE, 0)  # reset: samples 0..spp-1
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        itf.compute(npart * spp)
        itf.sync()
        t1 = time.perf_counter()
        dist.barrier()
        t2 = time.perf_counter()
        if own_comm:
            itf.gather_frame(0)
            out = None
        else:
            itf.copy_partition(gather.local_view().data_ptr())
            out = gather.gather()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        t = torch.tensor([t1 - t0, t3 - t2], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0]), float(t[1]), out

    frame()  # warm-up: sizes the path buffers
    itf.clear_stats()
    render, gath = [], []
    for _ in range(frames):
        r, g, out = frame()
        render.append(r)
        gath.append(g)
    st = itf.stats()
    r = torch.tensor([float(st["rays"] + st["shadow_rays"])], dtype=torch.float64, device=rdev)
    dist.all_reduce(r, op=dist.ReduceOp.SUM)
    rays = float(r.item()) / frames
    rec = None
    if rank == 0:
        gpu = itf.read_radiance(W, H)[0] if own_comm else np.ascontiguousarray(out[..., :3].cpu().numpy())
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        prow = np.array([0, 15, 16, H // 2, H - 1])
        ref = np.zeros((H, W, 3), np.float32)
        sc = pyoracle.OracleScene(cfg["scene"], cloud)
        for y in prow:
            sc.render(W, H, cam, cfg["nee"], cfg["nee"], cfg["depth"], 0xBABABEBE, 0, spp,
                      region=(0, int(y), W, int(y) + 1), threads=threads, acc=ref)
        rm, gm = min(render), min(gath)
        rec = {"workload": f"C4 {cfg['name']} (scene {cfg['scene']}), {W}x{H}, {spp} spp frame split over "
                           f"{world} ranks by 16x16 tiles (strong), depth {cfg['depth']}, NormalNEE",
               "frames": frames, "render_ms": [round(x * 1e3, 2) for x in render],
               "gather_ms": [round(x * 1e3, 2) for x in gath],
               "value": rays / (rm + gm) / 1e6, "unit": "Mray/s", "render_only_Mray_s": rays / rm / 1e6,
               "statistic": "best frame, render + gather (max over ranks)",
               "gather": "RCCL ncclSend/ncclRecv in libwpt.so" if own_comm else f"torch.distributed gather ({backend})",
               "parity": dict(_rows_parity(gpu, ref, prow), tolerance=1e-4,
                              check=f"rows {prow.tolist()} of the frame gathered from {world} ranks against the oracle's")}
    itf.shutdown()
    return rec


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, cmd=None, poll_s=0.2):
    """`bench.py --gpus N` without an outside launcher: start N fresh child
    processes of this script, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N,
    MASTER_ADDR 127.0.0.1 and a free MASTER_PORT), wait for them and return the
    job's exit code. The parent never imports torch or touches the GPU (the
    children start by exec of a fresh interpreter, which is allowed only
    before any HIP call). Rank 0 prints the JSON line on the inherited stdout.
    If a rank fails, the others are stopped (their exact PIDs) and its code is
    returned. `cmd` replaces [python, bench.py] (tests)."""
    import subprocess

    cmd = list(cmd) if cmd else [sys.executable, os.path.abspath(__file__)]
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen(cmd + list(argv), env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code  # -N (signal N) -> 128 + N
                    print(f"[bench] rank {procs.index(p)} exited with {code}; stopping the other ranks",
                          file=sys.stderr)
                    for q in live:
                        q.terminate()
            if live:
                time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main():
    if "WORLD_SIZE" not in os.environ:
        # one process per GPU: `--gpus N` (N > 1) started without torchrun
        # spawns its own N ranks before anything touches the GPU
        pre = argparse.ArgumentParser(add_help=False)
        pre.add_argument("--gpus", type=int, default=1)
        n = pre.parse_known_args()[0].gpus
        if n > 1:
            sys.exit(launch_ranks(n, sys.argv[1:]))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override spp per GPU share (testing only)")
    ap.add_argument("--batch", type=int, default=1 << 27, help="paths resident per wavefront batch (2^27: one C3 step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-serial-step", action="store_true", help="skip the one-lane step (standalone kernel times)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary configs (C2, museum, C5, init defaults; default C3 single-GPU runs only)")
    ap.add_argument("--no-strong-c4", action="store_true", help="N>1: skip the strong-scaling C4 frame block")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads of the CPU baseline (0: the job's CPU share, OMP_NUM_THREADS or affinity)")
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                    help="weak: every GPU traces the config's spp over its partition share (N x spp frame); "
                         "strong: the N GPUs split one fixed frame of the config's spp")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="process group for N>1 (gloo: rehearsal of several ranks on one GPU)")
    ap.add_argument("--traffic-csv", default="", help="rocprofv3 --pmc counter CSV to fill roofline.traffic")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="launch option of the session (interface.OPTIONS, e.g. traversal=bvh4, lanes=3); "
                         "repeatable; the defaults are the production settings")
    ap.add_argument("--gather", default="wpt", choices=("wpt", "torch"),
                    help="N>1 with RCCL: the product's communicator (wpt_set_comm / wpt_gather_frame) or "
                         "torch.distributed (multigpu.FrameGather)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist
    import wpt_loader

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dev = local_rank % max(torch.cuda.device_count(), 1) if args.backend == "gloo" else local_rank
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")

    pkg = wpt_loader.load()
    itf = pkg.interface
    cfg = dict(CONFIGS[args.config])
    if args.spp:
        cfg["spp"] = args.spp
    W, H = cfg["W"], cfg["H"]
    cloud = pkg.scenes.triangle_cloud(cfg["mesh"]) if cfg["mesh"] else None
    cam = pkg.scenes.scene_camera(cfg["scene"])

    itf.set_device(dev)
    for o in args.opt:
        k, v = o.split("=", 1)
        itf.set_option(k, v)  # the default of the session init starts
    itf.init(W, H, cfg["scene"], *cam)
    if cloud is not None:
        itf.store_mesh(1, cloud)
    ad = cfg.get("adaptive", 0)
    bvh_ms, bvh_on_gpu = itf.scene_build_info()  # scene load, outside the timed region
    # what the uploaded scene's traversal kernels run (not guessed
    # from the scene id): the kernel instantiations named in the roofline
    scene_trav = itf.get_option("scene_traversal")
    tri_scene = itf.get_option("scene_tri_only") == 1
    itf.update_settings(cfg["nee"], cfg["nee"], ad, ad, 0)
    itf.set_render_options(cfg["depth"], 0xBABABEBE, args.batch)
    own_comm = world > 1 and args.backend == "nccl" and args.gather == "wpt"
    comm_fallback = None
    if own_comm:
        # the product's RCCL communicator: rank 0's 128-byte id to every rank
        # (over the torch process group), then wpt_set_comm on every rank
        box = [itf.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        err = ""
        try:
            itf.set_comm(rank, world, 16, box[0])
        except Exception as e:  # noqa: BLE001 - reported below, every rank agrees on the fallback
            err = f"{type(e).__name__}: {e}"
        ok = torch.tensor([0 if err else 1], dtype=torch.int32, device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            # a rank could not create the product's communicator: all ranks
            # fall back to the torch.distributed gather (reported in the line)
            print(f"[rank {rank}] wpt_set_comm failed ({err or 'on another rank'}); "
                  f"falling back to --gather torch", file=sys.stderr)
            if not err:
                itf.comm_destroy()
            own_comm = False
            comm_fallback = err or "failed on another rank"
            itf.set_partition(rank, world, 16)
    elif world > 1:
        itf.set_partition(rank, world, 16)
    npart = len(itf.partition_pixels())
    exchange = None
    if ad and world > 1 and own_comm:
        exchange = "wpt"  # adaptive rounds exchange the frame over the communicator (ncclAllGather)
        paths_per_step = W * H * cfg["spp"]
    elif ad and world > 1:
        # adaptive rounds over several ranks: the frame is exchanged at each
        # round boundary (RCCL all-gather) and every rank plans the same global
        # round; compute(n) advances the GLOBAL round sequence, so the job
        # renders the one W x H x spp frame (strong scaling)
        from wasm_pathtracer_amd import multigpu
        exchange = multigpu.RoundExchange(world, device="cuda")
        paths_per_step = W * H * cfg["spp"]
    elif args.scaling == "strong":
        paths_per_step = npart * cfg["spp"]  # the fixed W x H x spp frame, split by tiles
    else:
        paths_per_step = npart * cfg["spp"] * world  # per-GPU work fixed: ~W*H*spp
    # timed steps run the production kernels (no work counters); the
    # algorithmic bytes of the roofline come from one extra counted step below
    itf.set_counting(False)
    itf.set_profiling(True)

    gather = None
    if world > 1 and not own_comm:
        from wasm_pathtracer_amd import multigpu
        gather = multigpu.FrameGather(W, H, rank, world, 16, device="cuda")
        assert gather.npart == npart

    gather_s = [0.0]  # wall time of the frame gathers (N > 1), timed steps only

    def do_gather():
        """Every rank's partition into rank 0's frame; returns rank 0's frame
        (H, W, 3) when `want` is set by the caller (parity), else None."""
        t0 = time.perf_counter()
        frame = None
        if own_comm:
            # every rank's packed partition into rank 0's frame: grouped
            # ncclSend / ncclRecv over xGMI inside libwpt.so. A failure ends
            # the job (non-zero exit; launch_ranks stops the other ranks)
            # instead of switching transport mid-run
            try:
                itf.gather_frame(0)
            except Exception as e:  # noqa: BLE001
                print(f"[rank {rank}] wpt_gather_frame failed: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
                os._exit(3)
        else:
            # pack this rank's partition (float4 acc+count) on the device, then
            # one gather to rank 0 over torch.distributed, which scatters it into the full frame
            itf.copy_partition(gather.local_view().data_ptr())
            frame = gather.gather()
        torch.cuda.synchronize()
        gather_s[0] += time.perf_counter() - t0
        return frame

    def step():
        itf.compute(paths_per_step)
        if world > 1:
            do_gather()

    for _ in range(args.warmup):
        step()
    itf.sync()
    gather_s[0] = 0.0
    itf.clear_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    itf.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0

    st = itf.stats()
    kt = itf.kernel_times()
    rays_local = st["rays"] + st["shadow_rays"]
    # the parity frame: one more PRODUCTION step (the timed kernels, work
    # counters off) after a reset, i.e. samples 0..spp-1 of every pixel of
    # this rank's partition, compared with the oracle's rows below
    gather_ms_per_step = gather_s[0] / args.steps * 1e3
    gpu_acc = None
    if world == 1 and not cfg.get("adaptive"):
        itf.set_render_options(cfg["depth"], 0xBABABEBE, args.batch)  # resets the accumulation
        itf.compute(paths_per_step)
        itf.sync()
        gpu_acc = itf.read_radiance(W, H)[0]
    elif world > 1 and not cfg.get("adaptive"):
        # the same for N ranks: one production step over every partition,
        # gathered to rank 0, whose frame is checked against oracle row bands
        itf.set_render_options(cfg["depth"], 0xBABABEBE, args.batch)
        itf.compute(paths_per_step)
        itf.sync()
        frame = do_gather()
        if rank == 0:
            gpu_acc = (itf.read_radiance(W, H)[0] if own_comm else
                       np.ascontiguousarray(frame[..., :3].cpu().numpy()))
    # one more step of the same workload (samples 0..spp-1 again) with the
    # device work counters on (the COUNT instantiations): node visits / prim
    # tests / node bytes per launch
    itf.clear_stats()
    itf.set_counting(True)
    itf.set_render_options(cfg["depth"], 0xBABABEBE, args.batch)
    itf.compute(paths_per_step)
    itf.sync()
    stc = itf.stats()
    photon_rays = st.get("photon_rays", 0)
    ktc = itf.kernel_times()
    itf.set_counting(False)
    # one more step with ONE lane: the kernels run serialised on the whole GPU
    # (one-lane batches get full-capacity traversal grids), so their busy
    # times are standalone times (with 4 lanes a kernel's busy time includes
    # the co-running lanes' kernels)
    kts = None
    if world == 1 and not args.no_serial_step:
        lanes_default = itf.get_option("lanes")
        itf.set_lanes(1)
        itf.clear_stats()
        itf.compute(paths_per_step)
        itf.sync()
        kts = itf.kernel_times()
        itf.set_lanes(lanes_default)
    if world > 1:
        rdev = "cuda" if args.backend == "nccl" else "cpu"
        t = torch.tensor([dt], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        r = torch.tensor([rays_local], dtype=torch.float64, device=rdev)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays_total = float(r.item())
    else:
        rays_total = float(rays_local)

    # Roofline of the dominant kernel: algorithmic bytes per launch / avg launch time.
    # extend: per ray 32 B (origin, dir) read + 8 B (t, id) written, node bytes
    # (root 32 B, 64 B per internal expansion = both children, 16 B per resumed
    # large-leaf stack entry) + 64 B per primitive test. shadow: 48 B ray record
    # read (+16 B colour RMW when lit, counted as 16 B), same node/prim bytes.
    ext_bytes = 40 * stc["rays"] + stc["ext_node_bytes"] + 64 * stc["ext_tests"]
    sh_bytes = 64 * stc["shadow_rays"] + stc["sh_node_bytes"] + 64 * stc["sh_tests"]
    # The lanes' launches of a kernel run concurrently (a batch is cut into
    # slices traced on separate streams), so a launch is counted LOGICALLY: once
    # per bounce, its duration = the union of the lanes' launch intervals.
    cand = {  # (timed busy ms, timed logical launches, counted-step bytes, counted-step logical launches)
        "extend": (kt["extend"]["busy_ms"], kt["extend"]["logical_launches"], ext_bytes,
                   ktc["extend"]["logical_launches"]),
        "shadow": (kt["shadow"]["busy_ms"], kt["shadow"]["logical_launches"], sh_bytes,
                   ktc["shadow"]["logical_launches"]),
    }
    if kt["trace"]["logical_launches"]:
        # fused extend + shadow launches (WPT_OPT_FUSED): their own device-counted bytes
        cand["trace"] = (kt["trace"]["busy_ms"], kt["trace"]["logical_launches"], stc["trace_bytes"],
                         ktc["trace"]["logical_launches"])
    dom = max(cand, key=lambda k: cand[k][0])
    ms, nl, byts, nlc = cand[dom]
    avg_ms = ms / max(nl, 1)
    bytes_per_launch = byts / max(nlc, 1)
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    lanes = kt[dom]["launches"] / max(kt[dom]["logical_launches"], 1)  # dispatches per logical launch
    traffic = None
    traffic_src = None
    # the timed kernel's own instantiation (work counters off): PMC figures
    # are never averaged with the COUNT build of the counted step
    # the traversal the scene runs (a scene without a BVH scans linearly in
    # the BVH2 kernels' instantiation)
    trav_id = 1 if scene_trav == 1 else 0
    trav_name = TRAVERSAL_NAMES.get(scene_trav, str(scene_trav))
    kname = (f"k_{dom}<{'true' if tri_scene else 'false'}, false>" if dom == "trace" else
             f"k_{dom}<{'true' if tri_scene else 'false'}, false, {trav_id}>")
    if not args.traffic_csv:
        # committed PMC summary of this same workload (tools/profile.sh ->
        # tools/collect_profile.py); used only when it was taken on this config
        prof = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
        if os.path.exists(prof):
            meta = json.load(open(prof))
            want = {"config": args.config, "batch": args.batch, "spp": cfg["spp"], "gpus": world,
                    "traversal": trav_name, "lanes": round(lanes)}
            if all(meta.get(k) == v for k, v in want.items()) and kname in meta["kernels"]:
                # rocprof counts per dispatch; a logical launch is `lanes` dispatches
                traffic = meta["kernels"][kname]["hbm_bytes_per_launch"] * lanes
                traffic_src = f"profiles/traffic_{args.config}.json ({meta['source']}), {kname} dispatches only"
    # VALU evidence for the same kernel (north_star: "VALU-busy against gfx950
    # peak"): lane-ops per logical launch from the committed PMC passes
    # (SQ_INSTS_VALU x active lanes, x dispatches per logical launch) over the
    # live busy time, against 256 CU x 4 SIMD32 x 2.4 GHz = 78.6 T lane-ops/s
    valu = None
    if not args.traffic_csv and traffic is not None:
        kmeta = meta["kernels"][kname]
        if kmeta.get("valu_insts_per_launch"):
            lane_ops = kmeta["valu_insts_per_launch"] * kmeta["active_lanes_per_valu"] * lanes
            v_ach = lane_ops / (avg_ms * 1e-3) / 1e12
            valu = {"achieved": v_ach, "peak": PEAK_VALU_TOPS, "unit": "T lane-ops/s", "frac": v_ach / PEAK_VALU_TOPS,
                    "issue_frac": kmeta["valu_insts_per_launch"] * lanes * 2 / (avg_ms * 1e-3 * 2.4e9 * 1024),
                    "active_lanes_per_valu": kmeta["active_lanes_per_valu"],
                    "source": f"{kname} dispatches only: SQ_INSTS_VALU per dispatch, lanes = SQ_THREAD_CYCLES_VALU / "
                              "SQ_ACTIVE_INST_VALU (reads 64.00 on full-lane kernels; profiles/traffic_c3.json); "
                              "issue_frac = wave-instructions x 2 cycles / (SIMD-cycles of the busy time)"}
    if args.traffic_csv and os.path.exists(args.traffic_csv):
        try:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import pmc
            traffic = pmc.bytes_per_launch(args.traffic_csv, kname) * lanes
            traffic_src = args.traffic_csv
        except Exception as e:  # noqa: BLE001
            traffic_src = f"unreadable: {e}"
    total_kernel_ms = sum(v["busy_ms"] for v in kt.values())
    strong = exchange is not None or args.scaling == "strong"

    result = {
        "metric": "Mray/s (primary+shadow+bounce) at 1920x1080, 1/2/4/8 GPU; L2 vs CPU ref",
        "value": rays_total / dt / 1e6,
        "unit": "Mray/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic: seeded 100k-triangle cloud in mesh slot 1 (bunny2.obj absent), per-path xorshift32 streams"
                 if cfg["mesh"] else "built-in scene geometry, per-path xorshift32 streams"),
        "config": {
            "workload": f"{args.config.upper()} {cfg['name']} (scene id {cfg['scene']}), {W}x{H}, "
                        + (f"{cfg['spp']} spp budget over {world} GPUs (strong), depth" if exchange is not None else
                           f"{cfg['spp']} spp frame split over {world} GPUs (strong), depth" if strong else
                           f"{cfg['spp']} spp per GPU share ({cfg['spp'] * world} spp frame), depth")
                        + f" {cfg['depth']}, {('NoNEE', 'NormalNEE', 'PNEE')[cfg['nee']]}"
                        f"{', adaptive' if cfg.get('adaptive') else ''}",
            "paths_per_step_per_gpu": paths_per_step if exchange is None else paths_per_step / world,
            "rays": int(rays_total),
            "parallelism": (f"tile-partition x{world}" + (" (gloo rehearsal)" if args.backend != "nccl" else
                                                          ", RCCL gather in libwpt.so" if own_comm else
                                                          ", torch.distributed gather"
                                                          + (f" (wpt_set_comm fell back: {comm_fallback})"
                                                             if comm_fallback else "")))
                           if world > 1 else "single GPU",
        },
        "scene_load": {"bvh2_build_ms": round(bvh_ms, 2), "bvh2_built_on": "gpu" if bvh_on_gpu else "host"},
        "traversal": trav_name,
        "roofline": {
            "bound": "hbm",
            "kernel": kname,
            "achieved": achieved,
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "bytes_per_launch": bytes_per_launch,
            "avg_launch_ms": avg_ms,
            "launches": nl,
            "launch": f"logical: one per bounce = {lanes:g} concurrent lane dispatches; duration = union of their intervals",
            # what actually bounds it (the contract's bound field only admits hbm / mfma): counter
            # traffic per launch over the same time against HBM peak, and the VALU figures below
            "fabric_frac": (traffic / (avg_ms * 1e-3) / 1e9 / PEAK_HBM_GBS) if (traffic and avg_ms > 0) else None,
            "valu_frac": valu["frac"] if valu else None,
            "issue_frac": valu["issue_frac"] if valu else None,
            "limiter": "latency of the dependent node -> primitive -> stack-pop loads at 8 waves/SIMD "
                       "(neither HBM nor VALU near peak; the BVH and primitives are L2/MALL-resident)",
        },
        # busy = union of a kernel's launch intervals (lanes overlap, and
        # different kernels of different lanes overlap each other too)
        "valu": valu,
        "kernel_share": {k: round(v["busy_ms"] / total_kernel_ms, 4) for k, v in kt.items()} if total_kernel_ms else {},
        "kernel_busy_ms_per_step": {k: round(v["busy_ms"] / args.steps, 2) for k, v in kt.items()},
        "kernel_launch_ms_per_step": {k: round(v["ms"] / args.steps, 2) for k, v in kt.items()},
        # the same step with one lane (serialised kernels): standalone time per kernel, and the step
        "kernel_serial_ms_per_step": ({k: round(v["busy_ms"], 2) for k, v in kts.items() if v["busy_ms"] > 0}
                                      if kts else None),
        "work": {"node_visits_per_ray": stc["node_visits"] / max(stc["rays"] + stc["shadow_rays"], 1),
                 "prim_tests_per_ray": stc["prim_tests"] / max(stc["rays"] + stc["shadow_rays"], 1),
                 "shadow_fraction": st["shadow_rays"] / max(rays_local, 1),
                 "ext_steps_per_ray": stc["ext_live_iters"] / max(stc["rays"], 1),
                 "ext_loop_live_frac": stc["ext_live_iters"] / max(stc["ext_lane_iters"], 1),
                 "sh_steps_per_ray": stc["sh_live_iters"] / max(stc["shadow_rays"], 1),
                 "sh_loop_live_frac": stc["sh_live_iters"] / max(stc["sh_lane_iters"], 1),
                 "exact_retrace_per_ray": (stc["fallback_ext"] + stc["fallback_sh"]) / max(stc["rays"] + stc["shadow_rays"], 1),
                 # SIMD use of the traversal loop's two bodies (device ballots, <= 64 by construction)
                 "lanes_per_expand_body": stc["ex_body_lanes"] / max(stc["ex_bodies"], 1),
                 "lanes_per_leaf_body": stc["lf_body_lanes"] / max(stc["lf_bodies"], 1),
                 "lanes_per_body": (stc["ex_body_lanes"] + stc["lf_body_lanes"]) / max(stc["ex_bodies"] + stc["lf_bodies"], 1),
                 # wave-level executions per traced ray (extension + shadow): loop
                 # iterations and the two bodies (tools/body_table.py's executed columns)
                 "wave_iters_per_ray": (stc["ext_lane_iters"] + stc["sh_lane_iters"]) / 64.0
                                       / max(stc["rays"] + stc["shadow_rays"], 1),
                 "expand_bodies_per_ray": stc["ex_bodies"] / max(stc["rays"] + stc["shadow_rays"], 1),
                 "leaf_bodies_per_ray": stc["lf_bodies"] / max(stc["rays"] + stc["shadow_rays"], 1)},
    }
    if world > 1:
        result["gather_ms_per_step"] = gather_ms_per_step
        result["render_ms_per_step"] = dt / args.steps * 1e3 - gather_ms_per_step
    if rank == 0 and not args.no_cpu_baseline:
        threads = args.cpu_threads or _host_threads()
        rec, rows, ref_rows = cpu_baseline(pkg, cfg, cloud, threads)
        result["cpu_baseline"] = rec
        if gpu_acc is not None and world == 1:
            result["parity"] = parity(gpu_acc, rows, ref_rows)
        elif gpu_acc is not None:
            # the gathered N-rank frame (spp_frame samples per pixel) against
            # oracle rows: top, a band straddling the first 16 px tile row,
            # the middle, the bottom
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle
            spp_frame = cfg["spp"] if strong else cfg["spp"] * world
            prow = np.array([0, 15, 16, H // 2, H - 1])
            ref = np.zeros((H, W, 3), np.float32)
            sc = pyoracle.OracleScene(cfg["scene"], cloud)
            for y in prow:
                sc.render(W, H, cam, cfg["nee"], cfg["nee"], cfg["depth"], 0xBABABEBE, 0, spp_frame,
                          region=(0, int(y), W, int(y) + 1), threads=threads, acc=ref)
            result["parity"] = dict(_rows_parity(gpu_acc, ref, prow), tolerance=1e-4,
                                    check=f"rows {prow.tolist()} of the frame gathered from {world} ranks "
                                          f"({spp_frame} spp) against the oracle's")
    itf.shutdown()
    if world > 1 and args.config == "c3" and not args.no_strong_c4:
        # the real inter-GPU question: C4's one fixed frame split over the N
        # ranks (tile balance + gather); the weak C3 line above has none
        rec = strong_c4(pkg, rank, world, args.backend, own_comm, args.cpu_threads or _host_threads())
        if rank == 0:
            result["strong_c4"] = rec
    if rank == 0 and world == 1 and args.config == "c3" and not args.no_secondary and not args.opt:
        t0 = time.perf_counter()
        result["secondary"] = secondary(pkg, args.cpu_threads or _host_threads())
        result["secondary_s"] = round(time.perf_counter() - t0, 1)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
