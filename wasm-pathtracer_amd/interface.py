"""Python mirror of the reference's operator interface, src/wasm_interface.rs.

Same function names and argument meaning as the reference's wasm exports
(init, results, update_scene, update_settings, update_viewport,
update_camera, allocate_mesh, mesh_vertices, notify_mesh_loaded,
allocate_texture, notify_texture_loaded, compute). Where the reference
panics (a WASM trap) these raise ``WptError`` carrying the library's status
code and message. Everything runs through libwpt.so; nothing here computes.
"""
import ctypes

import numpy as np

from ._lib import lib

OK = 0
ERR_NOT_INIT, ERR_ALREADY_INIT, ERR_INVALID_SCENE, ERR_INVALID_ARG = -1, -2, -3, -4
ERR_UNSUPPORTED, ERR_DEVICE, ERR_NO_MESH = -5, -6, -7
NO_NEE, NORMAL_NEE, PNEE = 0, 1, 2


class WptError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _check(rc):
    if rc < 0:
        raise WptError(rc, lib().wpt_last_error().decode())
    return rc


# ---- reference exports (wasm_interface.rs) ---------------------------------
def init(width, height, scene_id, cam_x, cam_y, cam_z, cam_rot_x, cam_rot_y):
    """wasm_interface.rs:67"""
    _check(lib().wpt_init(width, height, scene_id, cam_x, cam_y, cam_z, cam_rot_x, cam_rot_y))


def results(is_show_sampling=0, width=None, height=None):
    """wasm_interface.rs:120 — returns a (H, W, 4) uint8 copy of the buffer."""
    p = lib().wpt_results(is_show_sampling)
    if not p:
        raise WptError(ERR_NOT_INIT, lib().wpt_last_error().decode())
    n = width * height * 4
    return np.ctypeslib.as_array(p, shape=(n,)).copy().reshape(height, width, 4)


def update_scene(scene_id):
    """wasm_interface.rs:154"""
    _check(lib().wpt_update_scene(scene_id))


def update_settings(left_type, right_type, is_left_adaptive, is_right_adaptive, is_light_debug):
    """wasm_interface.rs:173"""
    _check(lib().wpt_update_settings(left_type, right_type, is_left_adaptive, is_right_adaptive, is_light_debug))


def update_viewport(width, height):
    """wasm_interface.rs:219"""
    _check(lib().wpt_update_viewport(width, height))


def update_camera(cam_x, cam_y, cam_z, cam_rot_x, cam_rot_y):
    """wasm_interface.rs:239"""
    _check(lib().wpt_update_camera(cam_x, cam_y, cam_z, cam_rot_x, cam_rot_y))


def allocate_mesh(mesh_id, num_vertices):
    """wasm_interface.rs:259"""
    _check(lib().wpt_allocate_mesh(mesh_id, num_vertices))


def mesh_vertices(mesh_id, num_vertices):
    """wasm_interface.rs:275 — a writable (num_vertices, 3) float32 view."""
    p = lib().wpt_mesh_vertices(mesh_id)
    if not p:
        raise WptError(ERR_NO_MESH, lib().wpt_last_error().decode())
    return np.ctypeslib.as_array(p, shape=(num_vertices * 3,)).reshape(num_vertices, 3)


def notify_mesh_loaded(mesh_id):
    """wasm_interface.rs:293 — True if the active scene was rebuilt."""
    return bool(_check(lib().wpt_notify_mesh_loaded(mesh_id)))


def _obj_args(text, scale):
    b = text.encode() if isinstance(text, str) else bytes(text)
    sc = None if scale is None else np.ascontiguousarray(scale, dtype=np.float32)
    return b, sc, (None if sc is None else sc.ctypes.data)


def parse_obj(text, scale=None):
    """obj_parser.ts:3-51 in libwpt.so (wpt_parse_obj, host only): float32
    (3 * vertices,) triangle soup, scaled per axis if `scale` is given."""
    b, sc, sp = _obj_args(text, scale)
    n = ctypes.c_uint64(0)
    _check(lib().wpt_parse_obj(b, len(b), sp, None, 0, ctypes.addressof(n)))
    out = np.empty(3 * n.value, dtype=np.float32)
    _check(lib().wpt_parse_obj(b, len(b), sp, out.ctypes.data if n.value else None, n.value, ctypes.addressof(n)))
    return out


def load_obj(mesh_id, text, scale=None):
    """OBJ text into mesh slot `mesh_id` (wpt_load_obj); then call
    notify_mesh_loaded(mesh_id). Returns the vertex count."""
    b, sc, sp = _obj_args(text, scale)
    n = ctypes.c_uint64(0)
    _check(lib().wpt_load_obj(mesh_id, b, len(b), sp, ctypes.addressof(n)))
    return n.value


def allocate_texture(tex_id, width, height):
    """wasm_interface.rs:335"""
    p = lib().wpt_allocate_texture(tex_id, width, height)
    if not p:
        raise WptError(ERR_NOT_INIT, lib().wpt_last_error().decode())
    return np.ctypeslib.as_array(p, shape=(width * height * 3,))


def notify_texture_loaded(tex_id):
    """wasm_interface.rs:358 (always False)"""
    return bool(_check(lib().wpt_notify_texture_loaded(tex_id)))


def compute(num_samples):
    """wasm_interface.rs:374"""
    _check(lib().wpt_compute(num_samples))


# ---- additions --------------------------------------------------------------
def store_mesh(mesh_id, vertices):
    """The worker's mesh upload protocol (worker.ts:171-179):
    allocate_mesh → fill mesh_vertices → notify_mesh_loaded."""
    v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
    allocate_mesh(mesh_id, v.shape[0])
    mesh_vertices(mesh_id, v.shape[0])[:] = v
    return notify_mesh_loaded(mesh_id)


def set_device(dev):
    _check(lib().wpt_set_device(dev))


def set_render_options(max_depth=0, frame_seed=0xBABABEBE, batch_paths=0):
    _check(lib().wpt_set_render_options(max_depth, frame_seed, batch_paths))


def set_partition(rank, nranks, tile=16):
    _check(lib().wpt_set_partition(rank, nranks, tile))


def partition_pixels():
    n = _check(lib().wpt_partition_pixels(None))
    out = np.empty(n, dtype=np.uint32)
    _check(lib().wpt_partition_pixels(out.ctypes.data))
    return out


def tile_partition(width, height, rank, nranks, tile=16):
    """Host-only: pixel indices set_partition(rank, nranks, tile) would give."""
    n = _check(lib().wpt_tile_partition(width, height, rank, nranks, tile, None))
    out = np.empty(n, dtype=np.uint32)
    _check(lib().wpt_tile_partition(width, height, rank, nranks, tile, out.ctypes.data))
    return out


def photon_tree(num_lights):
    """Frozen PNEE octree: (child[nodes], cum[nodes, num_lights], shot, stored)."""
    n = _check(lib().wpt_photon_tree(None, None, None))
    child = np.empty(n, dtype=np.uint32)
    cum = np.empty(n * max(num_lights, 1), dtype=np.float32)
    ss = np.empty(2, dtype=np.uint64)
    _check(lib().wpt_photon_tree(child.ctypes.data, cum.ctypes.data, ss.ctypes.data))
    return child, cum[: n * num_lights].reshape(n, num_lights), int(ss[0]), int(ss[1])


def read_radiance(width, height):
    acc = np.empty(width * height * 3, dtype=np.float32)
    cnt = np.empty(width * height, dtype=np.uint32)
    _check(lib().wpt_read_radiance(acc.ctypes.data, cnt.ctypes.data))
    return acc.reshape(height, width, 3), cnt.reshape(height, width)


def comm_unique_id():
    """ncclGetUniqueId (128 bytes): made on one rank, handed to every rank."""
    buf = ctypes.create_string_buffer(128)
    _check(lib().wpt_comm_unique_id(buf))
    return buf.raw


def set_comm(rank, nranks, tile, unique_id):
    """Collective: this rank's tile partition plus an RCCL communicator over
    all ranks; adaptive rounds then exchange the frame over it."""
    uid = ctypes.create_string_buffer(bytes(unique_id), 128)
    _check(lib().wpt_set_comm(rank, nranks, tile, uid))


def gather_frame(root=0):
    """Collective: every rank's partition into root's frame (RCCL over xGMI)."""
    _check(lib().wpt_gather_frame(root))


def gather_plan(rank, nranks, root, slot):
    """Host-only: the rooted gather's point-to-point transfers as `rank`
    posts them: (peer, float4 offset in root's buffer, float4 count, recv)."""
    n = _check(lib().wpt_gather_plan(rank, nranks, root, slot, None))
    out = np.zeros(4 * max(n, 1), dtype=np.uint64)
    _check(lib().wpt_gather_plan(rank, nranks, root, slot, out.ctypes.data))
    return [(int(a), int(b), int(c), bool(d)) for a, b, c, d in out[: 4 * n].reshape(-1, 4)]


def comm_destroy():
    _check(lib().wpt_comm_destroy())


def copy_partition(device_ptr):
    _check(lib().wpt_copy_partition(ctypes.c_void_p(device_ptr)))


def stats():
    keys = ("paths", "rays", "shadow_rays", "node_visits", "prim_tests", "bounces", "ext_visits", "ext_tests",
            "ext_node_bytes", "sh_visits", "sh_tests", "sh_node_bytes", "fallback_ext", "fallback_sh",
            "ext_lane_iters", "ext_live_iters", "sh_lane_iters", "sh_live_iters", "photon_rays", "photons",
            "sum_chunks", "sum_resummed", "sum_fetched", "stock_consumed", "fill_paths", "trace_bytes",
            "finish_paths", "finish_max_bounces", "max_ray_visits", "ex_body_lanes", "ex_bodies", "lf_body_lanes",
            "lf_bodies", "stock_traced", "stock_deficit", "stock_waits", "plan_us", "stock_us",
            "stock_rays", "stock_rays_used")
    out = (ctypes.c_uint64 * len(keys))()
    _check(lib().wpt_stats(ctypes.addressof(out), len(keys)))
    return dict(zip(keys, list(out)))


def kernel_times():
    """Per kernel: summed launch ms and launches, and (the lanes' launches
    overlap) busy_ms = union of the launch intervals, logical launches = one
    per bounce (generate / accumulate: one per batch)."""
    out = (ctypes.c_double * 28)()
    _check(lib().wpt_kernel_times(ctypes.addressof(out), 28))
    names = ("generate", "extend", "shade", "shadow", "accumulate", "trace")  # trace: fused extend + shadow
    kt = {n: {"ms": out[2 * i], "launches": int(out[2 * i + 1]), "busy_ms": out[12 + 2 * i],
              "logical_launches": int(out[13 + 2 * i])} for i, n in enumerate(names)}
    return kt


def set_counting(on):
    _check(lib().wpt_set_counting(1 if on else 0))


def set_profiling(on):
    _check(lib().wpt_set_profiling(1 if on else 0))


def scene_build_info():
    """The active scene's BVH2 build: (ms, built on the GPU)."""
    out = (ctypes.c_double * 2)()
    _check(lib().wpt_scene_build_info(ctypes.addressof(out)))
    return float(out[0]), bool(out[1])


def set_lanes(n):
    """Concurrent lanes of the next compute calls (1 serialises the kernels)."""
    _check(lib().wpt_set_lanes(int(n)))


# launch configuration (include/wpt.h WPT_OPT_*): no environment variable
# changes it; the frame is bit-identical for every setting
OPTIONS = {"defaults": 0, "traversal": 1, "traversal_sh": 2, "fused": 3, "fused_below": 4, "small_lanes": 5, "pixel_tile": 6,
           "grid_pct": 7, "refill": 8, "refill_sh": 9, "treelet": 10, "bvh_build": 11, "lanes": 12,
           "finish_below": 13, "trace_grid_pct": 14, "finish_every": 20, "probe": 22, "stock": 23, "stock_lanes": 24,
           "fill": 25, "async_prio": 26, "async_grid_pct": 27, "scene_traversal": 28, "scene_tri_only": 29,
           "stock_ahead": 30, "async_oneshot": 31, "stock_every": 32, "stock_extra": 33,
           "log": 34, "stock_prefill": 35, "async_fused_below": 36}
# symbolic values of the enumerated options
# traversal: exact BVH2, the BVH4 fast path, or auto (the default: BVH4 on
# scenes with other shapes than triangles, else BVH2)
TRAVERSALS = {"bvh2": 0, "bvh4": 1, "auto": 3}
OPTION_VALUES = {"traversal": TRAVERSALS, "traversal_sh": TRAVERSALS,
                 "bvh_build": {"auto": 0, "host": 1, "gpu": 2}}


def set_option(name, value):
    """wpt_set_option: with no session the default of every later init
    (set_option("defaults", 0) restores the built-in ones), with a session
    that session only (scene / partition rebuilt where the option shapes it)."""
    if isinstance(value, str) and not value.lstrip("-").isdigit():
        value = OPTION_VALUES[name][value]
    _check(lib().wpt_set_option(OPTIONS[name], int(value)))


def get_option(name):
    v = ctypes.c_int64(0)
    _check(lib().wpt_get_option(OPTIONS[name], ctypes.addressof(v)))
    return v.value


def probe_read():
    """Wave timelines recorded since set_option("probe", N) (wpt_probe_read):
    (meta, rec, ticks_per_us): meta (launches, 5) u32 = kernel (1 extend,
    3 shadow, 5 trace), lane, bounce, waves, first entry; rec (entries, 4) u32
    = start, feed dry, end (steady-clock ticks), rays taken."""
    L = lib()
    ent = ctypes.c_uint64(0)
    tpu = ctypes.c_double(0.0)
    n = L.wpt_probe_read(None, None, ctypes.addressof(ent), ctypes.addressof(tpu))
    if n < 0:
        raise WptError(int(n), L.wpt_last_error().decode())
    meta = np.zeros((n, 5), np.uint32)
    rec = np.zeros((ent.value, 4), np.uint32)
    if n:
        ent.value = rec.shape[0]  # rec's capacity (entries)
        _check(L.wpt_probe_read(meta.ctypes.data, rec.ctypes.data, ctypes.addressof(ent), ctypes.addressof(tpu)))
    return meta, rec, tpu.value


def clear_stats():
    _check(lib().wpt_clear_stats())


def sync():
    _check(lib().wpt_sync())


def bvh_depth():
    return _check(lib().wpt_bvh_depth())


def trace_rays(rays):
    r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
    n = r.shape[0]
    t = np.empty(n, dtype=np.float32)
    ids = np.empty(n, dtype=np.int32)
    _check(lib().wpt_trace_rays(n, r.ctypes.data, t.ctypes.data, ids.ctypes.data))
    return t, ids


def shadow_rays(pq, light_ids):
    p = np.ascontiguousarray(pq, dtype=np.float32).reshape(-1, 6)
    li = np.ascontiguousarray(light_ids, dtype=np.int32)
    occ = np.empty(p.shape[0], dtype=np.uint8)
    _check(lib().wpt_shadow_rays(p.shape[0], p.ctypes.data, li.ctypes.data, occ.ctypes.data))
    return occ.astype(bool)


def shutdown():
    _check(lib().wpt_shutdown())


class DebugScene:
    """View of a scene as wpt_init would build it: BVH2 built on the host (no
    GPU), or with gpu=True by the GPU build (wpt_debug_scene_new_gpu)."""

    def __init__(self, scene_id, mesh=None, gpu=False):
        L = lib()
        m = None if mesh is None else np.ascontiguousarray(mesh, dtype=np.float32)
        new = L.wpt_debug_scene_new_gpu if gpu else L.wpt_debug_scene_new
        self.h = new(scene_id, None if m is None else m.ctypes.data, 0 if m is None else m.size // 3)
        if not self.h:
            raise WptError(ERR_INVALID_SCENE, L.wpt_last_error().decode())
        bi = np.zeros(2, dtype=np.float64)
        _check(L.wpt_debug_scene_build_info(self.h, bi.ctypes.data))
        self.bvh_ms, self.bvh_on_gpu = float(bi[0]), bool(bi[1])
        info = np.zeros(8, dtype=np.uint64)
        L.wpt_debug_scene_info(self.h, info.ctypes.data)
        (self.num_shapes, self.num_inf, self.num_nodes, self.num_lights, self.depth, self.use_bvh,
         self.tri_only, self.num_nodes4) = (int(x) for x in info)

    def nodes(self):
        out = np.empty((self.num_nodes, 8), dtype=np.uint32)
        lib().wpt_debug_scene_nodes(self.h, out.ctypes.data)
        return out

    def nodes4(self):
        """The BVH4: (nodes, 37) u32 rows (include/wpt.h wpt_debug_scene_nodes4)."""
        out = np.empty((self.num_nodes4, 37), dtype=np.uint32)
        if self.num_nodes4:
            lib().wpt_debug_scene_nodes4(self.h, out.ctypes.data)
        return out

    def shapes(self):
        out = np.empty((self.num_shapes, 16), dtype=np.float32)
        lib().wpt_debug_scene_shapes(self.h, out.ctypes.data)
        return out

    def lights(self):
        out = np.empty(self.num_lights, dtype=np.uint32)
        lib().wpt_debug_scene_lights(self.h, out.ctypes.data)
        return out

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().wpt_debug_scene_free(self.h)
                self.h = None
        except Exception:
            pass
