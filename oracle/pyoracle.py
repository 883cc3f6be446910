"""ORACLE — TEST INFRASTRUCTURE ONLY. ctypes binding of oracle/liboracle.so
(the C++ CPU restatement of the reference, see ref_core.h). Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_L = None
c_p, c_u32, c_sz, c_int = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_int


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_new.restype = c_p
        L.oracle_new.argtypes = [c_int, c_p, c_sz]
        L.oracle_free.argtypes = [c_p]
        for f in ("oracle_num_shapes", "oracle_num_inf", "oracle_num_nodes", "oracle_num_lights"):
            getattr(L, f).restype = c_sz
            getattr(L, f).argtypes = [c_p]
        L.oracle_bvh_kind.argtypes = [c_p]
        L.oracle_get_nodes.argtypes = [c_p, c_p]
        L.oracle_get_shapes.argtypes = [c_p, c_p]
        L.oracle_verify_bvh.argtypes = [c_p]
        L.oracle_trace_rays.argtypes = [c_p, c_sz, c_p, c_p, c_p, c_p]
        L.oracle_shadow_rays.argtypes = [c_p, c_sz, c_p, c_p, c_p]
        L.oracle_render.argtypes = [c_p, c_u32, c_u32, c_p, c_int, c_int, c_int, c_u32, c_u32, c_u32, c_u32, c_u32,
                                    c_u32, c_u32, c_u32, c_int, c_p, c_p, c_int]
        L.oracle_reference_compute.argtypes = [c_p, c_u32, c_u32, c_p, c_int, c_int, c_int, c_p, c_sz, c_p, c_p, c_p]
        L.oracle_bvh4.restype = c_sz
        L.oracle_bvh4.argtypes = [c_p, c_p]
        L.oracle_torus_trace.argtypes = [c_p, ctypes.c_float, ctypes.c_float, c_p, ctypes.c_size_t, c_p, c_p, c_p]
        L.oracle_sinf.restype = ctypes.c_float
        L.oracle_sinf.argtypes = [ctypes.c_float]
        L.oracle_cosf.restype = ctypes.c_float
        L.oracle_cosf.argtypes = [ctypes.c_float]
        L.oracle_rng_floats.argtypes = [c_u32, c_sz, c_p]
        L.oracle_rng_u32.argtypes = [c_u32, c_sz, c_p]
        L.oracle_path_seed.restype = c_u32
        L.oracle_path_seed.argtypes = [c_u32, c_u32, c_u32]
        L.oracle_shape_trace.argtypes = [c_int, c_p, c_p, c_p, c_p]
        L.oracle_aabb_hit.argtypes = [c_p, c_p, c_p]
        L.oracle_adaptive_new.restype = c_p
        L.oracle_adaptive_new.argtypes = [c_p, c_u32, c_u32, c_p, c_int, c_int, c_int, c_int, c_int, c_u32]
        L.oracle_adaptive_compute.argtypes = [c_p, ctypes.c_uint64, c_int]
        L.oracle_adaptive_read.argtypes = [c_p, c_p, c_p, c_p]
        L.oracle_adaptive_free.argtypes = [c_p]
        L.oracle_photon_tree.restype = c_sz
        L.oracle_photon_tree.argtypes = [c_p, c_u32, c_int, c_p, c_p, c_p]
        _L = L
    return _L


class OracleScene:
    """Scene built by the restatement of scenes.rs (ids 2, 100, 101)."""

    def __init__(self, scene_id, mesh=None):
        L = lib()
        self._mesh = None if mesh is None else np.ascontiguousarray(mesh, dtype=np.float32)
        m = self._mesh
        self.h = L.oracle_new(scene_id, None if m is None else m.ctypes.data, 0 if m is None else m.size // 3)
        if not self.h:
            raise ValueError(f"oracle: unsupported scene {scene_id}")
        self.num_shapes = L.oracle_num_shapes(self.h)
        self.num_inf = L.oracle_num_inf(self.h)
        self.num_nodes = L.oracle_num_nodes(self.h)
        self.num_lights = L.oracle_num_lights(self.h)
        self.bvh_kind = L.oracle_bvh_kind(self.h)

    def nodes(self):
        out = np.empty((self.num_nodes, 8), dtype=np.uint32)
        lib().oracle_get_nodes(self.h, out.ctypes.data)
        return out

    def bvh4(self):
        """The DP tree-cut BVH4 (bvh4.rs:37-281, F4 leaf fix): (nodes, 37) u32 rows."""
        n = lib().oracle_bvh4(self.h, None)
        out = np.empty((n, 37), dtype=np.uint32)
        if n:
            lib().oracle_bvh4(self.h, out.ctypes.data)
        return out

    def shapes(self):
        out = np.empty((self.num_shapes, 16), dtype=np.float32)
        lib().oracle_get_shapes(self.h, out.ctypes.data)
        return out

    def verify_bvh(self):
        return bool(lib().oracle_verify_bvh(self.h))

    def trace_rays(self, rays):
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        n = r.shape[0]
        t = np.empty(n, np.float32)
        ids = np.empty(n, np.int32)
        visits = np.empty(n, np.uint32)
        lib().oracle_trace_rays(self.h, n, r.ctypes.data, t.ctypes.data, ids.ctypes.data, visits.ctypes.data)
        return t, ids, visits

    def shadow_rays(self, pq, light_ids):
        p = np.ascontiguousarray(pq, dtype=np.float32).reshape(-1, 6)
        li = np.ascontiguousarray(light_ids, dtype=np.int32)
        occ = np.empty(p.shape[0], np.uint8)
        lib().oracle_shadow_rays(self.h, p.shape[0], p.ctypes.data, li.ctypes.data, occ.ctypes.data)
        return occ.astype(bool)

    def render(self, width, height, cam, left_type=1, right_type=1, max_depth=0, seed=0xBABABEBE, s0=0, spp=1,
               region=None, row_step=1, threads=1, acc=None, light_debug=0):
        """Per-path-RNG render; returns (acc (H,W,3) float32 sums, stats dict).
        light_debug: the reference's is_light_debug view (is_debug_photons,
        tracer.rs:246-249, :297-299)."""
        if acc is None:
            acc = np.zeros((height, width, 3), dtype=np.float32)
        x0, y0, x1, y1 = region if region is not None else (0, 0, width, height)
        c = np.asarray(cam, dtype=np.float32)
        st = np.zeros(3, dtype=np.uint64)
        lib().oracle_render(self.h, width, height, c.ctypes.data, left_type, right_type, max_depth, seed, s0, spp, x0,
                            y0, x1, y1, row_step, threads, acc.ctypes.data, st.ctypes.data, int(light_debug))
        return acc, {"rays": int(st[0]), "shadow_rays": int(st[1]), "node_visits": int(st[2])}

    def reference_compute(self, width, height, cam, num_samples, left_type=1, right_type=1, max_depth=0,
                          rng_state=0xBABABEBE, acc=None, cnt=None):
        """The reference's own sequential execution model (one xorshift stream)."""
        if acc is None:
            acc = np.zeros((height, width, 3), dtype=np.float32)
        if cnt is None:
            cnt = np.zeros((height, width), dtype=np.uint32)
        c = np.asarray(cam, dtype=np.float32)
        st = np.zeros(3, dtype=np.uint64)
        s = (ctypes.c_uint32 * 1)(rng_state)
        lib().oracle_reference_compute(self.h, width, height, c.ctypes.data, left_type, right_type, max_depth,
                                       ctypes.addressof(s), num_samples, acc.ctypes.data, cnt.ctypes.data,
                                       st.ctypes.data)
        return acc, cnt, int(s[0]), {"rays": int(st[0]), "shadow_rays": int(st[1]), "node_visits": int(st[2])}

    def adaptive(self, width, height, cam, types=(1, 1), adaptive=(0, 1), max_depth=0, seed=0xBABABEBE):
        """Adaptive-sampling session in the GPU core's round schedule."""
        return AdaptiveSession(self, width, height, cam, types, adaptive, max_depth, seed)

    def photon_tree(self, seed=0xBABABEBE, threads=8):
        """PNEE octree (photon_tree.rs) for `seed`: pre-order leaf flags,
        cum_bins per node (num_lights), photons shot, photons stored."""
        L = lib()
        n = L.oracle_photon_tree(self.h, seed, threads, None, None, None)
        leafs = np.empty(n, dtype=np.uint8)
        cum = np.empty(n * max(self.num_lights, 1), dtype=np.float32)
        counts = np.empty(2, dtype=np.uint64)
        L.oracle_photon_tree(self.h, seed, threads, leafs.ctypes.data, cum.ctypes.data, counts.ctypes.data)
        return leafs, cum[: n * self.num_lights].reshape(n, self.num_lights), int(counts[0]), int(counts[1])

    def __del__(self):
        try:
            if getattr(self, "h", None) and _L is not None:
                _L.oracle_free(self.h)
                self.h = None
        except Exception:
            pass


class AdaptiveSession:
    def __init__(self, scene, width, height, cam, types, adaptive, max_depth, seed):
        self.scene, self.W, self.H = scene, width, height  # keeps the scene alive
        c = np.asarray(cam, dtype=np.float32)
        self.h = lib().oracle_adaptive_new(scene.h, width, height, c.ctypes.data, types[0], types[1], adaptive[0],
                                           adaptive[1], max_depth, seed)

    def compute(self, n, threads=8):
        lib().oracle_adaptive_compute(self.h, n, threads)

    def read(self):
        acc = np.empty((self.H, self.W, 3), dtype=np.float32)
        cnt = np.empty((self.H, self.W), dtype=np.uint32)
        samp = np.empty((self.H, self.W, 4), dtype=np.uint8)
        lib().oracle_adaptive_read(self.h, acc.ctypes.data, cnt.ctypes.data, samp.ctypes.data)
        return acc, cnt, samp

    def __del__(self):
        try:
            if self.h and _L is not None:
                _L.oracle_adaptive_free(self.h)
        except Exception:  # noqa: BLE001
            pass


def torus_trace(loc, big_r, small_r, rays):
    """Torus::trace (torus.rs:56-127) of the restatement: (t, normal, hit, entering) per ray."""
    r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
    n = r.shape[0]
    t = np.empty(n, np.float32)
    nrm = np.empty((n, 3), np.float32)
    fl = np.empty(n, np.uint8)
    c = np.ascontiguousarray(loc, dtype=np.float32)
    lib().oracle_torus_trace(c.ctypes.data, big_r, small_r, r.ctypes.data, n, t.ctypes.data, nrm.ctypes.data,
                             fl.ctypes.data)
    return t, nrm, (fl & 1) != 0, (fl & 2) != 0
