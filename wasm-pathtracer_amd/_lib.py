"""ctypes binding of libwpt.so (include/wpt.h).

PyTorch is imported first on purpose: it brings its own HIP runtime, and
libwpt.so binds to it by SONAME (libamdhip64.so.7) so one process holds one
HIP runtime. The library is always the in-tree build; there is no fallback.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# WPT_LIB_VARIANT=<v> loads an experiment build ../libwpt_<v>.so (csrc/Makefile
# `variant` target) for A/B measurements; unset = the product library.
_VARIANT = os.environ.get("WPT_LIB_VARIANT", "")
LIB_PATH = os.path.join(HERE, f"libwpt_{_VARIANT}.so" if _VARIANT else "libwpt.so")

_lib = None

c_u32, c_i32, c_f32, c_sz = ctypes.c_uint32, ctypes.c_int32, ctypes.c_float, ctypes.c_size_t
c_p = ctypes.c_void_p

_SIGS = {
    "wpt_init": (ctypes.c_int, [c_u32, c_u32, c_u32, c_f32, c_f32, c_f32, c_f32, c_f32]),
    "wpt_results": (ctypes.POINTER(ctypes.c_uint8), [c_u32]),
    "wpt_update_scene": (ctypes.c_int, [c_u32]),
    "wpt_update_settings": (ctypes.c_int, [c_u32, c_u32, c_u32, c_u32, c_u32]),
    "wpt_update_viewport": (ctypes.c_int, [c_u32, c_u32]),
    "wpt_update_camera": (ctypes.c_int, [c_f32, c_f32, c_f32, c_f32, c_f32]),
    "wpt_allocate_mesh": (ctypes.c_int, [c_u32, c_u32]),
    "wpt_mesh_vertices": (ctypes.POINTER(ctypes.c_float), [c_u32]),
    "wpt_notify_mesh_loaded": (ctypes.c_int, [c_u32]),
    "wpt_load_obj": (ctypes.c_int, [c_u32, ctypes.c_char_p, c_sz, c_p, c_p]),
    "wpt_parse_obj": (ctypes.c_int, [ctypes.c_char_p, c_sz, c_p, c_p, ctypes.c_uint64, c_p]),
    "wpt_allocate_texture": (ctypes.POINTER(ctypes.c_uint8), [c_u32, c_u32, c_u32]),
    "wpt_notify_texture_loaded": (ctypes.c_int, [c_u32]),
    "wpt_compute": (ctypes.c_int, [c_sz]),
    "wpt_last_error": (ctypes.c_char_p, []),
    "wpt_set_device": (ctypes.c_int, [ctypes.c_int]),
    "wpt_set_render_options": (ctypes.c_int, [c_i32, c_u32, ctypes.c_uint64]),
    "wpt_set_partition": (ctypes.c_int, [c_u32, c_u32, c_u32]),
    "wpt_partition_pixels": (ctypes.c_int64, [c_p]),
    "wpt_tile_partition": (ctypes.c_int64, [c_u32, c_u32, c_u32, c_u32, c_u32, c_p]),
    "wpt_photon_tree": (ctypes.c_int64, [c_p, c_p, c_p]),
    "wpt_read_radiance": (ctypes.c_int, [c_p, c_p]),
    "wpt_copy_partition": (ctypes.c_int, [c_p]),
    "wpt_set_exchange": (ctypes.c_int, [c_p, c_p, c_p, c_p, ctypes.c_uint64]),
    "wpt_exchange_slot": (ctypes.c_int64, []),
    "wpt_stats": (ctypes.c_int, [c_p, c_sz]),
    "wpt_kernel_times": (ctypes.c_int, [c_p, c_sz]),
    "wpt_set_counting": (ctypes.c_int, [ctypes.c_int]),
    "wpt_set_profiling": (ctypes.c_int, [ctypes.c_int]),
    "wpt_set_lanes": (ctypes.c_int, [ctypes.c_int32]),
    "wpt_set_option": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64]),
    "wpt_get_option": (ctypes.c_int, [ctypes.c_int32, c_p]),
    "wpt_probe_read": (ctypes.c_int64, [c_p, c_p, c_p, c_p]),
    "wpt_scene_build_info": (ctypes.c_int, [c_p]),
    "wpt_clear_stats": (ctypes.c_int, []),
    "wpt_sync": (ctypes.c_int, []),
    "wpt_bvh_depth": (ctypes.c_int, []),
    "wpt_trace_rays": (ctypes.c_int, [c_sz, c_p, c_p, c_p]),
    "wpt_shadow_rays": (ctypes.c_int, [c_sz, c_p, c_p, c_p]),
    "wpt_shutdown": (ctypes.c_int, []),
    "wpt_debug_scene_new": (c_p, [c_i32, c_p, c_sz]),
    "wpt_debug_scene_info": (ctypes.c_int, [c_p, c_p]),
    "wpt_debug_scene_nodes": (ctypes.c_int, [c_p, c_p]),
    "wpt_debug_scene_shapes": (ctypes.c_int, [c_p, c_p]),
    "wpt_debug_scene_nodes4": (ctypes.c_int, [c_p, c_p]),
    "wpt_comm_unique_id": (ctypes.c_int, [c_p]),
    "wpt_set_comm": (ctypes.c_int, [c_u32, c_u32, c_u32, c_p]),
    "wpt_gather_frame": (ctypes.c_int, [c_u32]),
    "wpt_comm_destroy": (ctypes.c_int, []),
    "wpt_set_transport": (ctypes.c_int, [c_p, c_p, c_p, c_p, ctypes.c_uint64]),
    "wpt_gather_plan": (ctypes.c_int64, [c_u32, c_u32, c_u32, ctypes.c_uint64, c_p]),
    "wpt_seq_sum": (ctypes.c_float, [c_p, ctypes.c_uint64]),
    "wpt_seq_sum_chunks": (ctypes.c_float, [c_p, ctypes.c_uint64]),
    "wpt_seq_sum_device": (ctypes.c_int, [c_p, ctypes.c_uint64, c_p]),
    "wpt_debug_scene_lights": (ctypes.c_int, [c_p, c_p]),
    "wpt_debug_scene_free": (None, [c_p]),
    "wpt_debug_scene_new_gpu": (c_p, [c_i32, c_p, c_sz]),
    "wpt_debug_scene_build_info": (ctypes.c_int, [c_p, c_p]),
}

EXPORTED = tuple(_SIGS)


def header_symbols():
    """Function names declared in include/wpt.h."""
    import re
    hdr = os.path.join(os.path.dirname(HERE), "include", "wpt.h")
    txt = open(hdr).read()
    return sorted(set(re.findall(r"\b(wpt_[a-z_0-9]+)\s*\(", txt)))


def lib():
    """Load the in-tree libwpt.so (fails loudly if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  (one HIP runtime per process: torch's)
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C wasm-pathtracer_amd/csrc)")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        f = getattr(L, name)  # every build (variants too: make variant checks the exports) binds every symbol
        f.restype = res
        f.argtypes = args
    _lib = L
    return L
