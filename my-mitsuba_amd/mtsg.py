"""ctypes bindings for the MI355X `path` integrator.

Two shared libraries, both built in-tree by ``make`` (``__graft_entry__.build()``):

* ``libmtsg_host.so`` -- Mitsuba-side scene loading + SAH kd-tree build
  (include/mtsh.h); no GPU code.
* ``libmtsg.so``      -- the HIP/gfx950 wavefront path tracer behind the C-ABI
  drop-in boundary (include/mtsg.h).

This module is the Python mirror of the reference's plugin surface used by the
tests and the benchmark.  It never falls back to a CPU path: if the HIP
library is missing, :func:`device_lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)

MTSG_OK = 0
MTSH_INSTANCING_FLATTEN = 0
MTSH_INSTANCING_TWO_LEVEL = 1
MTSG_FLAG_TIMING = 1
MTSG_FLAG_COUNT = 2
MTSG_FLAG_WAVETIME = 4
# mtsg_set_option keys (include/mtsg.h)
MTSG_OPT_TRACE_REFILL = 1
MTSG_OPT_FINISH_SHADE_MIN = 2
MTSG_OPT_LANES = 3
MTSG_OPT_STAGGER = 4
MTSG_OPT_SHADE_GENERIC = 5
MTSG_OPT_RAY_ORDER = 6
MTSG_OPT_CAMERA_DIFFS = 7


class RenderParams(C.Structure):
    """mtsg_render_params (include/mtsg.h)."""
    _fields_ = [
        ("max_depth", C.c_int32), ("rr_depth", C.c_int32),
        ("strict_normals", C.c_int32), ("hide_emitters", C.c_int32),
        ("spp", C.c_uint32), ("seed", C.c_uint32),
        ("tile_x", C.c_int32), ("tile_y", C.c_int32),
        ("tile_w", C.c_int32), ("tile_h", C.c_int32),
        ("tile_stride", C.c_int32), ("tile_offset", C.c_int32),
        ("integrator", C.c_int32), ("om_strategy", C.c_int32), ("om_mis", C.c_int32), ("om_jitter", C.c_int32),
    ]

    def copy(self) -> "RenderParams":
        p = RenderParams()
        C.memmove(C.byref(p), C.byref(self), C.sizeof(RenderParams))
        return p


class TestKnobs(C.Structure):
    """mtsg_test_knobs (TEST ONLY: the traversal's stack sizes and restart guard)."""
    _fields_ = [("stack_cap", C.c_int32), ("restart_guard", C.c_int32), ("restart_limit", C.c_int32),
                ("limit_shadow_only", C.c_int32), ("no_instance_prefilter", C.c_int32)]


class Stats(C.Structure):
    """mtsg_stats."""
    _fields_ = [
        ("ms_total", C.c_double), ("ms_trace_closest", C.c_double),
        ("ms_trace_shadow", C.c_double), ("ms_shade", C.c_double),
        ("ms_camera", C.c_double), ("ms_splat", C.c_double),
        ("launches_trace_closest", C.c_uint64),
        ("rays_closest", C.c_uint64), ("rays_shadow", C.c_uint64),
        ("samples", C.c_uint64),
        ("nodes_visited", C.c_uint64), ("leaf_refs", C.c_uint64),
        ("tri_tests", C.c_uint64),
        ("shadow_nodes_visited", C.c_uint64), ("shadow_leaf_refs", C.c_uint64),
        ("shadow_tri_tests", C.c_uint64),
        ("wave_node_iters", C.c_uint64), ("wave_test_iters", C.c_uint64),
        ("wave_steps", C.c_uint64), ("wave_active_lanes", C.c_uint64),
        ("shadow_wave_node_iters", C.c_uint64), ("shadow_wave_test_iters", C.c_uint64),
        ("shadow_wave_steps", C.c_uint64), ("shadow_wave_active_lanes", C.c_uint64),
        ("launches_trace_shadow", C.c_uint64),
        ("iter_max_closest", C.c_uint64), ("iter_max_shadow", C.c_uint64),
        ("iter_hist_closest", C.c_uint64 * 16), ("iter_hist_shadow", C.c_uint64 * 16),
        ("instance_visits", C.c_uint64), ("shadow_instance_visits", C.c_uint64),
        ("ms_finish", C.c_double), ("paths_finish", C.c_uint64), ("launches_finish", C.c_uint64),
        ("tie_retraces", C.c_uint64), ("guard_rays_closest", C.c_uint64), ("guard_rays_shadow", C.c_uint64),
        ("guard_steps_closest", C.c_uint64), ("guard_steps_shadow", C.c_uint64),
        ("restarts_closest", C.c_uint64), ("restarts_shadow", C.c_uint64),
        ("instance_rejects", C.c_uint64), ("instance_prefiltered", C.c_uint64),
        ("ms_sort", C.c_double),
    ]


class MipMapHeader(C.Structure):
    """mtsg_mipmap (include/mtsg.h)."""
    _fields_ = [
        ("levels", C.c_int32), ("filter", C.c_int32), ("wrap_u", C.c_int32), ("wrap_v", C.c_int32),
        ("level_w", C.c_int32 * 24), ("level_h", C.c_int32 * 24), ("level_offset", C.c_uint32 * 24),
        ("size_ratio_x", C.c_float * 24), ("size_ratio_y", C.c_float * 24),
        ("max_anisotropy", C.c_float), ("pad", C.c_int32 * 3), ("weight_lut", C.c_float * 64),
    ]


class KDBuildParams(C.Structure):
    """mtsg_kd_build_params (include/mtsg.h)."""
    _fields_ = [("traversal_cost", C.c_float), ("query_cost", C.c_float), ("empty_space_bonus", C.c_float),
                ("stop_prims", C.c_int32), ("max_depth", C.c_int32), ("pad", C.c_int32)]


class KDTree(C.Structure):
    """mtsg_kd_tree (include/mtsg.h)."""
    _fields_ = [("nodes", C.POINTER(C.c_uint32)), ("n_nodes", C.c_uint32), ("indices", C.POINTER(C.c_uint32)),
                ("n_indices", C.c_uint32), ("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3),
                ("max_depth", C.c_uint32), ("leaves", C.c_uint32), ("ms_build", C.c_double)]


def kd_build(scene: "Scene", bounds: np.ndarray | None = None, device: int = 0, **params) -> dict:
    """SAH kd-tree over the scene's primitives built on the GPU (mtsg_kd_build);
    bounds: their boxes (n, 6), by default scene.prim_bounds().  Costs are
    Mitsuba's (gkdtree.h:734-744); leaves stop at 4 primitives like the host
    build's GPU-tuned default (params, e.g. stop_prims=6, override them)."""
    lib = device_lib()
    b = np.ascontiguousarray(scene.prim_bounds() if bounds is None else bounds, dtype=np.float32)
    p = KDBuildParams(15.0, 20.0, 0.9, 4, 0, 0)
    for k, v in params.items():
        setattr(p, k, v)
    t = KDTree()
    if lib.mtsg_kd_build(device, scene.desc, _ptr(b), C.byref(p), C.byref(t)) != 0:
        raise RuntimeError(_err(lib, "mtsg_last_error"))
    return _take_tree(lib, t)


def _take_tree(lib, t: "KDTree") -> dict:
    try:
        out = dict(nodes=np.ctypeslib.as_array(t.nodes, (t.n_nodes * 2,)).reshape(-1, 2).copy(),
                   indices=np.ctypeslib.as_array(t.indices, (max(t.n_indices, 1),))[:t.n_indices].copy(),
                   aabb_min=np.array(t.aabb_min[:], np.float32), aabb_max=np.array(t.aabb_max[:], np.float32),
                   max_depth=t.max_depth, leaves=t.leaves, ms=t.ms_build)
    finally:
        lib.mtsg_kd_free(C.byref(t))
    return out


def kd_refit(scene: "Scene", tree: dict, bounds: np.ndarray | None = None, device: int = 0) -> dict:
    """The tree's nodes and split planes kept, its leaves refilled on the GPU
    from the scene's current primitives (mtsg_kd_refit); tree: a dict of
    kd_build's form (nodes (n, 2) uint32, indices)."""
    lib = device_lib()
    b = np.ascontiguousarray(scene.prim_bounds() if bounds is None else bounds, dtype=np.float32)
    nodes = np.ascontiguousarray(tree["nodes"], dtype=np.uint32)
    idx = np.ascontiguousarray(tree["indices"], dtype=np.uint32)
    tin = KDTree()
    tin.nodes = nodes.ctypes.data_as(C.POINTER(C.c_uint32))
    tin.n_nodes = nodes.shape[0]
    tin.indices = idx.ctypes.data_as(C.POINTER(C.c_uint32))
    tin.n_indices = idx.size
    t = KDTree()
    if lib.mtsg_kd_refit(device, scene.desc, _ptr(b), C.byref(tin), C.byref(t)) != 0:
        raise RuntimeError(_err(lib, "mtsg_last_error"))
    return _take_tree(lib, t)


class OMHeader(C.Structure):
    """mtsg_om (include/mtsg.h)."""
    _fields_ = [("aabb_min", C.c_float * 3), ("grid_size_recp", C.c_float), ("center", C.c_float * 3), ("pad", C.c_float),
                ("dir", (C.c_float * 3) * 16), ("rotate", (C.c_float * 9) * 16)]


class TextureHeader(C.Structure):
    """mtsg_texture (include/mtsg.h)."""
    _fields_ = [("mip", MipMapHeader), ("uv_offset", C.c_float * 2), ("uv_scale", C.c_float * 2), ("scale", C.c_float),
                ("average", C.c_float * 3), ("maximum", C.c_float * 3), ("pad", C.c_int32 * 3)]


class SceneInfo(C.Structure):
    """mtsh_scene_info."""
    _fields_ = [
        ("n_triangles", C.c_uint32), ("n_rects", C.c_uint32), ("n_shapes", C.c_uint32),
        ("n_emitters", C.c_uint32), ("n_bsdfs", C.c_uint32),
        ("kd_nodes", C.c_uint32), ("kd_indices", C.c_uint32), ("kd_max_depth", C.c_uint32),
        ("kd_leaves", C.c_uint32), ("kd_nonempty_leaves", C.c_uint32),
        ("kd_build_seconds", C.c_double),
        ("film_w", C.c_int32), ("film_h", C.c_int32), ("spp", C.c_int32),
        ("border", C.c_int32), ("max_depth", C.c_int32),
    ]


class SceneOverrides(C.Structure):
    """mtsh_scene_overrides: the values a Mitsuba plugin holds in memory."""
    _fields_ = [("mask", C.c_uint32), ("film_width", C.c_int32), ("film_height", C.c_int32),
                ("sample_count", C.c_int32), ("max_depth", C.c_int32), ("rr_depth", C.c_int32),
                ("strict_normals", C.c_int32), ("hide_emitters", C.c_int32),
                ("crop_x", C.c_int32), ("crop_y", C.c_int32), ("crop_width", C.c_int32), ("crop_height", C.c_int32)]


MTSH_OVERRIDE_FILM_SIZE, MTSH_OVERRIDE_SAMPLE_COUNT, MTSH_OVERRIDE_INTEGRATOR, MTSH_OVERRIDE_FILM_CROP = 1, 2, 4, 8


class Prop(C.Structure):
    """mtsh_prop: one entry of a Mitsuba Properties object (include/mtsh.h)."""
    _fields_ = [("name", C.c_char_p), ("type", C.c_int32), ("pad", C.c_int32), ("i", C.c_int64), ("f", C.c_float),
                ("v", C.c_float * 3), ("m", C.c_float * 16), ("inv", C.c_float * 16), ("s", C.c_char_p)]


class MeshArrays(C.Structure):
    """mtsh_mesh: a TriMesh's arrays."""
    _fields_ = [("name", C.c_char_p), ("n_vertices", C.c_uint32), ("n_triangles", C.c_uint32),
                ("positions", C.c_void_p), ("normals", C.c_void_p), ("texcoords", C.c_void_p), ("indices", C.c_void_p),
                ("face_normals", C.c_int32), ("flip_normals", C.c_int32), ("to_world", C.c_void_p),
                ("to_world_inv", C.c_void_p)]


class DigestEntry(C.Structure):
    """mtsh_digest_entry."""
    _fields_ = [("name", C.c_char * 32), ("bytes", C.c_uint64), ("hash", C.c_uint64)]


PROP_TYPES = {"boolean": 0, "integer": 1, "float": 2, "point": 3, "vector": 4, "transform": 5, "spectrum": 6,
              "string": 7, "texture": 8}

_host = None
_dev = None

DEVICE_SYMBOLS = [
    "mtsg_device_count", "mtsg_device_pci_id", "mtsg_scene_create", "mtsg_render", "mtsg_render_device",
    "mtsg_tile_windows", "mtsg_render_device_tiles", "mtsg_set_tile_list",
    "mtsg_device_alloc", "mtsg_device_free", "mtsg_device_memset", "mtsg_device_to_host",
    "mtsg_cancel", "mtsg_cancel_clear", "mtsg_set_flags", "mtsg_get_stats", "mtsg_set_batch_paths", "mtsg_set_finish_paths",
    "mtsg_trace_closest", "mtsg_trace_shadow", "mtsg_render_samples", "mtsg_scene_destroy",
    "mtsg_last_error", "mtsg_env_eval", "mtsg_tex_eval", "mtsg_om_query", "mtsg_kd_build", "mtsg_kd_refit", "mtsg_kd_free",
    "mtsg_sampler_draws", "mtsg_debug_wavetimes", "mtsg_set_tile_callback",
    "mtsg_debug_stragglers", "mtsg_set_test_knobs", "mtsg_set_option",
]
HOST_SYMBOLS = [
    "mtsh_scene_load", "mtsh_scene_load_overrides", "mtsh_scene_load_props", "mtsh_scene_set_scene_props", "mtsh_set_kd_threads", "mtsh_set_instancing", "mtsh_scene_desc", "mtsh_scene_render_params",
    "mtsh_scene_get_info", "mtsh_scene_free", "mtsh_develop", "mtsh_write_pfm", "mtsh_rough_transmittance",
    "mtsh_read_image", "mtsh_clip_triangle", "mtsh_texture_image", "mtsh_build_mipmap", "mtsh_scene_textures", "mtsh_scene_om", "mtsh_scene_prim_bounds", "mtsh_scene_set_kdtree",
    "mtsh_last_error",
    "mtsh_scene_begin", "mtsh_scene_add_texture", "mtsh_scene_add_bsdf", "mtsh_scene_add_emitter", "mtsh_scene_add_group",
    "mtsh_scene_add_shape", "mtsh_scene_add_mesh", "mtsh_scene_add_instance", "mtsh_scene_set_sensor", "mtsh_scene_set_film",
    "mtsh_scene_set_sampler", "mtsh_scene_set_integrator", "mtsh_scene_finish", "mtsh_scene_abort", "mtsh_scene_digest",
]
PATH_SYMBOLS = [
    "mtsh_path_job_create", "mtsh_path_job_gpus", "mtsh_path_job_render", "mtsh_path_job_cancel",
    "mtsh_path_job_destroy", "mtsh_path_render", "mtsh_path_last_error", "mtsh_path_job_set_tile_callback",
    "mtsh_path_job_set_balance", "mtsh_path_job_shares",
]

# tile completion hooks (mtsg_set_tile_callback, mtsh_path_job_set_tile_callback)
TILE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32)
_path = None


def path_lib() -> C.CDLL:
    """libmtsg_path.so: the multi-GPU render() / cancel() (include/mtsg_path.h)."""
    global _path
    if _path is None:
        device_lib()   # raises when the HIP library is missing
        path = os.path.join(PKG_DIR, "libmtsg_path.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: run `make` (or __graft_entry__.build())")
        lib = C.CDLL(path)
        lib.mtsh_path_job_create.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
        lib.mtsh_path_job_gpus.argtypes = [C.c_void_p]
        lib.mtsh_path_job_render.argtypes = [C.c_void_p, C.POINTER(RenderParams), C.c_void_p,
                                             C.POINTER(C.c_double)]
        lib.mtsh_path_job_cancel.argtypes = [C.c_void_p]
        lib.mtsh_path_job_destroy.argtypes = [C.c_void_p]
        lib.mtsh_path_job_set_tile_callback.argtypes = [C.c_void_p, TILE_FN, C.c_void_p]
        lib.mtsh_path_job_set_balance.argtypes = [C.c_void_p, C.c_int]
        lib.mtsh_path_job_shares.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        lib.mtsh_path_render.argtypes = [C.c_void_p, C.POINTER(RenderParams), C.c_int, C.c_void_p,
                                         C.POINTER(C.c_double)]
        lib.mtsh_path_last_error.argtypes = [C.c_char_p, C.c_size_t]
        _path = lib
    return _path


def host_lib() -> C.CDLL:
    global _host
    if _host is None:
        path = os.path.join(PKG_DIR, "libmtsg_host.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: run `make host` (or __graft_entry__.build())")
        lib = C.CDLL(path)
        lib.mtsh_scene_load.restype = C.c_void_p
        lib.mtsh_scene_load.argtypes = [C.c_char_p, C.POINTER(C.c_char_p), C.c_int]
        lib.mtsh_scene_load_overrides.restype = C.c_void_p
        lib.mtsh_scene_load_overrides.argtypes = [C.c_char_p, C.POINTER(C.c_char_p), C.c_int, C.POINTER(SceneOverrides)]
        lib.mtsh_scene_load_props.restype = C.c_void_p
        lib.mtsh_scene_load_props.argtypes = [C.c_char_p, C.POINTER(C.c_char_p), C.c_int, C.POINTER(SceneOverrides),
                                              C.POINTER(Prop), C.c_int32]
        lib.mtsh_scene_desc.restype = C.c_void_p
        lib.mtsh_scene_desc.argtypes = [C.c_void_p]
        lib.mtsh_scene_render_params.argtypes = [C.c_void_p, C.POINTER(RenderParams)]
        lib.mtsh_scene_get_info.argtypes = [C.c_void_p, C.POINTER(SceneInfo)]
        lib.mtsh_scene_free.argtypes = [C.c_void_p]
        lib.mtsh_develop.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        lib.mtsh_write_pfm.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_void_p]
        lib.mtsh_last_error.argtypes = [C.c_char_p, C.c_size_t]
        lib.mtsh_set_kd_threads.argtypes = [C.c_int]
        lib.mtsh_set_instancing.argtypes = [C.c_int]
        lib.mtsh_read_image.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_void_p, C.c_size_t]
        lib.mtsh_clip_triangle.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        lib.mtsh_scene_textures.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        lib.mtsh_scene_om.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        lib.mtsh_scene_prim_bounds.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        lib.mtsh_scene_prim_bounds.restype = C.c_int64
        lib.mtsh_scene_set_kdtree.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p,
                                              C.c_void_p, C.c_uint32]
        lib.mtsh_texture_image.argtypes = [C.c_char_p, C.c_float, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_void_p,
                                           C.c_size_t]
        lib.mtsh_build_mipmap.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float,
                                          C.POINTER(MipMapHeader), C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                                          C.c_void_p, C.c_void_p]
        PP = C.POINTER(Prop)
        lib.mtsh_scene_begin.restype = C.c_void_p
        lib.mtsh_scene_begin.argtypes = [C.c_char_p]
        for fn in ("mtsh_scene_add_texture", "mtsh_scene_add_emitter", "mtsh_scene_set_sensor", "mtsh_scene_set_sampler",
                   "mtsh_scene_set_integrator"):
            getattr(lib, fn).restype = C.c_int32
            getattr(lib, fn).argtypes = [C.c_void_p, C.c_char_p, PP, C.c_int32]
        lib.mtsh_scene_set_scene_props.restype = C.c_int32
        lib.mtsh_scene_set_scene_props.argtypes = [C.c_void_p, PP, C.c_int32]
        lib.mtsh_scene_add_bsdf.restype = C.c_int32
        lib.mtsh_scene_add_bsdf.argtypes = [C.c_void_p, C.c_char_p, PP, C.c_int32, C.POINTER(C.c_int32), C.c_int32]
        lib.mtsh_scene_add_group.restype = C.c_int32
        lib.mtsh_scene_add_group.argtypes = [C.c_void_p, C.c_char_p]
        lib.mtsh_scene_add_shape.restype = C.c_int32
        lib.mtsh_scene_add_shape.argtypes = [C.c_void_p, C.c_char_p, PP, C.c_int32, C.c_int32, C.c_int32, C.c_int32]
        lib.mtsh_scene_add_mesh.restype = C.c_int32
        lib.mtsh_scene_add_mesh.argtypes = [C.c_void_p, C.POINTER(MeshArrays), C.c_int32, C.c_int32, C.c_int32]
        lib.mtsh_scene_add_instance.restype = C.c_int32
        lib.mtsh_scene_add_instance.argtypes = [C.c_void_p, C.c_int32, PP, C.c_int32]
        lib.mtsh_scene_set_film.restype = C.c_int32
        lib.mtsh_scene_set_film.argtypes = [C.c_void_p, C.c_char_p, PP, C.c_int32, C.c_char_p, PP, C.c_int32]
        lib.mtsh_scene_finish.restype = C.c_void_p
        lib.mtsh_scene_finish.argtypes = [C.c_void_p, C.POINTER(SceneOverrides)]
        lib.mtsh_scene_abort.argtypes = [C.c_void_p]
        lib.mtsh_scene_digest.restype = C.c_int32
        lib.mtsh_scene_digest.argtypes = [C.c_void_p, C.POINTER(DigestEntry), C.c_int32]
        _host = lib
    return _host


def device_lib() -> C.CDLL:
    """The HIP library.  Raises (never falls back) when it is missing."""
    global _dev
    if _dev is None:
        # MTSG_LIB: alternative in-tree build, relative to the repository root
        # (measurement variants under build/var/ only)
        alt = os.environ.get("MTSG_LIB")
        path = os.path.join(os.path.dirname(PKG_DIR), alt) if alt else os.path.join(PKG_DIR, "libmtsg.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: the HIP extension was not built "
                               "(run `make device` / __graft_entry__.build()); no CPU fallback exists")
        lib = C.CDLL(path)
        lib.mtsg_device_count.restype = C.c_int
        lib.mtsg_device_pci_id.argtypes = [C.c_int, C.c_char_p, C.c_int]
        lib.mtsg_scene_create.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
        lib.mtsg_render.argtypes = [C.c_void_p, C.POINTER(RenderParams), C.c_void_p]
        lib.mtsg_render_device.argtypes = [C.c_void_p, C.POINTER(RenderParams), C.c_void_p]
        lib.mtsg_tile_windows.argtypes = [C.c_void_p, C.POINTER(RenderParams), C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_int32)]
        lib.mtsg_render_device_tiles.argtypes = [C.c_void_p, C.POINTER(RenderParams), C.c_void_p]
        lib.mtsg_set_tile_list.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
        lib.mtsg_device_alloc.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]
        lib.mtsg_device_free.argtypes = [C.c_void_p, C.c_void_p]
        lib.mtsg_device_memset.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        lib.mtsg_device_to_host.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        lib.mtsg_cancel.argtypes = [C.c_void_p]
        lib.mtsg_cancel_clear.argtypes = [C.c_void_p]
        lib.mtsg_set_flags.argtypes = [C.c_void_p, C.c_uint32]
        lib.mtsg_get_stats.argtypes = [C.c_void_p, C.POINTER(Stats)]
        lib.mtsg_set_batch_paths.argtypes = [C.c_void_p, C.c_uint32]
        lib.mtsg_set_finish_paths.argtypes = [C.c_void_p, C.c_uint32]
        lib.mtsg_set_option.argtypes = [C.c_void_p, C.c_int32, C.c_int64]
        lib.mtsg_trace_closest.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p]
        lib.mtsg_trace_shadow.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
        lib.mtsg_render_samples.argtypes = [C.c_void_p, C.POINTER(RenderParams), C.c_void_p]
        lib.mtsg_env_eval.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.mtsg_tex_eval.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.mtsg_kd_build.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.POINTER(KDBuildParams), C.POINTER(KDTree)]
        lib.mtsg_kd_free.argtypes = [C.POINTER(KDTree)]
        lib.mtsg_kd_refit.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.POINTER(KDTree), C.POINTER(KDTree)]
        lib.mtsg_om_query.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.mtsg_sampler_draws.argtypes = [C.c_void_p, C.POINTER(RenderParams), C.c_int, C.c_int, C.c_uint32,
                                           C.c_uint32, C.c_void_p, C.c_void_p]
        lib.mtsg_scene_destroy.argtypes = [C.c_void_p]
        lib.mtsg_set_tile_callback.argtypes = [C.c_void_p, TILE_FN, C.c_void_p]
        lib.mtsg_set_test_knobs.argtypes = [C.c_void_p, C.POINTER(TestKnobs)]
        lib.mtsg_last_error.argtypes = [C.c_char_p, C.c_size_t]
        _dev = lib
    return _dev


def device_pci_id(device: int) -> str:
    """PCI address of visible device `device` (mtsg_device_pci_id)."""
    buf = C.create_string_buffer(64)
    lib = device_lib()
    if lib.mtsg_device_pci_id(device, buf, 64) != MTSG_OK:
        raise RuntimeError(_err(lib, "mtsg_last_error"))
    return buf.value.decode()


def _err(lib, fn) -> str:
    buf = C.create_string_buffer(4096)
    getattr(lib, fn)(buf, 4096)
    return buf.value.decode(errors="replace")


def _ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


class Scene:
    """A loaded Mitsuba XML scene (host side; owns the flat descriptor)."""

    def __init__(self, path: str, defines: dict | None = None, kd_threads: int = 0, instancing: str = "flatten",
                 overrides: SceneOverrides | None = None, scene_props=None):
        """instancing: "flatten" (instances become world-space triangles of the
        one scene tree) or "two-level" (Mitsuba's instance / shapegroup
        structure: per-group trees, rays transformed per instance visit).
        scene_props: the Scene's own Properties as [(name, kind, value)] or
        {name: value} (ints -> integer, floats -> float, bools -> boolean),
        applied after the file's <scene>-level ones (mtsh_scene_load_props:
        the kd-tree build parameters of scene.cpp:47-83)."""
        lib = host_lib()
        lib.mtsh_set_kd_threads(kd_threads)
        if instancing not in ("flatten", "two-level"):
            raise ValueError(f"instancing must be 'flatten' or 'two-level', not {instancing!r}")
        lib.mtsh_set_instancing(MTSH_INSTANCING_TWO_LEVEL if instancing == "two-level" else MTSH_INSTANCING_FLATTEN)
        defs = [f"{k}={v}".encode() for k, v in (defines or {}).items()]
        arr = (C.c_char_p * max(1, len(defs)))(*defs)
        if scene_props:
            pa, pn, _keep = _props(_scene_prop_list(scene_props))
            self._h = lib.mtsh_scene_load_props(path.encode(), arr, len(defs),
                                                C.byref(overrides) if overrides is not None else None, pa, pn)
        elif overrides is None:
            self._h = lib.mtsh_scene_load(path.encode(), arr, len(defs))
        else:
            self._h = lib.mtsh_scene_load_overrides(path.encode(), arr, len(defs), C.byref(overrides))
        if not self._h:
            raise RuntimeError("scene load failed: " + _err(lib, "mtsh_last_error"))
        self.path = path
        self.defines = dict(defines or {})
        self.instancing = instancing
        self.info = SceneInfo()
        lib.mtsh_scene_get_info(self._h, C.byref(self.info))

    @classmethod
    def _adopt(cls, handle, label: str, instancing: str) -> "Scene":
        """A scene made by SceneBuilder.finish (it takes the handle over)."""
        self = cls.__new__(cls)
        self._h = handle
        self.path = label
        self.defines = {}
        self.instancing = instancing
        self.info = SceneInfo()
        host_lib().mtsh_scene_get_info(self._h, C.byref(self.info))
        return self

    def digest(self) -> dict:
        """mtsh_scene_digest: {descriptor array: (bytes, FNV-1a 64)}."""
        lib = host_lib()
        n = lib.mtsh_scene_digest(self._h, None, 0)
        arr = (DigestEntry * n)()
        lib.mtsh_scene_digest(self._h, arr, n)
        return {e.name.decode(): (int(e.bytes), int(e.hash)) for e in arr}

    @property
    def desc(self) -> C.c_void_p:
        return C.c_void_p(host_lib().mtsh_scene_desc(self._h))

    def params(self, **overrides) -> RenderParams:
        p = RenderParams()
        host_lib().mtsh_scene_render_params(self._h, C.byref(p))
        for k, v in overrides.items():
            setattr(p, k, v)
        return p

    @property
    def border(self) -> int:
        return self.info.border

    def prim_bounds(self) -> np.ndarray:
        """The top-level kd-tree's primitive boxes (n, 6); empty boxes mark
        primitives the tree leaves out."""
        lib = host_lib()
        n = lib.mtsh_scene_prim_bounds(self._h, None, 0)
        out = np.zeros((n, 6), np.float32)
        if lib.mtsh_scene_prim_bounds(self._h, _ptr(out), out.size) != n:
            raise RuntimeError(_err(lib, "mtsh_last_error"))
        return out

    def set_kdtree(self, tree: dict) -> None:
        """Install a kd-tree (kd_build's dict) as the scene's top-level tree."""
        lib = host_lib()
        nodes = np.ascontiguousarray(tree["nodes"], dtype=np.uint32)
        idx = np.ascontiguousarray(tree["indices"], dtype=np.uint32)
        lo = np.ascontiguousarray(tree["aabb_min"], dtype=np.float32)
        hi = np.ascontiguousarray(tree["aabb_max"], dtype=np.float32)
        if lib.mtsh_scene_set_kdtree(self._h, _ptr(nodes), nodes.shape[0], _ptr(idx), idx.size, _ptr(lo), _ptr(hi),
                                     int(tree["max_depth"])) != 0:
            raise RuntimeError(_err(lib, "mtsh_last_error"))

    def occupancy_maps(self):
        """myPath2_OM's maps: (header OMHeader, bits (16, 256, 256, 8) uint32)."""
        lib = host_lib()
        hdr = OMHeader()
        bits = np.zeros((16, 256, 256, 8), np.uint32)
        if lib.mtsh_scene_om(self._h, C.byref(hdr), _ptr(bits), bits.size) != 0:
            raise RuntimeError(_err(lib, "mtsh_last_error"))
        return hdr, bits

    def textures(self) -> list:
        """The scene's bitmap texture headers (TextureHeader)."""
        lib = host_lib()
        n = lib.mtsh_scene_textures(self._h, None, 0)
        arr = (TextureHeader * max(n, 1))()
        lib.mtsh_scene_textures(self._h, arr, n)
        return list(arr[:n])

    def __del__(self):
        if getattr(self, "_h", None):
            host_lib().mtsh_scene_free(self._h)
            self._h = None


def _scene_prop_list(props):
    """{name: value} -> [(name, kind, value)] (bool before int: bool is an int)."""
    if isinstance(props, dict):
        kind = lambda v: "boolean" if isinstance(v, bool) else "integer" if isinstance(v, int) else "float"  # noqa: E731
        return [(k, kind(v), v) for k, v in props.items()]
    return list(props)


def _props(props) -> tuple:
    """[(name, kind, value)] -> (Prop array, keep-alive list).  kind is a
    Properties type ("boolean", "integer", "float", "point", "vector",
    "spectrum", "string", "transform": (m 4x4[, inverse 4x4]), "texture": an
    id of SceneBuilder.texture)."""
    props = list(props or [])
    arr = (Prop * max(1, len(props)))()
    keep = []
    for k, (name, kind, value) in enumerate(props):
        p = arr[k]
        nb = name.encode()
        keep.append(nb)
        p.name = nb
        p.type = PROP_TYPES[kind]
        if kind in ("boolean", "integer", "texture"):
            p.i = int(value)
        elif kind == "float":
            p.f = float(value)
        elif kind in ("point", "vector", "spectrum"):
            v = np.broadcast_to(np.asarray(value, np.float32), (3,))
            p.v[:] = [float(x) for x in v]
        elif kind == "string":
            sb = str(value).encode()
            keep.append(sb)
            p.s = sb
        elif kind == "transform":
            m, inv = value if isinstance(value, tuple) else (value, None)
            p.m[:] = [float(x) for x in np.asarray(m, np.float32).reshape(16)]
            if inv is not None:
                p.inv[:] = [float(x) for x in np.asarray(inv, np.float32).reshape(16)]
        else:
            raise ValueError(f"unknown property kind {kind!r}")
    return arr, len(props), keep


class SceneBuilder:
    """The in-memory scene builder (mtsh_scene_begin / _add_* / _finish):
    what a Mitsuba-side plugin hands over from the objects it holds."""

    def __init__(self, base_dir: str = ".", instancing: str = "flatten", kd_threads: int = 0):
        lib = host_lib()
        lib.mtsh_set_kd_threads(kd_threads)
        lib.mtsh_set_instancing(MTSH_INSTANCING_TWO_LEVEL if instancing == "two-level" else MTSH_INSTANCING_FLATTEN)
        self.instancing = instancing
        self._b = lib.mtsh_scene_begin(base_dir.encode())
        if not self._b:
            raise RuntimeError(_err(lib, "mtsh_last_error"))

    def _rc(self, rc: int, what: str) -> int:
        if rc < 0:
            raise RuntimeError(f"{what}: " + _err(host_lib(), "mtsh_last_error"))
        return rc

    def texture(self, plugin: str, props) -> int:
        a, n, _k = _props(props)
        return self._rc(host_lib().mtsh_scene_add_texture(self._b, plugin.encode(), a, n), plugin)

    def bsdf(self, plugin: str, props, nested=()) -> int:
        a, n, _k = _props(props)
        kids = (C.c_int32 * max(1, len(nested)))(*nested)
        return self._rc(host_lib().mtsh_scene_add_bsdf(self._b, plugin.encode(), a, n, kids, len(nested)), plugin)

    def emitter(self, plugin: str, props) -> int:
        a, n, _k = _props(props)
        return self._rc(host_lib().mtsh_scene_add_emitter(self._b, plugin.encode(), a, n), plugin)

    def group(self, gid: str) -> int:
        return self._rc(host_lib().mtsh_scene_add_group(self._b, gid.encode()), "shapegroup")

    def shape(self, plugin: str, props, bsdf: int = -1, emitter: int = -1, group: int = -1) -> None:
        a, n, _k = _props(props)
        self._rc(host_lib().mtsh_scene_add_shape(self._b, plugin.encode(), a, n, bsdf, emitter, group), plugin)

    def mesh(self, positions, indices, normals=None, texcoords=None, to_world=None, to_world_inv=None,
             face_normals: bool = False, flip_normals: bool = False, bsdf: int = -1, emitter: int = -1, group: int = -1,
             name: str = "") -> None:
        pos = np.ascontiguousarray(positions, np.float32).reshape(-1, 3)
        idx = np.ascontiguousarray(indices, np.uint32).reshape(-1, 3)
        keep = [pos, idx]
        m = MeshArrays()
        nb = name.encode()
        m.name = nb
        m.n_vertices, m.n_triangles = pos.shape[0], idx.shape[0]
        m.positions, m.indices = _ptr(pos), _ptr(idx)
        for field, arr, width in (("normals", normals, 3), ("texcoords", texcoords, 2), ("to_world", to_world, 16),
                                  ("to_world_inv", to_world_inv, 16)):
            if arr is not None:
                a = np.ascontiguousarray(arr, np.float32).reshape(-1)
                keep.append(a)
                setattr(m, field, _ptr(a))
        m.face_normals, m.flip_normals = int(face_normals), int(flip_normals)
        self._rc(host_lib().mtsh_scene_add_mesh(self._b, C.byref(m), bsdf, emitter, group), "mesh " + name)

    def instance(self, group: int, props) -> None:
        a, n, _k = _props(props)
        self._rc(host_lib().mtsh_scene_add_instance(self._b, group, a, n), "instance")

    def sensor(self, plugin: str, props) -> None:
        a, n, _k = _props(props)
        self._rc(host_lib().mtsh_scene_set_sensor(self._b, plugin.encode(), a, n), plugin)

    def film(self, plugin: str, props, rfilter: str | None = None, rfilter_props=None) -> None:
        a, n, _k = _props(props)
        ra, rn, _rk = _props(rfilter_props)
        self._rc(host_lib().mtsh_scene_set_film(self._b, plugin.encode(), a, n, rfilter.encode() if rfilter else None,
                                                 ra, rn), plugin)

    def sampler(self, plugin: str, props) -> None:
        a, n, _k = _props(props)
        self._rc(host_lib().mtsh_scene_set_sampler(self._b, plugin.encode(), a, n), plugin)

    def integrator(self, plugin: str, props) -> None:
        a, n, _k = _props(props)
        self._rc(host_lib().mtsh_scene_set_integrator(self._b, plugin.encode(), a, n), plugin)

    def scene_props(self, props) -> None:
        """The Scene's own Properties (mtsh_scene_set_scene_props): kd build parameters."""
        a, n, _k = _props(_scene_prop_list(props))
        self._rc(host_lib().mtsh_scene_set_scene_props(self._b, a, n), "scene")

    def finish(self, overrides: SceneOverrides | None = None, label: str = "<builder>") -> Scene:
        lib = host_lib()
        b, self._b = self._b, None
        h = lib.mtsh_scene_finish(b, C.byref(overrides) if overrides is not None else None)
        if not h:
            raise RuntimeError("scene build failed: " + _err(lib, "mtsh_last_error"))
        return Scene._adopt(h, label, self.instancing)

    def __del__(self):
        if getattr(self, "_b", None):
            host_lib().mtsh_scene_abort(self._b)
            self._b = None


def tile_deal_keys(tile_w: int, tile_h: int) -> np.ndarray:
    """Deal key of every pixel of a tile_w x tile_h rectangle (include/mtsg.h
    mtsg_render_params.tile_stride): tile (tx, ty) has key ty * tiles_x +
    (tx - ty) mod tiles_x, and a call with (stride, offset) renders the tiles
    whose key % stride == offset."""
    tiles_x = (tile_w + 15) // 16
    ty, tx = np.meshgrid(np.arange(tile_h) // 16, np.arange(tile_w) // 16, indexing="ij")
    return ty * tiles_x + (tx - ty) % tiles_x


def put_tile_windows(block: np.ndarray, windows: np.ndarray, tile_w: int, tile_h: int, border: int,
                     stride: int, offset: int, keys=None) -> np.ndarray:
    """Add per-tile ImageBlocks (mtsg_render_device_tiles: window v = the tile of
    deal key offset + v * stride, or keys[v] for a tile list, window = 16 + 2 *
    border) into the block of the whole rectangle + border, as
    ImageBlock::put(const ImageBlock *) does (imageblock.h:103-107).
    block: (tile_h + 2b, tile_w + 2b, 5)."""
    tiles_x = (tile_w + 15) // 16
    stride = max(1, stride)
    offset = offset if stride > 1 else 0
    win = windows.shape[1]
    for v in range(windows.shape[0]):
        key = int(keys[v]) if keys is not None else offset + v * stride
        ty = key // tiles_x
        tx = (key % tiles_x + ty) % tiles_x
        x0, y0 = 16 * tx, 16 * ty   # window origin in block coordinates (the tile origin minus the border)
        h = min(win, block.shape[0] - y0)
        w = min(win, block.shape[1] - x0)
        block[y0:y0 + h, x0:x0 + w] += windows[v, :h, :w]
    return block


def balance_order(n_tiles: int) -> np.ndarray:
    """The deal keys 0..n_tiles-1 in the order balanced shares cut into
    contiguous runs: key k at position frac(k * golden ratio), so a run of any
    length is spread over the whole rectangle (as the stride deal is) and a
    share can grow or shrink by single tiles."""
    phi = (np.sqrt(5.0) - 1.0) / 2.0
    return np.argsort(np.modf(np.arange(n_tiles) * phi)[0], kind="stable").astype(np.int32)


def balance_cuts(counts, times, damping: float = 0.5):
    """New tile counts per share from the last step: share r took times[r]
    for counts[r] tiles, so it is given counts[r] / times[r] of the total
    (its measured rate), mixed with its old count by `damping`; the counts
    still sum to the total and every share keeps at least one tile."""
    counts = np.asarray(counts, dtype=np.float64)
    times = np.maximum(np.asarray(times, dtype=np.float64), 1e-9)
    total = int(round(counts.sum()))
    if total < len(counts):
        raise ValueError(f"balance_cuts: {total} tiles cannot give each of {len(counts)} shares one")
    target = counts / times
    target = target / target.sum() * total
    new = (1.0 - damping) * counts + damping * target
    out = np.maximum(1, np.floor(new)).astype(np.int64)
    # hand the rounding remainder to the fastest shares (largest fraction first)
    rest = total - int(out.sum())
    order = np.argsort(-(new - np.floor(new)))
    k = 0
    while rest != 0:
        i = order[k % len(order)]
        if rest > 0:
            out[i] += 1
            rest -= 1
        elif out[i] > 1:
            out[i] -= 1
            rest += 1
        k += 1
    return out


def develop(rgbaw: np.ndarray) -> np.ndarray:
    """hdrfilm develop: rgb = sum(w L) / sum(w) (fmtconv.cpp:962-974)."""
    rgbaw = np.ascontiguousarray(rgbaw, dtype=np.float32)
    h, w = rgbaw.shape[:2]
    out = np.zeros((h, w, 3), dtype=np.float32)
    host_lib().mtsh_develop(_ptr(rgbaw), w, h, _ptr(out))
    return out


def read_image(path: str) -> np.ndarray:
    """OpenEXR / PFM image as (h, w, 3) float32, rows top-down (the envmap loader's reader)."""
    lib = host_lib()
    w, h = C.c_int(), C.c_int()
    if lib.mtsh_read_image(path.encode(), C.byref(w), C.byref(h), None, 0) != 0:
        raise RuntimeError(_err(lib, "mtsh_last_error"))
    out = np.zeros((h.value, w.value, 3), np.float32)
    if lib.mtsh_read_image(path.encode(), C.byref(w), C.byref(h), _ptr(out), out.size) != 0:
        raise RuntimeError(_err(lib, "mtsh_last_error"))
    return out


def texture_image(path: str, gamma: float = 0.0) -> np.ndarray:
    """The bitmap texture's input as linear float RGB (h, w, 3), rows top-down
    (PNG / OpenEXR / PFM; gamma != 0 overrides the file's)."""
    lib = host_lib()
    w, h = C.c_int(), C.c_int()
    if lib.mtsh_texture_image(path.encode(), gamma, C.byref(w), C.byref(h), None, 0) != 0:
        raise RuntimeError(_err(lib, "mtsh_last_error"))
    out = np.zeros((h.value, w.value, 3), np.float32)
    if lib.mtsh_texture_image(path.encode(), gamma, C.byref(w), C.byref(h), _ptr(out), out.size) != 0:
        raise RuntimeError(_err(lib, "mtsh_last_error"))
    return out


MIP_NEAREST, MIP_BILINEAR, MIP_TRILINEAR, MIP_EWA = 0, 1, 2, 3
WRAP_CLAMP, WRAP_REPEAT, WRAP_MIRROR, WRAP_ZERO, WRAP_ONE = 0, 1, 2, 3, 4


def build_mipmap(rgb: np.ndarray, filter: int = MIP_EWA, wrap_u: int = WRAP_REPEAT, wrap_v: int = WRAP_REPEAT,
                 max_value: float = 1.0, max_anisotropy: float = 20.0):
    """TMIPMap of a linear RGB image (h, w, 3): (list of (h_l, w_l, 3) levels,
    header, level-0 average, level-0 maximum)."""
    lib = host_lib()
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[:2]
    hdr = MipMapHeader()
    n = C.c_size_t()
    avg = np.zeros(3, np.float32)
    mx = np.zeros(3, np.float32)
    args = (_ptr(rgb), w, h, filter, wrap_u, wrap_v, max_value, max_anisotropy, C.byref(hdr))
    if lib.mtsh_build_mipmap(*args, None, 0, C.byref(n), None, None) != 0:
        raise RuntimeError(_err(lib, "mtsh_last_error"))
    tex = np.zeros(n.value, np.float32)
    if lib.mtsh_build_mipmap(*args, _ptr(tex), tex.size, C.byref(n), _ptr(avg), _ptr(mx)) != 0:
        raise RuntimeError(_err(lib, "mtsh_last_error"))
    levels = []
    for l in range(hdr.levels):
        lw, lh, off = hdr.level_w[l], hdr.level_h[l], hdr.level_offset[l]
        levels.append(tex[off:off + lw * lh * 3].reshape(lh, lw, 3))
    return levels, hdr, avg, mx


def write_pfm(path: str, rgb: np.ndarray) -> None:
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    if host_lib().mtsh_write_pfm(path.encode(), rgb.shape[1], rgb.shape[0], _ptr(rgb)) != 0:
        raise RuntimeError(_err(host_lib(), "mtsh_last_error"))


class GPUScene:
    """A scene resident in HBM on one device (mtsg_scene_create)."""

    def __init__(self, scene: Scene, device: int = 0):
        lib = device_lib()
        h = C.c_void_p()
        rc = lib.mtsg_scene_create(scene.desc, device, C.byref(h))
        if rc != MTSG_OK:
            raise RuntimeError(f"mtsg_scene_create failed ({rc}): " + _err(lib, "mtsg_last_error"))
        self._h = h
        self.scene = scene
        self.device = device

    def _check(self, rc, what):
        if rc != MTSG_OK:
            raise RuntimeError(f"{what} failed ({rc}): " + _err(device_lib(), "mtsg_last_error"))

    def render(self, params: RenderParams, border: int) -> np.ndarray:
        out = np.zeros((params.tile_h + 2 * border, params.tile_w + 2 * border, 5), dtype=np.float32)
        self._check(device_lib().mtsg_render(self._h, C.byref(params), _ptr(out)), "mtsg_render")
        return out

    def render_samples(self, params: RenderParams) -> np.ndarray:
        """Per-sample radiance (tile_h, tile_w, spp, 4) -- debug/parity entry point."""
        out = np.zeros((params.tile_h, params.tile_w, params.spp, 4), dtype=np.float32)
        self._check(device_lib().mtsg_render_samples(self._h, C.byref(params), _ptr(out)), "mtsg_render_samples")
        return out

    def set_flags(self, flags: int) -> None:
        self._check(device_lib().mtsg_set_flags(self._h, flags), "mtsg_set_flags")

    def set_batch_paths(self, n: int) -> None:
        self._check(device_lib().mtsg_set_batch_paths(self._h, n), "mtsg_set_batch_paths")

    def set_test_knobs(self, stack_cap: int = 0, restart_guard: int = -1, restart_limit: int = -1,
                       limit_shadow_only: bool = False, no_instance_prefilter: bool = False) -> None:
        """TEST ONLY (mtsg_set_test_knobs): shrink the traversal stacks / move
        the kd-restart guard; the defaults restore the production limits."""
        k = TestKnobs(stack_cap, restart_guard, restart_limit, int(limit_shadow_only), int(no_instance_prefilter))
        self._check(device_lib().mtsg_set_test_knobs(self._h, C.byref(k)), "mtsg_set_test_knobs")

    def set_finish_paths(self, n: int) -> None:
        """Tail-mode threshold (paths; 0: off), see mtsg_set_finish_paths."""
        self._check(device_lib().mtsg_set_finish_paths(self._h, n), "mtsg_set_finish_paths")

    def set_option(self, key: int, value: int) -> None:
        """An execution option (MTSG_OPT_*, mtsg_set_option): scheduling only, never pixels."""
        self._check(device_lib().mtsg_set_option(self._h, key, value), "mtsg_set_option")

    def stats(self) -> Stats:
        s = Stats()
        self._check(device_lib().mtsg_get_stats(self._h, C.byref(s)), "mtsg_get_stats")
        return s

    def trace_closest(self, rays: np.ndarray):
        rays = np.ascontiguousarray(rays, dtype=np.float32)
        n = rays.shape[0]
        t = np.empty(n, np.float32); u = np.empty(n, np.float32); v = np.empty(n, np.float32)
        prim = np.empty(n, np.uint32)
        self._check(device_lib().mtsg_trace_closest(self._h, n, _ptr(rays), _ptr(t), _ptr(u), _ptr(v), _ptr(prim)),
                    "mtsg_trace_closest")
        return t, u, v, prim

    def env_eval(self, dirs: np.ndarray, rx: np.ndarray | None = None, ry: np.ndarray | None = None) -> np.ndarray:
        """Environment radiance along world directions (debug entry point)."""
        dirs = np.ascontiguousarray(dirs, dtype=np.float32)
        out = np.empty((dirs.shape[0], 3), np.float32)
        px = py = None
        if rx is not None:
            rx = np.ascontiguousarray(rx, dtype=np.float32)
            ry = np.ascontiguousarray(ry, dtype=np.float32)
            px, py = _ptr(rx), _ptr(ry)
        self._check(device_lib().mtsg_env_eval(self._h, dirs.shape[0], _ptr(dirs), px, py, _ptr(out)), "mtsg_env_eval")
        return out

    def tex_eval(self, tex: int, uv: np.ndarray, duv: np.ndarray | None = None) -> np.ndarray:
        """BitmapTexture::eval of texture `tex` at uv (n, 2), filtered with the
        uv partials duv (n, 4) when given (debug entry point)."""
        uv = np.ascontiguousarray(uv, dtype=np.float32)
        out = np.empty((uv.shape[0], 3), np.float32)
        pd = None
        if duv is not None:
            duv = np.ascontiguousarray(duv, dtype=np.float32)
            pd = _ptr(duv)
        self._check(device_lib().mtsg_tex_eval(self._h, tex, uv.shape[0], _ptr(uv), pd, _ptr(out)), "mtsg_tex_eval")
        return out

    def om_query(self, dirs: np.ndarray, o1: np.ndarray, o2: np.ndarray):
        """myPath2_OM visibility (debug entry point): (map ids, visible flags)."""
        dirs, o1, o2 = (np.ascontiguousarray(a, dtype=np.float32) for a in (dirs, o1, o2))
        n = dirs.shape[0]
        ids = np.empty(n, np.int32)
        vis = np.empty(n, np.int32)
        self._check(device_lib().mtsg_om_query(self._h, n, _ptr(dirs), _ptr(o1), _ptr(o2), _ptr(ids), _ptr(vis)),
                    "mtsg_om_query")
        return ids, vis

    def sampler_draws(self, params: RenderParams, x: int, y: int, s: int, kinds) -> np.ndarray:
        """The scene sampler's next1D (kind 1) / next2D (kind 2) draws of one
        sample, flattened (debug entry point)."""
        kinds = np.ascontiguousarray(kinds, dtype=np.int32)
        out = np.empty(int(np.where(kinds == 2, 2, 1).sum()), np.float32)
        self._check(device_lib().mtsg_sampler_draws(self._h, C.byref(params), x, y, s, kinds.size, _ptr(kinds), _ptr(out)),
                    "mtsg_sampler_draws")
        return out

    def trace_shadow(self, rays: np.ndarray) -> np.ndarray:
        rays = np.ascontiguousarray(rays, dtype=np.float32)
        occ = np.empty(rays.shape[0], np.uint8)
        self._check(device_lib().mtsg_trace_shadow(self._h, rays.shape[0], _ptr(rays), _ptr(occ)), "mtsg_trace_shadow")
        return occ

    # device-resident film for the benchmark
    def alloc(self, nbytes: int) -> C.c_void_p:
        p = C.c_void_p()
        self._check(device_lib().mtsg_device_alloc(self._h, nbytes, C.byref(p)), "mtsg_device_alloc")
        self._check(device_lib().mtsg_device_memset(self._h, p, nbytes), "mtsg_device_memset")
        return p

    def free(self, p: C.c_void_p) -> None:
        device_lib().mtsg_device_free(self._h, p)

    def render_device(self, params: RenderParams, film: C.c_void_p) -> None:
        self._check(device_lib().mtsg_render_device(self._h, C.byref(params), film), "mtsg_render_device")

    def tile_windows(self, params: RenderParams):
        """(ntiles, window) of params' per-tile ImageBlocks (mtsg_tile_windows)."""
        n, w = C.c_uint32(0), C.c_int32(0)
        self._check(device_lib().mtsg_tile_windows(self._h, C.byref(params), C.byref(n), C.byref(w)),
                    "mtsg_tile_windows")
        return n.value, w.value

    def set_tile_list(self, keys=None) -> None:
        """Render exactly these deal keys, in this order (mtsg_set_tile_list);
        None or empty: back to tile_stride / tile_offset."""
        if keys is None or len(keys) == 0:
            self._check(device_lib().mtsg_set_tile_list(self._h, None, 0), "mtsg_set_tile_list")
            return
        k = np.ascontiguousarray(keys, dtype=np.int32)
        self._check(device_lib().mtsg_set_tile_list(self._h, _ptr(k), len(k)), "mtsg_set_tile_list")

    def render_device_tiles(self, params: RenderParams, windows: C.c_void_p) -> None:
        self._check(device_lib().mtsg_render_device_tiles(self._h, C.byref(params), windows),
                    "mtsg_render_device_tiles")

    def download(self, film: C.c_void_p, shape) -> np.ndarray:
        out = np.zeros(shape, dtype=np.float32)
        self._check(device_lib().mtsg_device_to_host(self._h, _ptr(out), film, out.nbytes), "mtsg_device_to_host")
        return out

    def cancel(self) -> None:
        device_lib().mtsg_cancel(self._h)

    def set_tile_callback(self, fn) -> None:
        """fn(key, x, y, w, h) per completed tile (mtsg_set_tile_callback); None removes it."""
        self._tile_cb = TILE_FN(lambda _u, key, x, y, w, h: fn(key, x, y, w, h)) if fn else TILE_FN()
        self._check(device_lib().mtsg_set_tile_callback(self._h, self._tile_cb, None), "mtsg_set_tile_callback")

    def close(self):
        if getattr(self, "_h", None):
            device_lib().mtsg_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


class PathJob:
    """The `path` integrator's preprocess() / render() / cancel() over N GPUs
    (include/mtsg_path.h; SamplingIntegrator::render, integrator.cpp:99-133)."""

    def __init__(self, scene: Scene, n_gpus: int = 0):
        lib = path_lib()
        h = C.c_void_p()
        rc = lib.mtsh_path_job_create(C.c_void_p(scene._h), n_gpus, C.byref(h))
        if rc != MTSG_OK:
            raise RuntimeError(f"mtsh_path_job_create failed ({rc}): " + _err(lib, "mtsh_path_last_error"))
        self._h = h
        self.scene = scene
        self.gpus = lib.mtsh_path_job_gpus(h)

    def render(self, params: RenderParams, border: int) -> tuple[int, np.ndarray, float]:
        """Returns (error code, ImageBlock of the rectangle + border, seconds)."""
        out = np.zeros((params.tile_h + 2 * border, params.tile_w + 2 * border, 5), dtype=np.float32)
        secs = C.c_double(0.0)
        rc = path_lib().mtsh_path_job_render(self._h, C.byref(params), _ptr(out), C.byref(secs))
        return rc, out, secs.value

    def set_balance(self, on: bool) -> None:
        """Share balancing between renders of the same tile set (mtsh_path_job_set_balance)."""
        if path_lib().mtsh_path_job_set_balance(self._h, int(bool(on))) != MTSG_OK:
            raise RuntimeError(self.last_error())

    def shares(self):
        """(tiles, seconds) per GPU of the last render (mtsh_path_job_shares)."""
        t = np.zeros(self.gpus, np.int32)
        s = np.zeros(self.gpus, np.float64)
        if path_lib().mtsh_path_job_shares(self._h, _ptr(t), _ptr(s)) != MTSG_OK:
            raise RuntimeError(self.last_error())
        return t, s

    def last_error(self) -> str:
        return _err(path_lib(), "mtsh_path_last_error")

    def cancel(self) -> None:
        path_lib().mtsh_path_job_cancel(self._h)

    def set_tile_callback(self, fn) -> None:
        """fn(gpu, x, y, w, h) per completed tile (mtsh_path_job_set_tile_callback); None removes it."""
        self._tile_cb = TILE_FN(lambda _u, gpu, x, y, w, h: fn(gpu, x, y, w, h)) if fn else TILE_FN()
        if path_lib().mtsh_path_job_set_tile_callback(self._h, self._tile_cb, None) != MTSG_OK:
            raise RuntimeError(self.last_error())

    def close(self):
        if getattr(self, "_h", None):
            path_lib().mtsh_path_job_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


MTSG_ERR_CANCELLED = -4
MTSG_ERR_TRAVERSAL = -6
