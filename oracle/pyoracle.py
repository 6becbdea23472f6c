"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the CPU oracle (oracle.h).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  The product path (my-mitsuba_amd/mtsg.py, libmtsg.so) never loads it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
RNG_COUNTER = 0
RNG_SFMT = 1


class OracleStats(C.Structure):
    _fields_ = [
        ("seconds", C.c_double), ("samples", C.c_uint64),
        ("rays_closest", C.c_uint64), ("rays_shadow", C.c_uint64),
        ("nodes_visited", C.c_uint64), ("leaf_refs", C.c_uint64), ("tri_tests", C.c_uint64),
        ("path_vertices", C.c_uint64), ("threads", C.c_int),
    ]


_libs: dict = {}


def lib(fast: bool = False) -> C.CDLL:
    name = "liboracle_fast.so" if fast else "liboracle.so"
    if name not in _libs:
        path = os.path.join(HERE, name)
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make oracle`")
        L = C.CDLL(path)
        L.oracle_sfmt_new.restype = C.c_void_p
        L.oracle_sfmt_new.argtypes = [C.c_uint64]
        L.oracle_sfmt_clone.restype = C.c_void_p
        L.oracle_sfmt_clone.argtypes = [C.c_void_p]
        L.oracle_sfmt_next_ulong.restype = C.c_uint64
        L.oracle_sfmt_next_ulong.argtypes = [C.c_void_p]
        L.oracle_sfmt_next_float.restype = C.c_float
        L.oracle_sfmt_next_float.argtypes = [C.c_void_p]
        L.oracle_sfmt_free.argtypes = [C.c_void_p]
        L.oracle_counter_float.restype = C.c_float
        L.oracle_counter_float.argtypes = [C.c_uint32, C.c_uint64, C.c_uint32]
        L.oracle_trace_closest.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_int]
        L.oracle_trace_shadow.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int]
        L.oracle_trace_closest_brute.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_render.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.POINTER(OracleStats)]
        L.oracle_pixel_samples.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.oracle_bsdf_sample.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_bsdf_eval.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_last_error.restype = C.c_char_p
        _libs[name] = L
    return _libs[name]


def _p(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


def sfmt_sequence(seed: int, n: int) -> list[int]:
    L = lib()
    r = L.oracle_sfmt_new(seed)
    out = [L.oracle_sfmt_next_ulong(r) for _ in range(n)]
    L.oracle_sfmt_free(r)
    return out


def trace_closest(desc, rays: np.ndarray, threads: int = 0):
    rays = np.ascontiguousarray(rays, dtype=np.float32)
    n = rays.shape[0]
    t = np.empty(n, np.float32); u = np.empty(n, np.float32); v = np.empty(n, np.float32)
    prim = np.empty(n, np.uint32)
    lib().oracle_trace_closest(desc, n, _p(rays), _p(t), _p(u), _p(v), _p(prim), threads)
    return t, u, v, prim


def trace_shadow(desc, rays: np.ndarray, threads: int = 0) -> np.ndarray:
    rays = np.ascontiguousarray(rays, dtype=np.float32)
    occ = np.empty(rays.shape[0], np.uint8)
    lib().oracle_trace_shadow(desc, rays.shape[0], _p(rays), _p(occ), threads)
    return occ


def trace_closest_brute(desc, rays: np.ndarray):
    rays = np.ascontiguousarray(rays, dtype=np.float32)
    n = rays.shape[0]
    t = np.empty(n, np.float32); prim = np.empty(n, np.uint32)
    lib().oracle_trace_closest_brute(desc, n, _p(rays), _p(t), _p(prim))
    return t, prim


def render(desc, params, border: int, rng: int = RNG_COUNTER, threads: int = 0, fast: bool = False,
           count: bool = False):
    """Returns (rgbaw block of tile+border, OracleStats)."""
    out = np.zeros((params.tile_h + 2 * border, params.tile_w + 2 * border, 5), np.float32)
    st = OracleStats()
    st.threads = -1 if count else 0
    rc = lib(fast).oracle_render(desc, C.byref(params), rng, threads, _p(out), C.byref(st))
    if rc != 0:
        raise RuntimeError("oracle_render: " + lib(fast).oracle_last_error().decode())
    return out, st


def pixel_samples(desc, params, x: int, y: int) -> np.ndarray:
    out = np.zeros((params.spp, 3), np.float32)
    if lib().oracle_pixel_samples(desc, C.byref(params), x, y, _p(out)) != 0:
        raise RuntimeError("oracle_pixel_samples: " + lib().oracle_last_error().decode())
    return out


def sampler_draws(desc, params, x: int, y: int, s: int, kinds) -> np.ndarray:
    """The scene sampler's next1D (1) / next2D (2) draws of one sample, flattened."""
    L = lib()
    L.oracle_sampler_draws.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_uint32, C.c_uint32,
                                       C.c_void_p, C.c_void_p]
    kinds = np.ascontiguousarray(kinds, dtype=np.int32)
    out = np.empty(int(np.where(kinds == 2, 2, 1).sum()), np.float32)
    if L.oracle_sampler_draws(desc, C.byref(params), x, y, s, kinds.size, _p(kinds), _p(out)) != 0:
        raise RuntimeError("oracle_sampler_draws: " + L.oracle_last_error().decode())
    return out


def tex_eval(desc, tex: int, uv: np.ndarray, duv: np.ndarray | None = None) -> np.ndarray:
    """BitmapTexture::eval of texture `tex` at uv (n, 2), filtered with the uv
    partials duv (n, 4) when given (oracle_tex_eval_n)."""
    L = lib()
    uv = np.ascontiguousarray(uv, dtype=np.float32)
    out = np.empty((uv.shape[0], 3), np.float32)
    pd = None
    if duv is not None:
        duv = np.ascontiguousarray(duv, dtype=np.float32)
        pd = _p(duv)
    L.oracle_tex_eval_n.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
    if L.oracle_tex_eval_n(desc, tex, uv.shape[0], _p(uv), pd, _p(out)) != 0:
        raise RuntimeError(L.oracle_last_error().decode())
    return out


def om_query(desc, dirs: np.ndarray, o1: np.ndarray, o2: np.ndarray):
    """myPath2_OM's nearestOMindex + Visible (oracle_om_query_n): (ids, vis)."""
    L = lib()
    dirs, o1, o2 = (np.ascontiguousarray(a, dtype=np.float32) for a in (dirs, o1, o2))
    n = dirs.shape[0]
    ids = np.empty(n, np.int32)
    vis = np.empty(n, np.int32)
    L.oracle_om_query_n.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    if L.oracle_om_query_n(desc, n, _p(dirs), _p(o1), _p(o2), _p(ids), _p(vis)) != 0:
        raise RuntimeError(L.oracle_last_error().decode())
    return ids, vis
