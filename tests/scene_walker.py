"""A Mitsuba-side stand-in for the builder tests: what a `path` plugin sees in
memory after Mitsuba parsed a scene, handed to the in-memory builder
(mtsh_scene_begin / _add_* / _finish, include/mtsh.h).

Mitsuba's SceneHandler (src/librender/scenehandler.cpp:461-625) substitutes
`$name` parameters, turns each element's values into a Properties object
and composes <transform> children into a float Transform with its inverse
(include/mitsuba/core/transform.h).  This module restates that in Python,
independently of the host library's XML loader, so the tests can compare the
builder route with the XML route byte for byte:

* values are parsed as Mitsuba parses them (floats to float32, rgb to an RGB
  Spectrum);
* transforms are composed with the arithmetic of Transform (float32 vectors,
  matrices in double rounded to float, inverses by Gauss-Jordan in double;
  transform.cpp:99-123,191-214), the inverse carried alongside;
* meshes go through the array route (mtsh_scene_add_mesh) as the TriMesh
  arrays a PLY file holds (ply.cpp:73-220: quads split into (0,1,2),
  (3,0,2)), or through the plugin route (mtsh_scene_add_shape) with the
  shape's Properties.

Test infrastructure only.
"""
from __future__ import annotations

import math
import os
import re
import xml.etree.ElementTree as ET

import numpy as np

import mtsg

F = np.float32


# ---- Transform arithmetic (hmath.h mirrors include/mitsuba/core/transform.h) ----
def _invert4(a):
    m = [[a[i][j] if j < 4 else (1.0 if j - 4 == i else 0.0) for j in range(8)] for i in range(4)]
    for c in range(4):
        piv = c
        for r in range(c + 1, 4):
            if abs(m[r][c]) > abs(m[piv][c]):
                piv = r
        if abs(m[piv][c]) < 1e-300:
            return [[0.0] * 4 for _ in range(4)]
        if piv != c:
            m[c], m[piv] = m[piv], m[c]
        d = m[c][c]
        m[c] = [x / d for x in m[c]]
        for r in range(4):
            if r != c:
                f = m[r][c]
                if f != 0:
                    m[r] = [m[r][j] - f * m[c][j] for j in range(8)]
    return [[m[i][j + 4] for j in range(4)] for i in range(4)]


class Xf:
    """A float Transform and its inverse."""

    def __init__(self, m=None, inv=None):
        eye = [[F(1.0) if i == j else F(0.0) for j in range(4)] for i in range(4)]
        self.m = m or eye
        self.inv = inv or [row[:] for row in eye]

    @staticmethod
    def from_double(a):
        b = _invert4(a)
        return Xf([[F(a[i][j]) for j in range(4)] for i in range(4)], [[F(b[i][j]) for j in range(4)] for i in range(4)])

    def __mul__(self, o):
        r = Xf()
        for i in range(4):
            for j in range(4):
                s = si = 0.0
                for k in range(4):
                    s += float(self.m[i][k]) * float(o.m[k][j])
                    si += float(o.inv[i][k]) * float(self.inv[k][j])
                r.m[i][j], r.inv[i][j] = F(s), F(si)
        return r

    def arrays(self):
        return (np.array(self.m, np.float32), np.array(self.inv, np.float32))


def _dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def _length(a):
    return F(np.sqrt(_dot(a, a)))


def _normalize(a):
    r = F(1.0) / _length(a)
    return [a[0] * r, a[1] * r, a[2] * r]


def _cross(a, b):
    return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]


def translate(v):
    return Xf.from_double([[1, 0, 0, float(v[0])], [0, 1, 0, float(v[1])], [0, 0, 1, float(v[2])], [0, 0, 0, 1]])


def scale(v):
    return Xf.from_double([[float(v[0]), 0, 0, 0], [0, float(v[1]), 0, 0], [0, 0, float(v[2]), 0], [0, 0, 0, 1]])


def rotate(axis, angle):
    ax = _normalize(axis)
    a = float(angle) * math.pi / 180.0
    s, c = math.sin(a), math.cos(a)
    x, y, z = float(ax[0]), float(ax[1]), float(ax[2])
    return Xf.from_double([
        [x * x + (1 - x * x) * c, x * y * (1 - c) - z * s, x * z * (1 - c) + y * s, 0],
        [x * y * (1 - c) + z * s, y * y + (1 - y * y) * c, y * z * (1 - c) - x * s, 0],
        [x * z * (1 - c) - y * s, y * z * (1 - c) + x * s, z * z + (1 - z * z) * c, 0],
        [0, 0, 0, 1]])


def look_at(p, t, up):
    d = _normalize([t[0] - p[0], t[1] - p[1], t[2] - p[2]])
    left = _normalize(_cross(up, d))
    new_up = _cross(d, left)
    return Xf.from_double([[float(left[0]), float(new_up[0]), float(d[0]), float(p[0])],
                           [float(left[1]), float(new_up[1]), float(d[1]), float(p[1])],
                           [float(left[2]), float(new_up[2]), float(d[2]), float(p[2])],
                           [0, 0, 0, 1]])


def transform_points(m, p):
    """Transform::operator()(Point) in float32: x = m00 px + m01 py + m02 pz
    + m03 (left to right), divided by w unless w == 1."""
    m = np.asarray(m, np.float32)
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    r = [m[i, 0] * x + m[i, 1] * y + m[i, 2] * z + m[i, 3] for i in range(4)]
    out = np.stack(r[:3], 1).astype(np.float32)
    w = r[3]
    if not np.all(w == 1):
        inv = (np.float32(1) / w).astype(np.float32)
        out = np.where((w == 1)[:, None], out, out * inv[:, None]).astype(np.float32)
    return out


# ---- PLY (ply.cpp:73-220) ----
_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2", "ushort": "u2",
              "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4", "float": "f4",
              "float32": "f4", "double": "f8", "float64": "f8"}


def read_ply(path):
    """(positions, normals or None, uv or None, triangles) of a triangle / quad PLY."""
    data = open(path, "rb").read()
    end = data.index(b"end_header")
    body = data.index(b"\n", end) + 1
    elems, fmt = [], None
    for line in data[:end].decode().splitlines():
        tok = line.split()
        if not tok:
            continue
        if tok[0] == "format":
            fmt = tok[1]
        elif tok[0] == "element":
            elems.append((tok[1], int(tok[2]), []))
        elif tok[0] == "property":
            elems[-1][2].append(tuple(tok[1:]))
    if fmt != "binary_little_endian":
        raise NotImplementedError(fmt)
    off = body
    pos = nrm = uv = tris = None
    for name, count, props in elems:
        if name == "vertex":
            dt = np.dtype([(p[1], "<" + _PLY_TYPES[p[0]]) for p in props])
            v = np.frombuffer(data, dt, count, off)
            off += dt.itemsize * count
            pos = np.stack([v["x"], v["y"], v["z"]], 1).astype(np.float32)
            if "nx" in dt.names:
                nrm = np.stack([v["nx"], v["ny"], v["nz"]], 1).astype(np.float32)
            if "u" in dt.names:
                uv = np.stack([v["u"], v["v"]], 1).astype(np.float32)
        elif name == "face":
            (_, ct, it, _pname), = props
            ct, it = np.dtype("<" + _PLY_TYPES[ct]), np.dtype("<" + _PLY_TYPES[it])
            out = []
            for _ in range(count):
                c = int(np.frombuffer(data, ct, 1, off)[0])
                off += ct.itemsize
                ids = np.frombuffer(data, it, c, off).astype(np.uint32)
                off += it.itemsize * c
                out.append(ids[[0, 1, 2]])
                if c == 4:
                    out.append(ids[[3, 0, 2]])
            tris = np.array(out, np.uint32)
    return pos, nrm, uv, tris


# ---- SceneHandler ----
class Walker:
    """Walks a Mitsuba XML scene as SceneHandler would and drives a
    SceneBuilder with the Properties and TriMesh arrays Mitsuba would hold.
    meshes: "arrays" (mtsh_scene_add_mesh with the PLY's arrays) or "plugin"
    (mtsh_scene_add_shape with the ply shape's Properties)."""

    def __init__(self, path, defines=None, instancing="flatten", meshes="arrays", override_props=None):
        self.path = path
        self.dir = os.path.dirname(os.path.abspath(path))
        self.defines = {k: str(v) for k, v in (defines or {}).items()}
        self.meshes = meshes
        # {(element id or "#n" in document order, property name): (kind, value)}:
        # the values a plugin would see changed in memory
        self.override_props = dict(override_props or {})
        self.b = mtsg.SceneBuilder(self.dir, instancing=instancing)
        self.bsdf_ids, self.tex_ids, self.groups = {}, {}, {}
        self.log = []   # the builder calls, in order

    def sub(self, s):
        def rep(m):
            if m.group(1) not in self.defines:
                raise KeyError(f"Unresolved parameter \"${m.group(1)}\"")
            return self.defines[m.group(1)]
        return re.sub(r"\$([A-Za-z0-9_]+)", rep, s)

    def attr(self, e, k, d=None):
        v = e.get(k)
        return d if v is None else self.sub(v)

    def floats(self, s):
        return [F(x) for x in re.split(r"[,\s]+", self.sub(s).strip()) if x]

    def transform(self, e):
        t = Xf()
        for c in e:
            if c.tag == "translate":
                op = translate([F(self.attr(c, k, "0")) for k in "xyz"])
            elif c.tag == "rotate":
                op = rotate([F(self.attr(c, k, "0")) for k in "xyz"], F(self.attr(c, "angle")))
            elif c.tag == "scale":
                if c.get("value") is not None:
                    op = scale([F(self.attr(c, "value"))] * 3)
                else:
                    op = scale([F(self.attr(c, k, "1")) for k in "xyz"])
            elif c.tag in ("lookat", "lookAt"):
                op = look_at(self.floats(c.get("origin")), self.floats(c.get("target")), self.floats(c.get("up")))
            elif c.tag == "matrix":
                v = [float(x) for x in self.floats(c.get("value"))]
                op = Xf.from_double([v[4 * i:4 * i + 4] for i in range(4)])
            else:
                raise ValueError(c.tag)
            t = op * t
        return t

    def props(self, e, key):
        out, nested = [], []
        for c in e:
            name = self.attr(c, "name")
            if c.tag == "float":
                out.append((name, "float", F(self.attr(c, "value"))))
            elif c.tag == "integer":
                out.append((name, "integer", int(self.attr(c, "value"))))
            elif c.tag == "boolean":
                out.append((name, "boolean", self.attr(c, "value").lower() == "true"))
            elif c.tag == "string":
                out.append((name, "string", self.attr(c, "value")))
            elif c.tag in ("rgb", "spectrum"):
                v = self.floats(c.get("value"))
                out.append((name, "spectrum", v * 3 if len(v) == 1 else v))
            elif c.tag in ("point", "vector"):
                out.append((name, c.tag, [F(self.attr(c, k, "0")) for k in "xyz"]))
            elif c.tag == "transform":
                out.append((name, "transform", self.transform(c).arrays()))
            else:
                nested.append(c)
        for (k, pname), (kind, value) in self.override_props.items():
            if k == key:
                out = [p for p in out if p[0] != pname] + [(pname, kind, value)]
        return out, nested

    def call(self, what, *args, **kw):
        self.log.append(what)
        return getattr(self.b, what)(*args, **kw)

    def texture(self, e):
        p, _ = self.props(e, e.get("id"))
        t = self.call("texture", self.attr(e, "type"), p)
        if e.get("id"):
            self.tex_ids[e.get("id")] = t
        return t

    def bsdf(self, e):
        p, nested = self.props(e, e.get("id"))
        kids = []
        for c in nested:
            name = self.attr(c, "name")
            if c.tag == "texture":
                p.append((name, "texture", self.texture(c)))
            elif c.tag == "ref" and c.get("id") in self.tex_ids:
                p.append((name, "texture", self.tex_ids[c.get("id")]))
            elif c.tag == "bsdf":
                kids.append(self.bsdf(c))
            elif c.tag == "ref":
                kids.append(self.bsdf_ids[c.get("id")])
        i = self.call("bsdf", self.attr(e, "type"), p, kids)
        if e.get("id"):
            self.bsdf_ids[e.get("id")] = i
        return i

    def shape(self, e, group=-1):
        typ = self.attr(e, "type")
        if typ == "shapegroup":
            g = self.call("group", e.get("id"))
            for c in e:
                self.shape(c, g)
            self.groups[e.get("id")] = g
            return
        self.nshape = getattr(self, "nshape", 0) + 1
        p, nested = self.props(e, e.get("id") or f"#{self.nshape}")
        bsdf = emitter = inst = -1
        for c in nested:
            if c.tag == "bsdf":
                bsdf = self.bsdf(c)
            elif c.tag == "emitter":
                ep, _ = self.props(c, None)
                emitter = self.call("emitter", self.attr(c, "type"), ep)
            elif c.tag == "ref":
                rid = c.get("id")
                if rid in self.bsdf_ids:
                    bsdf = self.bsdf_ids[rid]
                else:
                    inst = self.groups[rid]
        pd = {n: v for n, _k, v in p}
        if typ == "instance":
            self.call("instance", inst, [pp for pp in p if pp[0] == "toWorld"])
            return
        if typ == "ply" and self.meshes in ("arrays", "world", "configured"):
            pos, nrm, uv, tris = read_ply(os.path.join(self.dir, pd["filename"]))
            m, inv = pd["toWorld"] if "toWorld" in pd else Xf().arrays()
            face, flip = bool(pd.get("faceNormals", False)), bool(pd.get("flipNormals", False))
            if self.meshes == "world" and nrm is None:
                # the positions as TriMesh holds them after the PLY loader
                # applied toWorld (Transform::operator()(Point), transform.h)
                pos, m, inv = transform_points(m, pos), None, None
            if self.meshes == "configured" and flip and (face or nrm is not None):
                # the flip as a configured TriMesh carries it (TriMesh::computeNormals,
                # trimesh.cpp:608-681, already ran): normals negated, or the
                # winding of a face-normal mesh swapped; the flag is not passed again
                # (negation commutes with the linear normal transform and with
                # normalisation, so the descriptor must not change)
                if face:
                    tris = tris[:, [1, 0, 2]].copy()
                else:
                    nrm = (-nrm).astype(np.float32)
                flip = False
            self.call("mesh", pos, tris, normals=nrm, texcoords=uv, to_world=m, to_world_inv=inv,
                      face_normals=face, flip_normals=flip,
                      bsdf=bsdf, emitter=emitter, group=group, name=pd["filename"])
            return
        self.call("shape", typ, p, bsdf, emitter, group)

    def sensor(self, e):
        p, nested = self.props(e, "sensor")
        self.call("sensor", self.attr(e, "type"), p)
        for c in nested:
            if c.tag == "film":
                fp, fn = self.props(c, "film")
                rf = [r for r in fn if r.tag == "rfilter"]
                rp = self.props(rf[0], "rfilter")[0] if rf else None
                self.call("film", self.attr(c, "type"), fp, self.attr(rf[0], "type") if rf else None, rp)
            elif c.tag == "sampler":
                self.call("sampler", self.attr(c, "type"), self.props(c, "sampler")[0])

    def walk(self, overrides=None) -> "mtsg.Scene":
        root = ET.parse(self.path).getroot()
        for e in root:
            if e.tag == "default":
                self.defines.setdefault(e.get("name"), e.get("value"))
            elif e.tag == "integrator":
                self.call("integrator", self.attr(e, "type"), self.props(e, "integrator")[0])
            elif e.tag in ("sensor", "camera"):
                self.sensor(e)
            elif e.tag == "bsdf":
                self.bsdf(e)
            elif e.tag == "texture":
                self.texture(e)
            elif e.tag == "shape":
                self.shape(e)
            elif e.tag == "emitter":
                self.call("emitter", self.attr(e, "type"), self.props(e, e.get("id"))[0])
        # the Scene's own Properties (scene->getProperties(): its kd* values)
        sp, _ = self.props([e for e in root if e.tag in ("float", "integer", "boolean", "string")], "scene")
        if sp:
            self.call("scene_props", sp)
        return self.b.finish(overrides, label=f"builder:{os.path.basename(self.path)}")


def build(path, defines=None, instancing="flatten", meshes="arrays", override_props=None, overrides=None):
    return Walker(path, defines, instancing, meshes, override_props).walk(overrides)
