"""The in-memory scene builder (mtsh_scene_begin / _add_* / _finish,
include/mtsh.h): the route a Mitsuba-side `path` plugin takes from the scene
Mitsuba already holds -- each object's plugin name and substituted Properties
(ConfigurableObject::getProperties, cobject.h:77) and each TriMesh's arrays
(trimesh.h:127-153) -- instead of re-reading the XML file.

tests/scene_walker.py plays Mitsuba: it parses the XML as SceneHandler does
(scenehandler.cpp:461-625), composes the transforms with Transform's own
arithmetic and hands Properties and PLY arrays to the builder.  The device
descriptor must then be byte-identical to the XML route's
(mtsh_scene_digest), and a `-D` that changes a BSDF or emitter parameter
must reach the descriptor and the render -- which the previous re-parse of
the scene file lost."""
import os

import numpy as np
import pytest

import scene_walker as W
from conftest import SCENES

SMALL = {"width": 64, "height": 48, "spp": 4}


def differing(a, b):
    return sorted(k for k in set(a) | set(b) if a.get(k) != b.get(k))


@pytest.mark.parametrize("xml,instancing,meshes", [
    ("cbox.xml", "flatten", "arrays"),
    ("env_glass.xml", "flatten", "arrays"),
    ("env_glass.xml", "flatten", "world"),
    ("env_glass.xml", "flatten", "plugin"),
    ("bunny15.xml", "flatten", "arrays"),
    ("bunny15.xml", "two-level", "world"),
    ("cbox_textured.xml", "flatten", "arrays"),
    ("cbox_materials.xml", "flatten", "arrays"),
    ("cbox_roughplastic.xml", "flatten", "plugin"),
    ("cbox_inst.xml", "two-level", "arrays"),
])
def test_builder_descriptor_is_byte_identical_to_the_xml_route(xml, instancing, meshes):
    import mtsg
    path = os.path.join(SCENES, xml)
    by_xml = mtsg.Scene(path, SMALL, instancing=instancing).digest()
    walker = W.Walker(path, SMALL, instancing=instancing, meshes=meshes)
    by_builder = walker.walk().digest()
    assert differing(by_xml, by_builder) == []
    # the array route really went through mtsh_scene_add_mesh
    if meshes != "plugin" and "bunny" in open(path).read():
        assert "mesh" in walker.log


OVERRIDE_XML = """<?xml version="1.0"?>
<scene version="0.5.0">
  <default name="wallR" value="0.63"/>
  <default name="lightR" value="17"/>
  <default name="alpha" value="0.2"/>
  <integrator type="path"><integer name="maxDepth" value="4"/></integrator>
  <sensor type="perspective">
    <float name="fov" value="39.3"/>
    <transform name="toWorld"><lookat origin="0, 0, 3.9" target="0, 0, 0" up="0, 1, 0"/></transform>
    <sampler type="independent"><integer name="sampleCount" value="4"/></sampler>
    <film type="hdrfilm"><integer name="width" value="24"/><integer name="height" value="20"/>
      <rfilter type="gaussian"/></film>
  </sensor>
  <bsdf type="diffuse" id="white"><rgb name="reflectance" value="0.725, 0.71, 0.68"/></bsdf>
  <bsdf type="diffuse" id="red"><rgb name="reflectance" value="$wallR, 0.065, 0.05"/></bsdf>
  <bsdf type="roughconductor" id="metal">
    <string name="distribution" value="beckmann"/><float name="alpha" value="$alpha"/></bsdf>
  <shape type="rectangle"><transform name="toWorld"><rotate x="1" angle="-90"/><translate y="-1"/></transform>
    <ref id="white"/></shape>
  <shape type="rectangle"><transform name="toWorld"><translate z="-1"/></transform><ref id="white"/></shape>
  <shape type="rectangle"><transform name="toWorld"><rotate y="1" angle="90"/><translate x="-1"/></transform>
    <ref id="red"/></shape>
  <shape type="ply"><string name="filename" value="{bunny}"/>
    <transform name="toWorld"><translate y="-0.0329874"/><scale value="6"/><translate y="-0.8"/></transform>
    <ref id="metal"/></shape>
  <shape type="rectangle">
    <transform name="toWorld"><scale x="0.23" y="0.19" z="1"/><rotate x="1" angle="90"/><translate y="0.99"/></transform>
    <emitter type="area"><rgb name="radiance" value="$lightR, 12, 4"/></emitter></shape>
</scene>
"""


@pytest.fixture(scope="module")
def override_xml(tmp_path_factory):
    d = tmp_path_factory.mktemp("builder")
    p = d / "cbox_params.xml"
    p.write_text(OVERRIDE_XML.replace("{bunny}", os.path.join(SCENES, "bunny.ply")))
    return str(p)


@pytest.mark.parametrize("defines,changed", [
    ({"wallR": "0.2"}, ["bsdfs"]),                       # a diffuse reflectance
    ({"alpha": "0.45"}, ["bsdfs"]),                      # the microfacet roughness
    ({"lightR": "40"}, ["emitters"]),                    # the area light's radiance
])
def test_bsdf_and_emitter_defines_reach_the_scene_and_the_render(override_xml, defines, changed):
    """`mitsuba -D wallR=0.2 scene.xml`: Mitsuba substitutes the value while
    parsing (mitsuba.cpp:168-174, scenehandler.cpp:211) and the plugin sees
    it only in the objects' Properties.  The builder route carries it; the
    old route (re-reading the file without the map) rendered the default."""
    import mtsg
    from oracle import pyoracle as O
    mitsuba_side = W.build(override_xml, defines)             # what the plugin hands over
    reference = mtsg.Scene(override_xml, defines)             # the scene the -D describes
    stale = mtsg.Scene(override_xml, {})                      # the previous plugin's re-parse
    assert differing(mitsuba_side.digest(), reference.digest()) == []
    assert differing(stale.digest(), reference.digest()) == changed
    params = mitsuba_side.params()
    img_b, _ = O.render(mitsuba_side.desc, params, mitsuba_side.border, rng=O.RNG_COUNTER)
    img_r, _ = O.render(reference.desc, reference.params(), reference.border, rng=O.RNG_COUNTER)
    img_s, _ = O.render(stale.desc, stale.params(), stale.border, rng=O.RNG_COUNTER)
    np.testing.assert_array_equal(img_b, img_r)
    assert np.abs(mtsg.develop(img_b) - mtsg.develop(img_s)).mean() > 1e-3 * mtsg.develop(img_s).mean()


def test_in_memory_property_change_without_a_define(override_xml):
    """A plugin may also hold objects changed programmatically (no XML
    parameter exists for them): the values it passes are the ones rendered."""
    import mtsg
    from oracle import pyoracle as O
    changed = W.build(override_xml, {}, override_props={("white", "reflectance"): ("spectrum", [0.3, 0.3, 0.9])})
    base = W.build(override_xml, {})
    assert differing(changed.digest(), base.digest()) == ["bsdfs"]
    img_c, _ = O.render(changed.desc, changed.params(), changed.border, rng=O.RNG_COUNTER)
    img_b, _ = O.render(base.desc, base.params(), base.border, rng=O.RNG_COUNTER)
    rgb_c, rgb_b = mtsg.develop(img_c), mtsg.develop(img_b)
    # a bluer floor and back wall
    assert rgb_c[..., 2].mean() > rgb_b[..., 2].mean() and rgb_c[..., 0].mean() < rgb_b[..., 0].mean()


def test_builder_overrides_and_render_params(override_xml):
    import mtsg
    ov = mtsg.SceneOverrides()
    ov.mask = mtsg.MTSH_OVERRIDE_FILM_SIZE | mtsg.MTSH_OVERRIDE_SAMPLE_COUNT
    ov.film_width, ov.film_height, ov.sample_count = 40, 30, 7
    s = W.build(override_xml, {}, overrides=ov)
    p = s.params()
    assert (p.tile_w, p.tile_h, p.spp, p.max_depth) == (40, 30, 7, 4)
    assert (s.info.film_w, s.info.film_h) == (40, 30)


def minimal_builder():
    import mtsg
    b = mtsg.SceneBuilder(SCENES)
    b.integrator("path", [("maxDepth", "integer", 3)])
    b.sensor("perspective", [("fov", "float", 45.0)])
    b.film("hdrfilm", [("width", "integer", 8), ("height", "integer", 8)], "box", [])
    b.sampler("independent", [("sampleCount", "integer", 2)])
    return b


def test_builder_from_bare_arrays():
    """A mesh given only as arrays (no file): positions, triangles, no
    normals (computed as TriMesh::computeNormals does), a default BSDF."""
    import mtsg
    b = minimal_builder()
    tri = np.array([[-1, -1, -2], [1, -1, -2], [0, 1, -2]], np.float32)
    b.mesh(tri, [[0, 1, 2]], name="tri")
    e = b.emitter("area", [("radiance", "spectrum", [2.0, 2.0, 2.0])])
    b.shape("rectangle", [("toWorld", "transform", np.diag([0.2, 0.2, 1, 1]).astype(np.float32))], emitter=e)
    s = b.finish()
    assert (s.info.n_triangles, s.info.n_rects, s.info.n_emitters, s.info.n_bsdfs) == (1, 1, 1, 2)
    d = s.digest()
    assert d["vtx_nrm"][0] == 36


def test_builder_errors_are_reported_and_leave_it_usable():
    import mtsg
    b = minimal_builder()
    with pytest.raises(RuntimeError, match="outside this build's scope"):
        b.bsdf("hk", [])
    with pytest.raises(RuntimeError, match="Microfacet model"):
        b.bsdf("roughconductor", [("alpha", "float", 0.1), ("alphaU", "float", 0.2)])
    with pytest.raises(RuntimeError, match="specified multiple times"):
        b.bsdf("diffuse", [("reflectance", "spectrum", [0.5] * 3), ("reflectance", "spectrum", [0.2] * 3)])
    with pytest.raises(RuntimeError, match="texture"):
        b.emitter("area", [("radiance", "texture", 0)])
    with pytest.raises(RuntimeError, match="invalid BSDF id"):
        b.shape("cube", [], bsdf=7)
    with pytest.raises(RuntimeError, match="nested BSDFs"):
        b.bsdf("diffuse", [], nested=[0])
    e = b.emitter("area", [])
    b.shape("cube", [], emitter=e)
    with pytest.raises(RuntimeError, match="only be attached to one shape"):
        b.shape("cube", [], emitter=e)
    with pytest.raises(RuntimeError, match="invalid shape group"):
        b.instance(3, [])
    g = b.group("g")
    with pytest.raises(RuntimeError, match="emitters inside shapegroups"):
        b.shape("cube", [], emitter=b.emitter("area", []), group=g)
    # an unattached area light fails the finish, as the XML route does
    with pytest.raises(RuntimeError, match="area emitter without a parent shape"):
        b.finish()
    b2 = minimal_builder()
    d = b2.bsdf("diffuse", [("reflectance", "spectrum", [0.2, 0.4, 0.6])])
    b2.shape("cube", [], bsdf=d)
    with pytest.raises(RuntimeError, match="no emitters"):   # scene.cpp:382-397's sun/sky fallback
        b2.finish()
    b3 = minimal_builder()
    b3.shape("cube", [], bsdf=b3.bsdf("diffuse", [("reflectance", "spectrum", [0.2, 0.4, 0.6])]))
    b3.shape("rectangle", [], emitter=b3.emitter("area", []))
    assert b3.finish().info.n_triangles == 12


def test_builder_needs_a_sensor():
    import mtsg
    b = mtsg.SceneBuilder(SCENES)
    b.shape("cube", [])
    with pytest.raises(RuntimeError, match="no <sensor>"):
        b.finish()


def _ply_with_normals(path, n=6):
    """A small binary PLY grid with per-vertex normals (a bumped sheet)."""
    import numpy as np
    xs = np.linspace(-0.5, 0.5, n, dtype=np.float32)
    X, Y = np.meshgrid(xs, xs)
    Z = (0.1 * np.sin(3 * X) * np.cos(2 * Y)).astype(np.float32)
    pos = np.stack([X.ravel(), Y.ravel(), Z.ravel()], 1).astype(np.float32)
    nrm = np.stack([-0.3 * np.cos(3 * X.ravel()), 0.2 * np.sin(2 * Y.ravel()), np.ones(n * n)], 1)
    nrm = (nrm / np.linalg.norm(nrm, axis=1, keepdims=True)).astype(np.float32)
    faces = []
    for j in range(n - 1):
        for i in range(n - 1):
            a, b, c, d = j * n + i, j * n + i + 1, (j + 1) * n + i + 1, (j + 1) * n + i
            faces += [(a, b, c), (a, c, d)]
    head = ("ply\nformat binary_little_endian 1.0\nelement vertex %d\nproperty float x\nproperty float y\n"
            "property float z\nproperty float nx\nproperty float ny\nproperty float nz\nelement face %d\n"
            "property list uchar int vertex_indices\nend_header\n" % (n * n, len(faces))).encode()
    body = np.concatenate([pos, nrm], 1).astype("<f4").tobytes()
    for f in faces:
        body += np.uint8(3).tobytes() + np.array(f, "<i4").tobytes()
    open(path, "wb").write(head + body)


FLIP_XML = """<?xml version="1.0"?>
<scene version="0.5.0">
  <integer name="kdStopPrims" value="2"/>
  <float name="kdEmptySpaceBonus" value="0.8"/>
  <integrator type="path"><integer name="maxDepth" value="3"/></integrator>
  <sensor type="perspective">
    <transform name="toWorld"><lookat origin="0, 0, 3" target="0, 0, 0" up="0, 1, 0"/></transform>
    <sampler type="independent"><integer name="sampleCount" value="2"/></sampler>
    <film type="hdrfilm"><integer name="width" value="16"/><integer name="height" value="16"/></film>
  </sensor>
  <shape type="ply"><string name="filename" value="sheet.ply"/><boolean name="flipNormals" value="true"/>
    <transform name="toWorld"><rotate y="1" angle="20"/><translate x="0.3"/></transform>
    <bsdf type="diffuse"/></shape>
  <shape type="ply"><string name="filename" value="sheet.ply"/><boolean name="faceNormals" value="true"/>
    <boolean name="flipNormals" value="true"/>
    <transform name="toWorld"><translate x="-0.4" z="-0.5"/></transform><bsdf type="diffuse"/></shape>
  <shape type="ply"><string name="filename" value="sheet.ply"/><transform name="toWorld"><translate y="0.6"/></transform>
    <bsdf type="diffuse"/></shape>
  <shape type="rectangle"><transform name="toWorld"><translate z="2"/></transform>
    <emitter type="area"><rgb name="radiance" value="5"/></emitter></shape>
</scene>
"""


@pytest.mark.parametrize("meshes", ["arrays", "configured"])
def test_flipped_meshes_and_scene_kd_properties_through_the_builder(tmp_path, meshes):
    """mtsh_mesh's flip contract (include/mtsh.h): flip_normals is the normal
    pass's m_flipNormals, applied by the builder to the arrays it is given.
    Loader arrays with the flag ("arrays") and arrays that already carry the
    flip, negated normals / a swapped face-normal winding, without it
    ("configured", a configured TriMesh) both give the XML route's descriptor
    byte for byte; the <scene> kd properties travel as the Scene's Properties."""
    import mtsg
    _ply_with_normals(str(tmp_path / "sheet.ply"))
    xml = tmp_path / "flip.xml"
    xml.write_text(FLIP_XML)
    by_xml = mtsg.Scene(str(xml)).digest()
    walker = W.Walker(str(xml), {}, meshes=meshes)
    by_builder = walker.walk().digest()
    assert "mesh" in walker.log and "scene_props" in walker.log
    assert differing(by_xml, by_builder) == []
    # without the scene's kd properties the tree differs (they reached the build)
    plain = tmp_path / "plain.xml"
    plain.write_text(FLIP_XML.replace('<integer name="kdStopPrims" value="2"/>', "")
                     .replace('<float name="kdEmptySpaceBonus" value="0.8"/>', ""))
    assert differing(by_xml, mtsg.Scene(str(plain)).digest()) != []
