// Scene::finalize -- flatten the loaded scene into the mtsg_scene_desc SoA
// arrays that cross the C-ABI.  Restates the preprocessing
// Mitsuba performs before rendering:
//   TriMesh::computeUVTangents      src/librender/trimesh.cpp:683-743
//   TriMesh::prepareSamplingTable   src/librender/trimesh.cpp:388-402
//   Scene emitter PDF               src/librender/scene.cpp:399-404
//   DiscreteDistribution::normalize include/mitsuba/core/pmf.h:101-116
//   ShapeKDTree::build (TriAccel)   src/librender/skdtree.cpp:68-110
//   TriAccel::load                  include/mitsuba/render/triaccel.h:61-94
//   PerspectiveCamera::configure    src/sensors/perspective.cpp:126-176
//   ReconstructionFilter::configure src/libcore/rfilter.cpp:37-57
#include <cstring>
#include <functional>

#include "scene.h"

namespace mtsh {

// Triangle::getClippedAABB (src/libcore/triangle.cpp; Sutherland-Hodgman
// against the 6 box planes), used by the kd build's perfect splits
AABB clipTriangle(const V3 &a, const V3 &b, const V3 &c, const AABB &box) {
    double poly[16][3], tmp[16][3];
    int n = 3;
    const V3 *v[3] = {&a, &b, &c};
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) poly[i][k] = (*v[i])[k];
    for (int axis = 0; axis < 3; ++axis) {
        for (int side = 0; side < 2; ++side) {
            // sutherlandHodgman (triangle.cpp:70-73) gives up on fewer than
            // three vertices: the triangle only touches the box there
            if (n < 3) return AABB();
            double plane = side == 0 ? box.mn[axis] : box.mx[axis];
            int m = 0;
            for (int i = 0; i < n; ++i) {
                const double *cur = poly[i], *nxt = poly[(i + 1) % n];
                bool curIn = side == 0 ? cur[axis] >= plane : cur[axis] <= plane;
                bool nxtIn = side == 0 ? nxt[axis] >= plane : nxt[axis] <= plane;
                if (curIn) { for (int k = 0; k < 3; ++k) tmp[m][k] = cur[k]; ++m; }
                if (curIn != nxtIn && m < 15) {
                    double t = (plane - cur[axis]) / (nxt[axis] - cur[axis]);
                    for (int k = 0; k < 3; ++k) tmp[m][k] = cur[k] + (nxt[k] - cur[k]) * t;
                    tmp[m][axis] = plane;
                    ++m;
                }
            }
            n = m;
            for (int i = 0; i < n; ++i)
                for (int k = 0; k < 3; ++k) poly[i][k] = tmp[i][k];
        }
    }
    if (n == 0) return AABB();
    // rounded outwards (math::castflt_down / castflt_up, triangle.cpp:134-141):
    // a clipped bound rounded to nearest can land on the far side of a later
    // split plane and drop the triangle from a child it overlaps
    AABB r;
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            float lo = (float)poly[i][k], hi = lo;
            if ((double)lo > poly[i][k]) lo = std::nextafter(lo, -INFINITY);
            if ((double)hi < poly[i][k]) hi = std::nextafter(hi, INFINITY);
            r.mn[k] = std::min(r.mn[k], lo);
            r.mx[k] = std::max(r.mx[k], hi);
        }
    r.clip(box);
    return r;
}

namespace {

struct ScenePrims : PrimSource {
    const Scene &s;
    const std::vector<uint8_t> &grouped;   // triangle belongs to a shape group (two-level)
    ScenePrims(const Scene &sc, const std::vector<uint8_t> &g) : s(sc), grouped(g) {}
    size_t count() const override { return s.triIdx.size() / 3 + s.rectDesc.size() + s.instanceDesc.size(); }
    V3 vtx(uint32_t i) const { return V3(s.vtxPos[3 * i], s.vtxPos[3 * i + 1], s.vtxPos[3 * i + 2]); }
    AABB bounds(size_t i) const override {
        AABB b;
        size_t nt = s.triIdx.size() / 3, nr = s.rectDesc.size();
        if (i < nt) {
            if (s.triaccel[i].k == 3 || grouped[i]) return AABB();   // degenerate, or in a group's own tree
            for (int k = 0; k < 3; ++k) b.expand(vtx(s.triIdx[3 * i + k]));
        } else if (i < nt + nr) {
            const mtsg_rect &r = s.rectDesc[i - nt];
            for (int cx = -1; cx <= 1; cx += 2)
                for (int cy = -1; cy <= 1; cy += 2) {
                    const float *m = r.to_world;
                    V3 p(m[0] * cx + m[1] * cy + m[3], m[4] * cx + m[5] * cy + m[7], m[8] * cx + m[9] * cy + m[11]);
                    b.expand(p);
                }
        } else {
            // Instance::getAABB (instance.cpp:78-96): the group tree's AABB
            // corners through the instance transform
            const InstanceDef &in = s.instances[i - nt - nr];
            const AABB &ga = s.groupTrees[in.group].aabb;
            if (!ga.valid()) return AABB();
            for (int c = 0; c < 8; ++c)
                b.expand(in.toWorld.point(V3((c & 1) ? ga.mx.x : ga.mn.x, (c & 2) ? ga.mx.y : ga.mn.y,
                                             (c & 4) ? ga.mx.z : ga.mn.z)));
        }
        return b;
    }
    AABB clippedBounds(size_t i, const AABB &box) const override {
        size_t nt = s.triIdx.size() / 3;
        if (i < nt) return clipTriangle(vtx(s.triIdx[3 * i]), vtx(s.triIdx[3 * i + 1]), vtx(s.triIdx[3 * i + 2]), box);
        AABB b = bounds(i);
        b.clip(box);
        return b;
    }
};

// the triangles of one shape group, in group space (ShapeGroup's ShapeKDTree)
struct GroupPrims : PrimSource {
    const Scene &s;
    const std::vector<uint32_t> &tris;   // global triangle indices
    GroupPrims(const Scene &sc, const std::vector<uint32_t> &t) : s(sc), tris(t) {}
    size_t count() const override { return tris.size(); }
    V3 vtx(uint32_t i) const { return V3(s.vtxPos[3 * i], s.vtxPos[3 * i + 1], s.vtxPos[3 * i + 2]); }
    AABB bounds(size_t i) const override {
        AABB b;
        const uint32_t t = tris[i];
        if (s.triaccel[t].k == 3) return AABB();
        for (int k = 0; k < 3; ++k) b.expand(vtx(s.triIdx[3 * t + k]));
        return b;
    }
    AABB clippedBounds(size_t i, const AABB &box) const override {
        const uint32_t t = tris[i];
        return clipTriangle(vtx(s.triIdx[3 * t]), vtx(s.triIdx[3 * t + 1]), vtx(s.triIdx[3 * t + 2]), box);
    }
};

// TriAccel::load (triaccel.h:61-94); returns false for degenerate triangles
bool loadTriAccel(mtsg_triaccel &t, const V3 &A, const V3 &B, const V3 &C) {
    static const int waldModulo[4] = {1, 2, 0, 1};
    V3 b = C - A, c = B - A, N = cross(c, b);
    int k = 0;
    for (int j = 0; j < 3; j++)
        if (std::abs(N[j]) > std::abs(N[k])) k = j;
    int u = waldModulo[k], v = waldModulo[k + 1];
    const float n_k = N[k], denom = b[u] * c[v] - b[v] * c[u];
    if (denom == 0) { t.k = 3; return false; }
    t.k = (uint32_t)k;
    t.n_u = N[u] / n_k;
    t.n_v = N[v] / n_k;
    t.n_d = dot(A, N) / n_k;
    t.b_nu = b[u] / denom;
    t.b_nv = -b[v] / denom;
    t.a_u = A[u];
    t.a_v = A[v];
    t.c_nu = c[v] / denom;
    t.c_nv = -c[u] / denom;
    return true;
}

void setRow34(float *dst, const Transform &t, bool inverse) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) dst[4 * r + c] = inverse ? t.inv[r][c] : t.m[r][c];
}

}  // namespace

// The top-level tree's primitive boxes (6 floats each; empty for primitives
// it leaves out): the input of the device build (mtsg_kd_build)
void Scene::primBounds(std::vector<float> &out) const {
    ScenePrims src(*this, triGrouped);
    out.assign(src.count() * 6, 0.0f);
    for (size_t i = 0; i < src.count(); ++i) {
        const AABB b = src.bounds(i);
        float *o = &out[6 * i];
        if (!b.valid()) { o[0] = 1; o[3] = -1; continue; }
        for (int k = 0; k < 3; ++k) { o[k] = b.mn[k]; o[3 + k] = b.mx[k]; }
    }
}

// Replace the top-level tree (a device-built one) and point the descriptor at it
void Scene::setTree(const mtsg_kdnode *nodes, uint32_t nNodes, const uint32_t *indices, uint32_t nIndices, const float *aabbMin,
                    const float *aabbMax, uint32_t maxDepth) {
    tree.nodes.assign(nodes, nodes + nNodes);
    tree.indices.assign(indices, indices + nIndices);
    for (int k = 0; k < 3; ++k) { tree.aabb.mn[k] = aabbMin[k]; tree.aabb.mx[k] = aabbMax[k]; }
    tree.maxDepth = maxDepth;
    desc.n_nodes = nNodes;
    desc.nodes = tree.nodes.data();
    desc.n_indices = nIndices;
    desc.indices = tree.indices.data();
    for (int k = 0; k < 3; ++k) { desc.aabb_min[k] = aabbMin[k]; desc.aabb_max[k] = aabbMax[k]; }
    desc.max_depth = maxDepth;
}

void Scene::finalize() {
    // ---------------- geometry ----------------
    vtxPos.clear(); vtxNrm.clear(); triIdx.clear(); triDpdu.clear(); triUv.clear(); triDpdv.clear();
    const bool texData = !textures.empty();
    shapeDesc.clear(); rectDesc.clear();
    std::vector<uint32_t> meshTriBegin(meshes.size());
    for (size_t si = 0; si < shapes.size(); ++si) {
        const ShapeRef &sr = shapes[si];
        mtsg_shape sd{};
        sd.type = sr.type;
        sd.emitter = -1;
        if (sr.type == MTSG_SHAPE_MESH) {
            Mesh &m = meshes[sr.index];
            if (m.idx.empty()) throw std::runtime_error("Encountered an empty triangle mesh!");
            uint32_t vbase = (uint32_t)(vtxPos.size() / 3);
            uint32_t tbase = (uint32_t)(triIdx.size() / 3);
            meshTriBegin[sr.index] = tbase;
            for (size_t v = 0; v < m.p.size(); ++v) {
                vtxPos.insert(vtxPos.end(), {m.p[v].x, m.p[v].y, m.p[v].z});
                V3 n = m.n.empty() ? V3(0.0f) : m.n[v];
                vtxNrm.insert(vtxNrm.end(), {n.x, n.y, n.z});
            }
            bool hasUV = !m.uv.empty();
            for (size_t t = 0; t < m.idx.size(); t += 3) {
                uint32_t i0 = m.idx[t], i1 = m.idx[t + 1], i2 = m.idx[t + 2];
                triIdx.insert(triIdx.end(), {vbase + i0, vbase + i1, vbase + i2});
                V3 dP1 = m.p[i1] - m.p[i0], dP2 = m.p[i2] - m.p[i0];
                V3 dpdu = dP1, dpdv = dP2;   // no UV tangents: side1, side2 (skdtree.h:373-380)
                if (hasUV) {
                    // computeUVTangents (trimesh.cpp:701-735); degenerate
                    // triangles keep the zeroed tangents
                    V3 n = cross(dP1, dP2);
                    float len = length(n);
                    if (len == 0) {
                        dpdu = dpdv = V3(0.0f);
                    } else {
                        float du1 = m.uv[2 * i1] - m.uv[2 * i0], dv1 = m.uv[2 * i1 + 1] - m.uv[2 * i0 + 1];
                        float du2 = m.uv[2 * i2] - m.uv[2 * i0], dv2 = m.uv[2 * i2 + 1] - m.uv[2 * i0 + 1];
                        float det = du1 * dv2 - dv1 * du2;
                        if (det == 0) {
                            coordinateSystem(n / len, dpdu, dpdv);
                        } else {
                            float invDet = 1.0f / det;
                            dpdu = (dP1 * dv2 - dP2 * dv1) * invDet;
                            dpdv = (dP1 * (-du2) + dP2 * du1) * invDet;
                        }
                    }
                }
                if (texData) {
                    if (hasUV) {
                        for (uint32_t vi : {i0, i1, i2}) triUv.insert(triUv.end(), {m.uv[2 * vi], m.uv[2 * vi + 1]});
                    } else {
                        triUv.insert(triUv.end(), {0.0f, 0.0f, 1.0f, 0.0f, 0.0f, 1.0f});   // -> Point2(b.y, b.z)
                    }
                    triDpdv.insert(triDpdv.end(), {dpdv.x, dpdv.y, dpdv.z});
                }
                triDpdu.insert(triDpdu.end(), {dpdu.x, dpdu.y, dpdu.z});
            }
            sd.bsdf = m.bsdf;
            sd.face_normals = m.faceNormals ? 1 : 0;
            sd.tri_begin = tbase;
            sd.tri_count = (uint32_t)(m.idx.size() / 3);
            sd.emitter = m.emitter;
        } else if (sr.type == MTSG_SHAPE_INSTANCE) {
            sd.bsdf = -1;
            sd.emitter = -1;
            sd.instance = (uint32_t)sr.index;
        } else {
            Rect &r = rects[sr.index];
            // rectangle.cpp:78-94 configure()
            mtsg_rect rd{};
            setRow34(rd.to_world, r.toWorld, false);
            setRow34(rd.to_object, r.toWorld, true);
            V3 dpdu = r.toWorld.vector(V3(2, 0, 0)), dpdv = r.toWorld.vector(V3(0, 2, 0));
            V3 nrm = normalize(r.toWorld.normal(V3(0, 0, 1)));
            V3 fs = normalize(dpdu), ft = normalize(dpdv);
            if (std::abs(dot(fs, ft)) > 1e-4f) throw std::runtime_error("Error: 'toWorld' transformation contains shear!");
            for (int k = 0; k < 3; ++k) {
                rd.frame_s[k] = fs[k]; rd.frame_t[k] = ft[k]; rd.frame_n[k] = nrm[k];
                rd.dpdu[k] = dpdu[k]; rd.dpdv[k] = dpdv[k];
            }
            rd.inv_area = 1.0f / (length(dpdu) * length(dpdv));
            rd.shape_index = (uint32_t)si;
            sd.rect = (uint32_t)rectDesc.size();
            rectDesc.push_back(rd);
            sd.bsdf = r.bsdf;
            sd.emitter = r.emitter;
        }
        shapeDesc.push_back(sd);
    }
    size_t nTri = triIdx.size() / 3;

    // ---------------- BSDFs ----------------
    bsdfDesc.clear();
    for (auto &b : bsdfs) bsdfDesc.push_back(b.d);

    // ---------------- emitters ----------------
    emitterDesc.clear(); emitterCdf.clear(); emitterTriCdf.clear();
    if (emitters.empty()) throw std::runtime_error("scene has no emitters (the sun/sky fallback of scene.cpp:382-397 is outside this build's scope)");
    float wsum = 0;
    emitterCdf.push_back(0.0f);
    for (auto &e : emitters) {
        mtsg_emitter ed{};
        ed.type = e.type;
        ed.shape = e.shape;
        for (int k = 0; k < 3; ++k) ed.radiance[k] = e.radiance[k];
        if (e.type == MTSG_EMITTER_ENVMAP) {   // tables are built after the kd-tree (needs its AABB)
            emitterDesc.push_back(ed);
            wsum += e.samplingWeight;
            emitterCdf.push_back(wsum);
            continue;
        }
        const mtsg_shape &sd = shapeDesc[e.shape];
        if (sd.type == MTSG_SHAPE_MESH) {
            ed.cdf_offset = (uint32_t)emitterTriCdf.size();
            std::vector<float> cdf;
            cdf.reserve(sd.tri_count + 1);
            cdf.push_back(0.0f);
            for (uint32_t t = 0; t < sd.tri_count; ++t) {
                uint32_t g = sd.tri_begin + t;
                auto P = [&](int k) { uint32_t vi = triIdx[3 * g + k]; return V3(vtxPos[3 * vi], vtxPos[3 * vi + 1], vtxPos[3 * vi + 2]); };
                V3 p0 = P(0), p1 = P(1), p2 = P(2);
                float area = 0.5f * length(cross(p1 - p0, p2 - p0));   // Triangle::surfaceArea
                cdf.push_back(cdf.back() + area);
            }
            float sum = cdf.back();
            if (!(sum > 0)) throw std::runtime_error("area emitter on a mesh with zero surface area");
            float norm = 1.0f / sum;
            for (size_t i = 1; i < cdf.size(); ++i) cdf[i] *= norm;
            cdf.back() = 1.0f;
            ed.inv_area = 1.0f / sum;
            emitterTriCdf.insert(emitterTriCdf.end(), cdf.begin(), cdf.end());
        } else {
            ed.inv_area = rectDesc[sd.rect].inv_area;
        }
        emitterDesc.push_back(ed);
        wsum += e.samplingWeight;
        emitterCdf.push_back(wsum);
    }
    {
        float norm = 1.0f / wsum;
        for (size_t i = 1; i < emitterCdf.size(); ++i) emitterCdf[i] *= norm;
        emitterCdf.back() = 1.0f;
        for (size_t i = 0; i < emitters.size(); ++i) emitterDesc[i].pdf_discrete = emitters[i].samplingWeight * norm;
    }

    // ---------------- TriAccel + kd-tree ----------------
    const size_t nInst = instances.size();
    triaccel.assign(nTri + rectDesc.size() + nInst, mtsg_triaccel{});
    triGrouped.assign(nTri, 0);
    std::vector<uint8_t> &grouped = triGrouped;
    std::vector<std::vector<uint32_t>> groupTris(groups.size());
    for (size_t si = 0; si < shapeDesc.size(); ++si) {
        const mtsg_shape &sd = shapeDesc[si];
        if (sd.type == MTSG_SHAPE_MESH) {
            const int grp = meshes[shapes[si].index].group;
            for (uint32_t t = 0; t < sd.tri_count; ++t) {
                uint32_t g = sd.tri_begin + t;
                auto P = [&](int k) { uint32_t vi = triIdx[3 * g + k]; return V3(vtxPos[3 * vi], vtxPos[3 * vi + 1], vtxPos[3 * vi + 2]); };
                mtsg_triaccel &ta = triaccel[g];
                loadTriAccel(ta, P(0), P(1), P(2));
                ta.shape_index = (uint32_t)si;
                ta.prim_index = g;
                if (grp >= 0) { grouped[g] = 1; groupTris[grp].push_back(g); }
            }
        } else if (sd.type == MTSG_SHAPE_RECT) {
            mtsg_triaccel &ta = triaccel[nTri + sd.rect];
            memset(&ta, 0, sizeof(ta));
            ta.k = MTSG_TRIACCEL_SHAPE;
            ta.shape_index = (uint32_t)si;
            ta.prim_index = sd.rect;
        } else {
            mtsg_triaccel &ta = triaccel[nTri + rectDesc.size() + sd.instance];
            memset(&ta, 0, sizeof(ta));
            ta.k = MTSG_TRIACCEL_SHAPE;
            ta.shape_index = (uint32_t)si;
            ta.prim_index = sd.instance;
        }
    }
    // one kd-tree per shape group, in group space (ShapeGroup::configure,
    // shapegroup.cpp:94-101); leaf references index `triaccel`
    groupTrees.assign(groups.size(), KDTree());
    groupDesc.clear(); groupNodes.clear(); groupIndices.clear(); instanceDesc.clear();
    for (size_t g = 0; g < groups.size(); ++g) {
        if (groupTris[g].empty()) throw std::runtime_error("shapegroup \"" + groups[g].id + "\" holds no triangles");
        GroupPrims gp(*this, groupTris[g]);
        buildKDTree(gp, groupKd, groupTrees[g]);
        const KDTree &T = groupTrees[g];
        mtsg_group gd{};
        gd.node_offset = (uint32_t)groupNodes.size();
        gd.n_nodes = (uint32_t)T.nodes.size();
        gd.index_offset = (uint32_t)groupIndices.size();
        gd.n_indices = (uint32_t)T.indices.size();
        for (int k = 0; k < 3; ++k) { gd.aabb_min[k] = T.aabb.mn[k]; gd.aabb_max[k] = T.aabb.mx[k]; }
        gd.max_depth = T.maxDepth;
        // leaf ranges stay relative to the group's own index block
        groupNodes.insert(groupNodes.end(), T.nodes.begin(), T.nodes.end());
        for (uint32_t i : T.indices) groupIndices.push_back(groupTris[g][i]);
        groupDesc.push_back(gd);
    }
    for (const InstanceDef &in : instances) {
        mtsg_instance id{};
        setRow34(id.to_world, in.toWorld, false);
        setRow34(id.to_local, in.toWorld, true);
        id.group = (uint32_t)in.group;
        instanceDesc.push_back(id);
    }
    for (size_t si = 0; si < shapeDesc.size(); ++si)
        if (shapeDesc[si].type == MTSG_SHAPE_INSTANCE) instanceDesc[shapeDesc[si].instance].shape_index = (uint32_t)si;
    ScenePrims src(*this, grouped);
    buildKDTree(src, kd, tree);

    // ---------------- sensor / film ----------------
    Film &f = film;
    // Film::Film's check (film.cpp:44-48); the crop window is the rectangle
    // the render params cover (mtsh_scene_render_params), the camera keeps the
    // full film's projection
    if (f.cropX < 0 || f.cropY < 0 || f.cropW <= 0 || f.cropH <= 0 || f.cropX + f.cropW > f.width ||
        f.cropY + f.cropH > f.height)
        throw std::runtime_error("Invalid crop window specification!");
    mtsg_camera &cam = camera;
    memset(&cam, 0, sizeof(cam));
    float aspect = (float)f.width / (float)f.height;
    float xfov;
    {
        float fov = sensor.fov;
        std::string axis = sensor.fovAxis;
        auto fromY = [&](float yfov) { return (float)(2 * std::atan(std::tan(0.5 * yfov * M_PI / 180.0) * aspect) * 180.0 / M_PI); };
        auto fromDiag = [&](float dfov) {
            double diagonal = 2 * std::tan(0.5 * dfov * M_PI / 180.0);
            double width = diagonal / std::sqrt(1.0 + 1.0 / (aspect * aspect));
            return (float)(2 * std::atan(width * 0.5) * 180.0 / M_PI);
        };
        if (fov < 0) {
            xfov = fromDiag((float)(2 * 180 / M_PI * std::atan(std::sqrt(36.0 * 36 + 24 * 24) / (2 * 50.0))));
        } else {
            if (axis == "smaller") axis = aspect > 1 ? "y" : "x";
            else if (axis == "larger") axis = aspect > 1 ? "x" : "y";
            if (axis == "x") xfov = fov;
            else if (axis == "y") xfov = fromY(fov);
            else if (axis == "diagonal") xfov = fromDiag(fov);
            else throw std::runtime_error("The 'fovAxis' parameter must be set to one of 'smaller', 'larger', 'diagonal', 'x', or 'y'!");
        }
        if (xfov <= 0 || xfov >= 180) throw std::runtime_error("The horizontal field of view must be in the interval (0, 180)!");
    }
    // perspective.cpp:147-152 (crop window is the full film)
    Transform cameraToSample =
        Transform::scale(V3(-0.5f, -0.5f * aspect, 1.0f)) *
        Transform::translate(V3(-1.0f, -1.0f / aspect, 0.0f)) *
        Transform::perspective(xfov, sensor.nearClip, sensor.farClip);
    Transform sampleToCamera = cameraToSample.inverse();
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) cam.sample_to_camera[4 * r + c] = sampleToCamera.m[r][c];
    setRow34(cam.camera_to_world, sensor.toWorld, false);
    float invResX = 1.0f / (float)f.width, invResY = 1.0f / (float)f.height;
    V3 o = sampleToCamera.point(V3(0.0f));
    V3 dx = sampleToCamera.point(V3(invResX, 0.0f, 0.0f)) - o;
    V3 dy = sampleToCamera.point(V3(0.0f, invResY, 0.0f)) - o;
    for (int k = 0; k < 3; ++k) { cam.dx[k] = dx[k]; cam.dy[k] = dy[k]; }
    cam.near_clip = sensor.nearClip;
    cam.far_clip = sensor.farClip;
    cam.inv_res_x = invResX;
    cam.inv_res_y = invResY;
    cam.film_w = f.width;
    cam.film_h = f.height;
    cam.crop_x = f.cropX; cam.crop_y = f.cropY; cam.crop_w = f.cropW; cam.crop_h = f.cropH;
    cam.has_alpha = f.hasAlpha ? 1 : 0;
    // myPath2_OM accumulates each pixel's running mean of its own samples
    // and hands the film a finished bitmap (myPath2_OM.cpp:229-281): a box of
    // exactly one pixel, no alpha
    const bool om = integrator.type == "myPath2_OM";
    if (om) cam.has_alpha = 0;

    // rfilter.cpp:37-57 with MTS_FILTER_RESOLUTION = 31
    const int RES = 31;
    float radius;
    std::function<float(float)> eval;
    if (f.filter == "gaussian" && !om) {
        float stddev = f.stddev;
        radius = 4 * stddev;
        eval = [stddev, radius](float x) {
            float alpha = -1.0f / (2.0f * stddev * stddev);
            return std::max(0.0f, (float)std::exp((double)(alpha * x * x)) - (float)std::exp((double)(alpha * radius * radius)));
        };
        cam.filter_type = MTSG_FILTER_GAUSSIAN;
    } else {
        radius = om ? 0.5f : f.boxRadius + 1e-5f;
        eval = [radius](float x) { return std::abs(x) <= radius ? 1.0f : 0.0f; };
        cam.filter_type = MTSG_FILTER_BOX;
    }
    float sum = 0.0f;
    for (int i = 0; i < RES; ++i) {
        float v = eval((radius * i) / RES);
        cam.filter_values[i] = v;
        sum += v;
    }
    cam.filter_values[RES] = 0.0f;
    cam.filter_scale = RES / radius;
    cam.border = (int)std::ceil(radius - 0.5f);
    sum *= 2 * radius / RES;
    float normalization = 1.0f / sum;
    for (int i = 0; i < RES; ++i) cam.filter_values[i] *= normalization;
    cam.filter_radius = radius;

    // ---------------- descriptor ----------------
    mtsg_scene_desc &d = desc;
    memset(&d, 0, sizeof(d));
    d.abi_version = MTSG_ABI_VERSION;
    d.n_vertices = (uint32_t)(vtxPos.size() / 3);
    d.vtx_pos = vtxPos.data();
    d.vtx_nrm = vtxNrm.data();
    d.n_triangles = (uint32_t)nTri;
    d.tri_idx = triIdx.data();
    d.tri_dpdu = triDpdu.data();
    d.n_textures = (uint32_t)textures.size();
    textureDesc.clear();
    for (auto &t : textures) textureDesc.push_back(t.d);
    d.textures = textureDesc.empty() ? nullptr : textureDesc.data();
    d.n_tex_texels = (uint32_t)texTexels.size();
    d.tex_texels = texTexels.empty() ? nullptr : texTexels.data();
    d.tri_uv = triUv.empty() ? nullptr : triUv.data();
    d.tri_dpdv = triDpdv.empty() ? nullptr : triDpdv.data();
    if (om) {
        // the fork's integrator draws from one sampler per core without
        // generate()/advance() (myPath2_OM.cpp:198-265): only the independent
        // sampler has a defined sequence there
        if (samplerType != "independent")
            throw std::runtime_error("myPath2_OM: only the independent sampler is supported by this build");
        buildOccupancyMaps(*this);
        d.om = &omDesc;
        d.om_bits = omBits.data();
    }
    d.n_rects = (uint32_t)rectDesc.size();
    d.rects = rectDesc.data();
    d.n_shapes = (uint32_t)shapeDesc.size();
    d.shapes = shapeDesc.data();
    d.n_bsdfs = (uint32_t)bsdfDesc.size();
    d.bsdfs = bsdfDesc.data();
    d.n_emitters = (uint32_t)emitterDesc.size();
    d.emitters = emitterDesc.data();
    d.emitter_cdf = emitterCdf.data();
    d.n_emitter_tri_cdf = (uint32_t)emitterTriCdf.size();
    d.emitter_tri_cdf = emitterTriCdf.data();
    d.n_nodes = (uint32_t)tree.nodes.size();
    d.nodes = tree.nodes.data();
    d.n_indices = (uint32_t)tree.indices.size();
    d.indices = tree.indices.data();
    d.n_prims = (uint32_t)triaccel.size();
    d.triaccel = triaccel.data();
    for (int k = 0; k < 3; ++k) { d.aabb_min[k] = tree.aabb.mn[k]; d.aabb_max[k] = tree.aabb.mx[k]; }
    d.max_depth = tree.maxDepth;
    d.n_instances = (uint32_t)instanceDesc.size();
    d.instances = instanceDesc.empty() ? nullptr : instanceDesc.data();
    d.n_groups = (uint32_t)groupDesc.size();
    d.groups = groupDesc.empty() ? nullptr : groupDesc.data();
    d.n_group_nodes = (uint32_t)groupNodes.size();
    d.group_nodes = groupNodes.empty() ? nullptr : groupNodes.data();
    d.n_group_indices = (uint32_t)groupIndices.size();
    d.group_indices = groupIndices.empty() ? nullptr : groupIndices.data();
    d.camera = cam;
    // ---------------- sampler ----------------
    d.sampler = sampler;
    if (sampler.type == MTSG_SAMPLER_HALTON || sampler.type == MTSG_SAMPLER_HAMMERSLEY) {
        buildQmcTables(sampler.scramble, qmcPrimes, qmcOffsets, qmcPerm);
        d.qmc_primes = qmcPrimes.data();
        d.qmc_perm_offset = qmcOffsets.data();
        d.qmc_perm = qmcPerm.empty() ? nullptr : qmcPerm.data();
    }
    if (sampler.type == MTSG_SAMPLER_SOBOL) {
        sobolTables(d.sobol_matrices, d.sobol_vdc, d.sobol_vdc_rows, d.sobol_vdc_inv, d.sobol_vdc_inv_rows);
        d.sobol_scramble = sobolScramble(sobolScrambleProp);
    }
    // ---------------- environment emitter ----------------
    d.has_envmap = 0;
    for (size_t i = 0; i < emitters.size(); ++i) {
        if (emitters[i].type != MTSG_EMITTER_ENVMAP) continue;
        float aabbMin[3], aabbMax[3], camPos[3];
        for (int k = 0; k < 3; ++k) { aabbMin[k] = d.aabb_min[k]; aabbMax[k] = d.aabb_max[k]; }
        camPos[0] = cam.camera_to_world[3]; camPos[1] = cam.camera_to_world[7]; camPos[2] = cam.camera_to_world[11];
        buildEnvmap(emitters[i], aabbMin, aabbMax, camPos, envTexels, envCdfRows, envCdfCols, envRowWeights, d.envmap);
        d.envmap.emitter = (int)i;
        d.has_envmap = 1;
        d.n_env_texels = (uint32_t)envTexels.size();
        d.env_texels = envTexels.data();
        d.env_cdf_rows = envCdfRows.data();
        d.env_cdf_cols = envCdfCols.data();
        d.env_row_weights = envRowWeights.data();
    }
}

}  // namespace mtsh
