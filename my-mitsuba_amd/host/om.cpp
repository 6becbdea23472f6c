// Occupancy maps of the fork's `myPath2_OM` integrator (host side, shared by
// the GPU upload and the CPU oracle through mtsg_scene_desc):
//
//   scene AABB        myPath2OMIntegrator::preprocess (myPath2_OM.cpp:137-158):
//                     union of the TriMesh AABBs, a cube of half-size
//                     |max - min| / 2 * 1.001 around their centre
//   base map          OccupancyMap<256, 8>::setScene / setMesh / setTriangle
//                     (src/integrators/testOM/myOM.h:115-194): every
//                     triangle's vertices in grid coordinates, recursively
//                     split at its edge midpoints until the three cells are
//                     within an L1 distance of 4, every visited vertex cell set
//   rotated maps      generateROMA (myOM.h:534-567) for the 16 directions
//                     concentricMap((i + 0.5) / 4, (j + 0.5) / 4)
//                     (myOM.h:506-532): the base map resampled along each
//                     rotated column (Quaternion::fromDirectionPair((0,0,1),
//                     dir), include/mitsuba/core/quat.h:205-227, 301-327)
//
// The reference sets bits from several OpenMP threads without atomics
// (myOM.h:125-137); this build sets them serially, so its maps are the
// reference's without lost updates.
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "scene.h"

namespace mtsh {
namespace {

constexpr int N = MTSG_OM_SIZE, D = MTSG_OM_SIZE / 32;
constexpr float kEps = 1e-4f;   // Epsilon (constants.h:28)

struct Grid {
    std::vector<uint32_t> bits;   // [x][y][z / 32]
    Grid() : bits((size_t)N * N * D, 0u) {}
    void set(int x, int y, int z) { bits[((size_t)x * N + y) * D + (z >> 5)] |= 1u << (z & 31); }
    bool check(int x, int y, int z) const { return x >= 0 && x < N && y >= 0 && y < N && z >= 0 && z < N; }
    bool get(int x, int y, int z) const { return bits[((size_t)x * N + y) * D + (z >> 5)] & (1u << (z & 31)); }
};

struct P3 { float x, y, z; };

// setTriangle (myOM.h:140-161) on grid coordinates
void setTriangle(Grid &g, const P3 &p0, const P3 &p1, const P3 &p2) {
    const int a[3] = {(int)p0.x, (int)p0.y, (int)p0.z}, b[3] = {(int)p1.x, (int)p1.y, (int)p1.z},
              c[3] = {(int)p2.x, (int)p2.y, (int)p2.z};
    for (const int *q : {a, b, c})
        if (g.check(q[0], q[1], q[2])) g.set(q[0], q[1], q[2]);   // getGridIndexf2i assumes the cube holds the mesh
    int l = 0;
    for (int k = 0; k < 3; ++k) l += std::abs(b[k] - a[k]) + std::abs(c[k] - b[k]) + std::abs(a[k] - c[k]);
    if (l <= 4) return;   // closeEnough
    auto mid = [](const P3 &u, const P3 &v) { return P3{u.x + (v.x - u.x) / 2, u.y + (v.y - u.y) / 2, u.z + (v.z - u.z) / 2}; };
    const P3 p01 = mid(p0, p1), p12 = mid(p1, p2), p20 = mid(p2, p0);
    setTriangle(g, p0, p01, p20);
    setTriangle(g, p1, p12, p01);
    setTriangle(g, p2, p20, p12);
    setTriangle(g, p01, p12, p20);
}

// OccupancyMap::concentricMap (myOM.h:506-532)
V3 concentricMap(float u, float v) {
    const float x = u * 2 - 1, y = v * 2 - 1;
    float phi, r;
    if (x > -y) {
        if (x > y) { r = x; phi = (float)((M_PI / 4) * (y / x)); }
        else { r = y; phi = (float)((M_PI / 4) * (2 - x / y)); }
    } else if (x < y) {
        r = -x; phi = (float)((M_PI / 4) * (4 + y / x));
    } else {
        r = -y;
        phi = y != 0 ? (float)((M_PI / 4) * (6 - x / y)) : 0.0f;
    }
    const float z = 1 - r * r;
    return V3(std::cos(phi) * std::sqrt(1 - z * z) / r, std::sin(phi) * std::sqrt(1 - z * z) / r, z);
}

struct Quat { V3 v; float w; };

// Quaternion::fromDirectionPair (quat.h:205-227), then normalize (quat.h:352-354)
Quat fromDirectionPair(const V3 &from, const V3 &to) {
    const float dp = dot(from, to);
    Quat q{V3(0.0f), 1.0f};
    if (dp > 1 - kEps) {
        q = Quat{V3(0.0f), 1.0f};
    } else if (dp < -(1 - kEps)) {
        V3 axis = cross(from, V3(1, 0, 0));
        float len = length(axis);
        if (len < kEps) { axis = cross(from, V3(0, 1, 0)); len = length(axis); }
        q = Quat{axis / len, 0.0f};
    } else {
        const float cosTheta = std::sqrt(0.5f * (1 + dp)), sinTheta = std::sqrt(0.5f * (1 - dp));
        q = Quat{normalize(cross(from, to)) * sinTheta, cosTheta};
    }
    const float n = std::sqrt(dot(q.v, q.v) + q.w * q.w);
    return Quat{q.v / n, q.w / n};
}

// Quaternion::toTransform (quat.h:301-327): the PBRT matrix m; the
// transform's matrix is m transposed and its inverse m itself
void quatMatrix(const Quat &q, float m[3][3]) {
    const float xx = q.v.x * q.v.x, yy = q.v.y * q.v.y, zz = q.v.z * q.v.z;
    const float xy = q.v.x * q.v.y, xz = q.v.x * q.v.z, yz = q.v.y * q.v.z;
    const float wx = q.v.x * q.w, wy = q.v.y * q.w, wz = q.v.z * q.w;
    m[0][0] = 1.f - 2.f * (yy + zz); m[0][1] = 2.f * (xy + wz);       m[0][2] = 2.f * (xz - wy);
    m[1][0] = 2.f * (xy - wz);       m[1][1] = 1.f - 2.f * (xx + zz); m[1][2] = 2.f * (yz + wx);
    m[2][0] = 2.f * (xz + wy);       m[2][1] = 2.f * (yz - wx);       m[2][2] = 1.f - 2.f * (xx + yy);
}

}  // namespace

void buildOccupancyMaps(Scene &scene) {
    // the scene's TriMeshes (Scene::addShape, scene.cpp:642-643): not
    // rectangles, not instances
    V3 mn(1e30f), mx(-1e30f);
    size_t nMesh = 0;
    for (const Mesh &m : scene.meshes) {
        if (m.instanced || m.group >= 0) continue;
        ++nMesh;
        for (const V3 &p : m.p)
            for (int k = 0; k < 3; ++k) { mn[k] = std::min(mn[k], p[k]); mx[k] = std::max(mx[k], p[k]); }
    }
    if (!nMesh) throw std::runtime_error("myPath2_OM: the occupancy maps need at least one triangle mesh in the scene");
    mtsg_om &om = scene.omDesc;
    memset(&om, 0, sizeof(om));
    const V3 d = mx - mn;
    float r = length(d);
    r *= 0.5f * 1.001f;
    const V3 center = mn + d / 2.0f;
    const V3 lcorner = center - V3(r);
    const V3 amax = lcorner + V3(2 * r);
    // OccupancyMap::setAABB (myOM.h:36-44)
    const V3 ocenter = lcorner + (amax - lcorner) / 2;
    const float size = amax.x - lcorner.x, gridSize = size / N, recp = 1 / gridSize;
    for (int k = 0; k < 3; ++k) { om.aabb_min[k] = lcorner[k]; om.center[k] = ocenter[k]; }
    om.grid_size_recp = recp;

    Grid base;
    for (const Mesh &m : scene.meshes) {
        if (m.instanced || m.group >= 0) continue;
        auto gi = [&](const V3 &p) { return P3{(p.x - lcorner.x) * recp, (p.y - lcorner.y) * recp, (p.z - lcorner.z) * recp}; };
        for (size_t t = 0; t < m.idx.size(); t += 3) setTriangle(base, gi(m.p[m.idx[t]]), gi(m.p[m.idx[t + 1]]), gi(m.p[m.idx[t + 2]]));
    }

    scene.omBits.assign((size_t)MTSG_OM_COUNT * N * N * D, 0u);
    auto roma = [&](int id) {
        const int i = id / MTSG_OM_SQRT, j = id % MTSG_OM_SQRT;
        const V3 dir = normalize(concentricMap((i + 0.5f) / MTSG_OM_SQRT, (j + 0.5f) / MTSG_OM_SQRT));
        const Quat q = fromDirectionPair(V3(0, 0, 1), dir);
        float m[3][3];
        quatMatrix(q, m);
        for (int k = 0; k < 3; ++k) om.dir[id][k] = dir[k];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) om.rotate[id][3 * a + b] = m[a][b];   // m_rotate = toTransform().inverse()
        uint32_t *out = scene.omBits.data() + (size_t)id * N * N * D;
        // the transform's forward matrix (m transposed) applied to vectors
        auto fwd = [&](const V3 &v) {
            return V3(m[0][0] * v.x + m[1][0] * v.y + m[2][0] * v.z, m[0][1] * v.x + m[1][1] * v.y + m[2][1] * v.z,
                      m[0][2] * v.x + m[1][2] * v.y + m[2][2] * v.z);
        };
        const float radiu = (float)N / 2.0f;
        for (int x = 0; x < N; ++x)
            for (int y = 0; y < N; ++y) {
                const V3 xs((float)(x - radiu), (float)(y - radiu), 0.5f - radiu), xe((float)(x - radiu), (float)(y - radiu), radiu - 0.5f);
                V3 s = fwd(xs) + V3(radiu);
                const V3 e = fwd(xe) + V3(radiu);
                const V3 step = (e - s) / (float)(N - 1);
                uint32_t *col = out + ((size_t)x * N + y) * D;
                for (int k = 0; k < N; ++k) {
                    const int bx = (int)std::floor(s.x + kEps), by = (int)std::floor(s.y + kEps), bz = (int)std::floor(s.z + kEps);
                    if (base.check(bx, by, bz) && base.get(bx, by, bz)) col[k >> 5] |= 1u << (k & 31);
                    s = s + step;
                }
            }
    };
    std::vector<std::thread> th;
    for (int id = 0; id < MTSG_OM_COUNT; ++id) th.emplace_back(roma, id);
    for (auto &t : th) t.join();
}

}  // namespace mtsh
