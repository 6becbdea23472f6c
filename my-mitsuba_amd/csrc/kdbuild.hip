// kdbuild.hip -- SAH kd-tree construction on the GPU, the
// device-side counterpart of the host build (host/kdtree.cpp, after
// GenericKDTree::build, include/mitsuba/render/gkdtree.h:958-1240).
//
// Breadth-first, one level of the tree per step, every node of the level
// processed together:
//   k_bin      min-max binning (gkdtree.h MinMaxBins): per node and axis,
//              KD_BINS bins counting reference boxes by their minimum and by
//              their maximum; one workgroup per (node, chunk of refs) with an
//              LDS histogram flushed by global atomics
//   k_sah      the SAH sweep over the bin planes of the three axes with
//              Mitsuba's costs (traversal 15, query 20, empty-space bonus
//              0.9: gkdtree.h:734-744); one thread per node
//   k_count    exact child sizes for the chosen planes: a reference goes left
//              if its box starts below the plane, right if it ends above it
//              (a planar box on the plane goes left), a straddling triangle
//              only to the children its clipped polygon reaches
//   k_scatter  references of inner nodes into the next level's array, a
//              straddling triangle clipped to each child box (Sutherland-
//              Hodgman, dropped from a child it misses: Mitsuba's perfect
//              splits), other boxes clipped to the child; leaves' primitive
//              indices into the final index list
//   k_sort_leaves  each leaf's indices ascending (the scatter's atomics
//              order them arbitrarily; sorting makes the tree deterministic)
// The host loop keeps the node list of the level (a few MB at most), makes
// the leaf decisions (stopPrims 4 by default, maxDepth 8 + 1.3 log2 N, SAH cost not
// below the leaf's) and writes the nodes in Mitsuba's KDNode encoding, so the
// result plugs into mtsg_scene_desc like the host-built tree.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mtsg.h"

namespace mtsg {
void set_last_error(const std::string &e);   // mtsg.hip
}

namespace {

constexpr int KD_BINS = 32;
constexpr int BIN_WORDS = 3 * KD_BINS * 2;    // [axis][bin][min, max]
constexpr uint32_t CHUNK = 4096;              // refs per binning workgroup
constexpr int BLK = 256;

struct Ref {
    float4 mn;   // w: primitive index (bits)
    float4 mx;   // w: node index within the level (bits)
};

struct NodeDev {
    uint32_t begin, count;
    float lo[3], hi[3];
};

struct Decision {   // k_sah -> host
    int axis;       // -1: no split candidate
    float split;
    float cost;
    uint32_t pad;
};

struct Plan {       // host -> k_count / k_scatter
    int axis;       // -1: leaf
    float split;
    uint32_t out0, out1;   // inner: next-level ref offsets of the children; leaf: index-list offset
    uint32_t child0;       // inner: next-level node index of the left child (right = +1)
    uint32_t pad[3];
};

struct Task { uint32_t node, begin, end, pad; };

__device__ inline float axisOf(const float4 &v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

__device__ inline int binOf(float x, float lo, float scale) {
    int b = (int)((x - lo) * scale);
    return b < 0 ? 0 : (b >= KD_BINS ? KD_BINS - 1 : b);
}

// Triangle::getClippedAABB's Sutherland-Hodgman polygon clipping against a
// box (in double precision, as the reference and host/build.cpp clip): false
// when nothing of the triangle is inside; else its box, clipped to the box
__device__ bool clip_triangle(const float4 &a, const float4 &b, const float4 &c, const float lo[3], const float hi[3], float3 &cmn,
                              float3 &cmx) {
    double poly[10][3], tmp[10][3];
    int n = 3;
    poly[0][0] = a.x; poly[0][1] = a.y; poly[0][2] = a.z;
    poly[1][0] = b.x; poly[1][1] = b.y; poly[1][2] = b.z;
    poly[2][0] = c.x; poly[2][1] = c.y; poly[2][2] = c.z;
    for (int axis = 0; axis < 3; ++axis)
        for (int side = 0; side < 2; ++side) {
            // sutherlandHodgman (triangle.cpp:70-73) gives up on fewer than
            // three vertices: the triangle only touches the box there
            if (n < 3) return false;
            const double plane = side == 0 ? lo[axis] : hi[axis];
            int m = 0;
            for (int i = 0; i < n; ++i) {
                const double *cur = poly[i], *nxt = poly[i + 1 < n ? i + 1 : 0];
                const bool curIn = side == 0 ? cur[axis] >= plane : cur[axis] <= plane;
                const bool nxtIn = side == 0 ? nxt[axis] >= plane : nxt[axis] <= plane;
                if (curIn && m < 10) { tmp[m][0] = cur[0]; tmp[m][1] = cur[1]; tmp[m][2] = cur[2]; ++m; }
                if (curIn != nxtIn && m < 10) {
                    const double t = (plane - cur[axis]) / (nxt[axis] - cur[axis]);
                    for (int k = 0; k < 3; ++k) tmp[m][k] = cur[k] + (nxt[k] - cur[k]) * t;
                    tmp[m][axis] = plane;
                    ++m;
                }
            }
            n = m;
            for (int i = 0; i < n; ++i) { poly[i][0] = tmp[i][0]; poly[i][1] = tmp[i][1]; poly[i][2] = tmp[i][2]; }
        }
    if (n == 0) return false;
    // rounded outwards (math::castflt_down / castflt_up, triangle.cpp:134-141):
    // a clipped bound rounded to nearest can land on the far side of a later
    // split plane and drop the triangle from a child it overlaps
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            mn[k] = fminf(mn[k], __double2float_rd(poly[i][k]));
            mx[k] = fmaxf(mx[k], __double2float_ru(poly[i][k]));
        }
    for (int k = 0; k < 3; ++k) { mn[k] = fmaxf(mn[k], lo[k]); mx[k] = fminf(mx[k], hi[k]); }
    cmn = make_float3(mn[0], mn[1], mn[2]);
    cmx = make_float3(mx[0], mx[1], mx[2]);
    return true;
}

struct Geo { const float4 *vtx; const uint4 *tri; uint32_t nTri; };

// the children a reference goes to, with its boxes there: straddling
// triangles are clipped to each child box and dropped where nothing of them
// is left (Mitsuba's perfect splits, gkdtree.h:2150-2230)
__device__ void classify(const Ref &r, const Plan &p, const NodeDev &n, const Geo &g, bool &goL, bool &goR, Ref &L, Ref &R) {
    const float mn = axisOf(r.mn, p.axis), mx = axisOf(r.mx, p.axis);
    goL = mn < p.split;
    goR = mx > p.split;
    if (!goL && !goR) goL = true;   // planar on the plane
    L = r;
    R = r;
    if (p.axis == 0) { L.mx.x = fminf(L.mx.x, p.split); R.mn.x = fmaxf(R.mn.x, p.split); }
    else if (p.axis == 1) { L.mx.y = fminf(L.mx.y, p.split); R.mn.y = fmaxf(R.mn.y, p.split); }
    else { L.mx.z = fminf(L.mx.z, p.split); R.mn.z = fmaxf(R.mn.z, p.split); }
    const uint32_t prim = __float_as_uint(r.mn.w);
    if (goL && goR && prim < g.nTri) {
        const uint4 t = g.tri[prim];
        const float4 a = g.vtx[t.x], b = g.vtx[t.y], c = g.vtx[t.z];
        float lhi[3] = {n.hi[0], n.hi[1], n.hi[2]}, rlo[3] = {n.lo[0], n.lo[1], n.lo[2]};
        lhi[p.axis] = p.split;
        rlo[p.axis] = p.split;
        float3 cmn, cmx;
        if (clip_triangle(a, b, c, n.lo, lhi, cmn, cmx)) { L.mn = make_float4(cmn.x, cmn.y, cmn.z, L.mn.w); L.mx = make_float4(cmx.x, cmx.y, cmx.z, L.mx.w); }
        else goL = false;
        if (clip_triangle(a, b, c, rlo, n.hi, cmn, cmx)) { R.mn = make_float4(cmn.x, cmn.y, cmn.z, R.mn.w); R.mx = make_float4(cmx.x, cmx.y, cmx.z, R.mx.w); }
        else goR = false;
    }
}

__global__ void k_bin(const Ref *refs, const NodeDev *nodes, const Task *tasks, uint32_t *bins) {
    __shared__ uint32_t h[BIN_WORDS];
    const Task t = tasks[blockIdx.x];
    for (int i = threadIdx.x; i < BIN_WORDS; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const NodeDev n = nodes[t.node];
    float scale[3];
    for (int a = 0; a < 3; ++a) {
        const float ext = n.hi[a] - n.lo[a];
        scale[a] = ext > 0 ? (float)KD_BINS / ext : 0.0f;
    }
    for (uint32_t i = t.begin + threadIdx.x; i < t.end; i += blockDim.x) {
        const Ref r = refs[i];
        for (int a = 0; a < 3; ++a) {
            atomicAdd(&h[(a * KD_BINS + binOf(axisOf(r.mn, a), n.lo[a], scale[a])) * 2], 1u);
            atomicAdd(&h[(a * KD_BINS + binOf(axisOf(r.mx, a), n.lo[a], scale[a])) * 2 + 1], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < BIN_WORDS; i += blockDim.x)
        if (h[i]) atomicAdd(&bins[(size_t)t.node * BIN_WORDS + i], h[i]);
}

__device__ inline float area(const float lo[3], const float hi[3]) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

__global__ void k_sah(const NodeDev *nodes, uint32_t nNodes, const uint32_t *bins, Decision *out, float travCost, float queryCost,
                      float emptyBonus) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nNodes) return;
    const NodeDev n = nodes[i];
    const uint32_t *b = bins + (size_t)i * BIN_WORDS;
    const float sa = area(n.lo, n.hi);
    Decision best{-1, 0.0f, INFINITY, 0u};
    for (int a = 0; a < 3; ++a) {
        const float ext = n.hi[a] - n.lo[a];
        if (!(ext > 0) || !(sa > 0)) continue;
        uint32_t nR = 0;
        for (int k = 0; k < KD_BINS; ++k) nR += b[(a * KD_BINS + k) * 2 + 1];
        uint32_t nL = 0;
        for (int k = 1; k < KD_BINS; ++k) {
            nL += b[(a * KD_BINS + k - 1) * 2];
            nR -= b[(a * KD_BINS + k - 1) * 2 + 1];
            const float s = n.lo[a] + ext * ((float)k / (float)KD_BINS);
            if (!(s > n.lo[a] && s < n.hi[a])) continue;
            float lhi[3] = {n.hi[0], n.hi[1], n.hi[2]}, rlo[3] = {n.lo[0], n.lo[1], n.lo[2]};
            lhi[a] = s;
            rlo[a] = s;
            const float pL = area(n.lo, lhi) / sa, pR = area(rlo, n.hi) / sa;
            float cost = travCost + queryCost * (pL * (float)nL + pR * (float)nR);
            if (nL == 0 || nR == 0) cost *= emptyBonus;
            if (cost < best.cost) best = Decision{a, s, cost, 0u};
        }
    }
    out[i] = best;
}

// one counter pair per inner node: wave-aggregated when a wave's lanes share
// a node (the big nodes of the top levels)
__global__ void k_count(const Ref *refs, uint32_t nRefs, const Plan *plans, const NodeDev *nodes, Geo g, uint32_t *counts) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < nRefs;
    uint32_t node = 0xFFFFFFFFu;
    bool goL = false, goR = false;
    if (live) {
        const Ref r = refs[i];
        node = __float_as_uint(r.mx.w);
        const Plan p = plans[node];
        if (p.axis >= 0) {
            Ref L, R;
            classify(r, p, nodes[node], g, goL, goR, L, R);
        }
    }
    const uint32_t node0 = __shfl(node, 0);
    const bool uniform = __ballot(live && node != node0) == 0ull && node0 != 0xFFFFFFFFu;
    if (uniform) {
        const uint32_t cl = (uint32_t)__popcll(__ballot(goL)), cr = (uint32_t)__popcll(__ballot(goR));
        if ((threadIdx.x & 63) == 0) {
            if (cl) atomicAdd(&counts[2 * node0], cl);
            if (cr) atomicAdd(&counts[2 * node0 + 1], cr);
        }
    } else {
        if (goL) atomicAdd(&counts[2 * node], 1u);
        if (goR) atomicAdd(&counts[2 * node + 1], 1u);
    }
}

__global__ void k_scatter(const Ref *refs, uint32_t nRefs, const Plan *plans, const NodeDev *nodes, Geo g, uint32_t *cursors, Ref *next,
                          uint32_t *indices) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nRefs) return;
    const Ref r = refs[i];
    const uint32_t node = __float_as_uint(r.mx.w);
    const Plan p = plans[node];
    if (p.axis < 0) {
        const uint32_t at = atomicAdd(&cursors[2 * node], 1u);
        indices[p.out0 + at] = __float_as_uint(r.mn.w);
        return;
    }
    bool goL, goR;
    Ref L, R;
    classify(r, p, nodes[node], g, goL, goR, L, R);
    if (goL) {
        L.mx.w = __uint_as_float(p.child0);
        next[p.out0 + atomicAdd(&cursors[2 * node], 1u)] = L;
    }
    if (goR) {
        R.mx.w = __uint_as_float(p.child0 + 1);
        next[p.out1 + atomicAdd(&cursors[2 * node + 1], 1u)] = R;
    }
}

__global__ void k_sort_leaves(uint32_t *indices, const uint2 *ranges, uint32_t nLeaves) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= nLeaves) return;
    const uint2 r = ranges[l];
    for (uint32_t i = r.x + 1; i < r.y; ++i) {
        const uint32_t v = indices[i];
        uint32_t j = i;
        while (j > r.x && indices[j - 1] > v) { indices[j] = indices[j - 1]; --j; }
        indices[j] = v;
    }
}

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    bool reserve(size_t b) {
        if (b <= bytes) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, b) != hipSuccess) return false;
        bytes = b;
        return true;
    }
    template <class T> T *as() const { return (T *)p; }
};

struct HostNode { uint32_t begin, count, out, depth; float lo[3], hi[3]; };

inline float bitsToFloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

}  // namespace

extern "C" {

int mtsg_kd_build(int device, const mtsg_scene_desc *scene, const float *prim_bounds, const mtsg_kd_build_params *params,
                  mtsg_kd_tree *out) {
    using clock = std::chrono::steady_clock;
    const uint32_t n_prims = scene ? scene->n_prims : 0;
    if (!out || !scene || (n_prims && !prim_bounds) || (scene->n_triangles && (!scene->vtx_pos || !scene->tri_idx)) ||
        scene->n_triangles > n_prims) {
        mtsg::set_last_error("mtsg_kd_build: invalid arguments");
        return MTSG_ERR_INVALID;
    }
    memset(out, 0, sizeof(*out));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        mtsg::set_last_error("mtsg_kd_build: no such device");
        return MTSG_ERR_NODEVICE;
    }
    if (hipSetDevice(device) != hipSuccess) { mtsg::set_last_error("hipSetDevice failed"); return MTSG_ERR_DEVICE; }
    const auto t0 = clock::now();
    mtsg_kd_build_params P{15.0f, 20.0f, 0.9f, 4, 0, 0};   // NULL: the host build's defaults
    if (params) P = *params;
    // live primitives (an empty box marks one the tree leaves out) and the root box
    std::vector<Ref> refs0;
    refs0.reserve(n_prims);
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < n_prims; ++i) {
        const float *b = prim_bounds + 6 * (size_t)i;
        if (!(b[0] <= b[3] && b[1] <= b[4] && b[2] <= b[5])) continue;
        Ref r;
        r.mn = make_float4(b[0], b[1], b[2], bitsToFloat(i));
        r.mx = make_float4(b[3], b[4], b[5], bitsToFloat(0u));
        refs0.push_back(r);
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b[k]); hi[k] = std::max(hi[k], b[3 + k]); }
    }
    const uint32_t nLive = (uint32_t)refs0.size();
    // m_maxDepth = 8 + 1.3 log2i(N) (gkdtree.h:986-988)
    const int maxDepth = P.max_depth > 0 ? P.max_depth : (int)(8 + 1.3f * (float)(31 - __builtin_clz(std::max(1u, nLive))));
    std::vector<mtsg_kdnode> nodes(1);
    std::vector<uint2> leafRanges;
    if (nLive == 0) {
        nodes[0].combined = 0x80000000u;
        nodes[0].data = 0;
        for (int k = 0; k < 3; ++k) { lo[k] = 0; hi[k] = 0; }
    }
    DevBuf dRefs, dNext, dNodes, dTasks, dBins, dDec, dPlans, dCnt, dIdx, dRanges, dVtx, dTri;
    auto fail = [&](const char *what) {
        mtsg::set_last_error(std::string("mtsg_kd_build: ") + what);
        return MTSG_ERR_DEVICE;
    };
    size_t capRefs = std::max<size_t>(1024, (size_t)nLive * 4);
    size_t capIdx = capRefs;
    if (!dRefs.reserve(capRefs * sizeof(Ref)) || !dNext.reserve(capRefs * sizeof(Ref)) || !dIdx.reserve(capIdx * sizeof(uint32_t)))
        return fail("out of device memory");
    if (nLive && hipMemcpy(dRefs.p, refs0.data(), (size_t)nLive * sizeof(Ref), hipMemcpyHostToDevice) != hipSuccess) return fail("upload");
    // the triangles, for clipping straddling references
    Geo geo{nullptr, nullptr, scene->n_triangles};
    if (scene->n_triangles) {
        std::vector<float4> v(scene->n_vertices);
        std::vector<uint4> t(scene->n_triangles);
        for (uint32_t i = 0; i < scene->n_vertices; ++i)
            v[i] = make_float4(scene->vtx_pos[3 * i], scene->vtx_pos[3 * i + 1], scene->vtx_pos[3 * i + 2], 0.f);
        for (uint32_t i = 0; i < scene->n_triangles; ++i) {
            t[i] = make_uint4(scene->tri_idx[3 * i], scene->tri_idx[3 * i + 1], scene->tri_idx[3 * i + 2], 0u);
            if (t[i].x >= scene->n_vertices || t[i].y >= scene->n_vertices || t[i].z >= scene->n_vertices) {
                mtsg::set_last_error("mtsg_kd_build: triangle index out of range");
                return MTSG_ERR_INVALID;
            }
        }
        if (!dVtx.reserve(v.size() * sizeof(float4)) || !dTri.reserve(t.size() * sizeof(uint4)) ||
            hipMemcpy(dVtx.p, v.data(), v.size() * sizeof(float4), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(dTri.p, t.data(), t.size() * sizeof(uint4), hipMemcpyHostToDevice) != hipSuccess)
            return fail("upload");
        geo.vtx = dVtx.as<float4>();
        geo.tri = dTri.as<uint4>();
    }
    std::vector<HostNode> level;
    if (nLive) level.push_back(HostNode{0, nLive, 0, 0, {lo[0], lo[1], lo[2]}, {hi[0], hi[1], hi[2]}});
    uint32_t nRefs = nLive, nIndices = 0, depthReached = 0;
    std::vector<NodeDev> nd;
    std::vector<Task> tasks;
    std::vector<Decision> dec;
    std::vector<Plan> plans;
    std::vector<uint32_t> counts;
    while (!level.empty()) {
        const uint32_t nN = (uint32_t)level.size();
        nd.resize(nN);
        tasks.clear();
        for (uint32_t i = 0; i < nN; ++i) {
            const HostNode &h = level[i];
            nd[i] = NodeDev{h.begin, h.count, {h.lo[0], h.lo[1], h.lo[2]}, {h.hi[0], h.hi[1], h.hi[2]}};
            depthReached = std::max(depthReached, h.depth);
            if (h.count <= (uint32_t)P.stop_prims || (int)h.depth >= maxDepth) continue;   // leaf without binning
            for (uint32_t b = h.begin; b < h.begin + h.count; b += CHUNK) tasks.push_back(Task{i, b, std::min(b + CHUNK, h.begin + h.count), 0});
        }
        if (!dNodes.reserve(nN * sizeof(NodeDev)) || !dBins.reserve((size_t)nN * BIN_WORDS * 4) || !dDec.reserve(nN * sizeof(Decision)) ||
            !dPlans.reserve(nN * sizeof(Plan)) || !dCnt.reserve((size_t)nN * 2 * 4) || !dTasks.reserve(std::max<size_t>(1, tasks.size()) * sizeof(Task)))
            return fail("out of device memory");
        if (hipMemcpy(dNodes.p, nd.data(), nN * sizeof(NodeDev), hipMemcpyHostToDevice) != hipSuccess) return fail("upload");
        dec.assign(nN, Decision{-1, 0.0f, INFINITY, 0u});
        if (!tasks.empty()) {
            if (hipMemset(dBins.p, 0, (size_t)nN * BIN_WORDS * 4) != hipSuccess ||
                hipMemcpy(dTasks.p, tasks.data(), tasks.size() * sizeof(Task), hipMemcpyHostToDevice) != hipSuccess)
                return fail("upload");
            hipLaunchKernelGGL(k_bin, dim3((uint32_t)tasks.size()), dim3(BLK), 0, 0, dRefs.as<Ref>(), dNodes.as<NodeDev>(), dTasks.as<Task>(),
                               dBins.as<uint32_t>());
            hipLaunchKernelGGL(k_sah, dim3((nN + BLK - 1) / BLK), dim3(BLK), 0, 0, dNodes.as<NodeDev>(), nN, dBins.as<uint32_t>(),
                               dDec.as<Decision>(), P.traversal_cost, P.query_cost, P.empty_space_bonus);
            if (hipMemcpy(dec.data(), dDec.p, nN * sizeof(Decision), hipMemcpyDeviceToHost) != hipSuccess) return fail("download");
        }
        // leaf decisions
        plans.assign(nN, Plan{-1, 0.0f, 0, 0, 0, {0, 0, 0}});
        for (uint32_t i = 0; i < nN; ++i) {
            const HostNode &h = level[i];
            const bool leaf = h.count <= (uint32_t)P.stop_prims || (int)h.depth >= maxDepth || dec[i].axis < 0 ||
                              !(dec[i].cost < P.query_cost * (float)h.count);
            if (!leaf) { plans[i].axis = dec[i].axis; plans[i].split = dec[i].split; }
        }
        if (hipMemcpy(dPlans.p, plans.data(), nN * sizeof(Plan), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemset(dCnt.p, 0, (size_t)nN * 2 * 4) != hipSuccess)
            return fail("upload");
        hipLaunchKernelGGL(k_count, dim3((nRefs + BLK - 1) / BLK), dim3(BLK), 0, 0, dRefs.as<Ref>(), nRefs, dPlans.as<Plan>(), dNodes.as<NodeDev>(),
                           geo, dCnt.as<uint32_t>());
        counts.resize((size_t)nN * 2);
        if (hipMemcpy(counts.data(), dCnt.p, counts.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return fail("download");
        // allocate children, leaves and the next level
        std::vector<HostNode> next;
        uint32_t nextRefs = 0;
        for (uint32_t i = 0; i < nN; ++i) {
            const HostNode &h = level[i];
            Plan &p = plans[i];
            if (p.axis < 0) {
                p.out0 = nIndices;
                nodes[h.out].combined = 0x80000000u | nIndices;
                nodes[h.out].data = nIndices + h.count;
                leafRanges.push_back(make_uint2(nIndices, nIndices + h.count));
                nIndices += h.count;
                continue;
            }
            const uint32_t left = (uint32_t)nodes.size();
            nodes.resize(nodes.size() + 2);
            uint32_t splitBits;
            memcpy(&splitBits, &p.split, 4);
            nodes[h.out].combined = (uint32_t)p.axis | ((left - h.out) << 2);
            nodes[h.out].data = splitBits;
            p.child0 = (uint32_t)next.size();
            p.out0 = nextRefs;
            p.out1 = nextRefs + counts[2 * i];
            HostNode L{p.out0, counts[2 * i], left, h.depth + 1, {h.lo[0], h.lo[1], h.lo[2]}, {h.hi[0], h.hi[1], h.hi[2]}};
            HostNode R{p.out1, counts[2 * i + 1], left + 1, h.depth + 1, {h.lo[0], h.lo[1], h.lo[2]}, {h.hi[0], h.hi[1], h.hi[2]}};
            L.hi[p.axis] = p.split;
            R.lo[p.axis] = p.split;
            next.push_back(L);
            next.push_back(R);
            nextRefs += counts[2 * i] + counts[2 * i + 1];
        }
        if (nodes.size() >= (1u << 28)) return fail("too many nodes");
        // capacity of the next level and of the index list
        if (nextRefs > capRefs) {
            const size_t cap = (size_t)nextRefs * 3 / 2;
            DevBuf grown;
            if (!grown.reserve(cap * sizeof(Ref)) ||
                hipMemcpy(grown.p, dRefs.p, (size_t)nRefs * sizeof(Ref), hipMemcpyDeviceToDevice) != hipSuccess)
                return fail("out of device memory");
            std::swap(dRefs.p, grown.p);
            std::swap(dRefs.bytes, grown.bytes);
            if (!dNext.reserve(cap * sizeof(Ref))) return fail("out of device memory");
            capRefs = cap;
        }
        if (nIndices > capIdx) {
            const size_t cap = (size_t)nIndices * 3 / 2;
            DevBuf grown;
            if (!grown.reserve(cap * 4) || hipMemcpy(grown.p, dIdx.p, capIdx * 4, hipMemcpyDeviceToDevice) != hipSuccess)
                return fail("out of device memory");
            std::swap(dIdx.p, grown.p);
            std::swap(dIdx.bytes, grown.bytes);
            capIdx = cap;
        }
        if (hipMemcpy(dPlans.p, plans.data(), nN * sizeof(Plan), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemset(dCnt.p, 0, (size_t)nN * 2 * 4) != hipSuccess)
            return fail("upload");
        hipLaunchKernelGGL(k_scatter, dim3((nRefs + BLK - 1) / BLK), dim3(BLK), 0, 0, dRefs.as<Ref>(), nRefs, dPlans.as<Plan>(),
                           dNodes.as<NodeDev>(), geo, dCnt.as<uint32_t>(), dNext.as<Ref>(), dIdx.as<uint32_t>());
        std::swap(dRefs.p, dNext.p);
        std::swap(dRefs.bytes, dNext.bytes);
        nRefs = nextRefs;
        level.swap(next);
    }
    const uint32_t nLeaves = (uint32_t)leafRanges.size();
    if (nLeaves) {
        if (!dRanges.reserve(nLeaves * sizeof(uint2)) ||
            hipMemcpy(dRanges.p, leafRanges.data(), nLeaves * sizeof(uint2), hipMemcpyHostToDevice) != hipSuccess)
            return fail("upload");
        hipLaunchKernelGGL(k_sort_leaves, dim3((nLeaves + BLK - 1) / BLK), dim3(BLK), 0, 0, dIdx.as<uint32_t>(), dRanges.as<uint2>(), nLeaves);
    }
    out->n_nodes = (uint32_t)nodes.size();
    out->n_indices = nIndices;
    out->nodes = (mtsg_kdnode *)malloc(nodes.size() * sizeof(mtsg_kdnode));
    out->indices = (uint32_t *)malloc(std::max<size_t>(1, nIndices) * sizeof(uint32_t));
    if (!out->nodes || !out->indices) { mtsg_kd_free(out); mtsg::set_last_error("mtsg_kd_build: out of host memory"); return MTSG_ERR_OOM; }
    memcpy(out->nodes, nodes.data(), nodes.size() * sizeof(mtsg_kdnode));
    if (nIndices && hipMemcpy(out->indices, dIdx.p, (size_t)nIndices * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        mtsg_kd_free(out);
        return fail("download");
    }
    if (hipDeviceSynchronize() != hipSuccess) { mtsg_kd_free(out); return fail("kernel failure"); }
    // the enlarged tree AABB (MTS_KD_AABB_EPSILON, gkdtree.h:1213-1220), as host/kdtree.cpp
    const float eps = 1e-3f;
    for (int k = 0; k < 3; ++k) {
        const float ext = hi[k] - lo[k];
        out->aabb_min[k] = lo[k] - ext * eps - eps;
        out->aabb_max[k] = hi[k] + (hi[k] - out->aabb_min[k]) * eps + eps;
    }
    out->max_depth = depthReached;
    out->leaves = nLeaves;
    out->ms_build = std::chrono::duration<double, std::milli>(clock::now() - t0).count();
    return MTSG_OK;
}

void mtsg_kd_free(mtsg_kd_tree *t) {
    if (!t) return;
    free(t->nodes);
    free(t->indices);
    t->nodes = nullptr;
    t->indices = nullptr;
    t->n_nodes = t->n_indices = 0;
}

}  // extern "C"
