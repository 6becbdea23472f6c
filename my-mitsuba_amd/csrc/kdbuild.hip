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

constexpr int KD_BINS = 128;                  // Mitsuba's m_minMaxBins (gkdtree.h:2406-2500)
constexpr int BIN_WORDS = 3 * KD_BINS * 2;    // [axis][bin][min, max]
// nodes of at most EXACT_MAX references get Mitsuba's exact O(n log n) SAH
// sweep over their sorted edge events (gkdtree.h:1954-2400), one workgroup
// per node with the events in LDS; larger ones are binned.  (Mitsuba sweeps
// exactly below 65,536; the host build's sweep at a 4,096 threshold renders
// C3 within 1% of that)
constexpr uint32_t EXACT_MAX = 4096;
constexpr int EXACT_BLK = 1024;
constexpr int MAX_BAD_REFINES = 3;            // m_maxBadRefines
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

struct Decision {   // k_sah / k_exact -> host
    int axis;       // -1: no split candidate
    float split;
    float cost;
    uint32_t planarLeft;   // primitives lying in the split plane go left (exact sweep)
};

struct Plan {       // host -> k_count / k_scatter
    int axis;       // -1: leaf
    float split;
    uint32_t out0, out1;   // inner: next-level ref offsets of the children; leaf: index-list offset
    uint32_t child0;       // inner: next-level node index of the left child (right = +1)
    uint32_t planarLeft;
    uint32_t pad[2];
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
    if (!goL && !goR) { goL = p.planarLeft != 0; goR = !goL; }   // planar, in the plane
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
        scale[a] = ext > 0 ? (float)KD_BINS / ext : 0.0f;   // invW of findBinned
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

// SurfaceAreaHeuristic3 (sahkdtree3.h:39-84) in the host build's form
// (host/kdtree.cpp cost), so both builds price a split identically
__device__ inline float sah_cost(const float lo[3], const float hi[3], int axis, float pos, uint32_t nL, uint32_t nR,
                                 float travCost, float queryCost, float emptyBonus) {
    const float ex = hi[0] - lo[0], ey = hi[1] - lo[1], ez = hi[2] - lo[2];
    const float tmp = ex * ey + ey * ez + ex * ez;
    if (tmp <= 0) return INFINITY;
    const float inv = 1.0f / tmp;
    const float e[3] = {ex, ey, ez};
    const int a1 = axis == 2 ? 0 : axis + 1, a2 = axis == 0 ? 2 : axis - 1;
    const float t0 = e[a1] * e[a2] * inv, t1 = (e[a1] + e[a2]) * inv;
    const float pL = t0 + t1 * (pos - lo[axis]), pR = t0 + t1 * (hi[axis] - pos);
    float c = travCost + queryCost * (pL * (float)nL + pR * (float)nR);
    if (nL == 0 || nR == 0) c *= emptyBonus;
    return c;
}

__global__ void k_sah(const NodeDev *nodes, uint32_t nNodes, const uint32_t *bins, Decision *out, float travCost, float queryCost,
                      float emptyBonus) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nNodes) return;
    const NodeDev n = nodes[i];
    if (n.count <= EXACT_MAX) return;   // k_exact's node, or a leaf
    const uint32_t *b = bins + (size_t)i * BIN_WORDS;
    Decision best{-1, 0.0f, INFINITY, 1u};
    // findBinned (host/kdtree.cpp; gkdtree.h:2406-2500 MinMaxBins::bestSplit)
    for (int a = 0; a < 3; ++a) {
        const float ext = n.hi[a] - n.lo[a];
        if (!(ext > 0)) continue;
        const float w = ext / (float)KD_BINS;
        uint32_t nR = n.count, nL = 0;
        for (int k = 1; k < KD_BINS; ++k) {
            nL += b[(a * KD_BINS + k - 1) * 2];
            nR -= b[(a * KD_BINS + k - 1) * 2 + 1];
            const float s = n.lo[a] + w * (float)k;
            if (!(s > n.lo[a] && s < n.hi[a])) continue;
            const float cost = sah_cost(n.lo, n.hi, a, s, nL, nR, travCost, queryCost, emptyBonus);
            if (cost < best.cost) best = Decision{a, s, cost, 1u};
        }
    }
    out[i] = best;
}

// The exact SAH sweep of one node (findExact, host/kdtree.cpp; Mitsuba's
// buildTree edge-event sweep, gkdtree.h:1954-2400): per axis, the edge events
// of the node's references -- start / end of a box, one planar event for a
// box flat on that axis -- sorted by (position, end < planar < start) with a
// bitonic sort in LDS; two exclusive scans give, at the first event of each
// position, the references left of the plane (started or planar before it)
// and right of it (not yet ended); both placements of the planar ones are
// priced.  The winner is the cheapest candidate, the earliest one in
// (axis, position, left-before-right) order on ties, as the serial sweep.
__device__ inline uint32_t ordered(float f) {
    const uint32_t u = __float_as_uint(f == 0.0f ? 0.0f : f);   // -0 and +0: one position
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float unordered(uint32_t o) { return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o); }

__global__ void __launch_bounds__(EXACT_BLK) k_exact(const Ref *refs, const NodeDev *nodes, const uint32_t *taskNodes, Decision *out,
                                                     float travCost, float queryCost, float emptyBonus) {
    extern __shared__ unsigned long long ev[];                 // 2 * EXACT_MAX events
    __shared__ uint32_t scanA[EXACT_BLK], scanB[EXACT_BLK];   // per-thread totals -> exclusive prefixes
    __shared__ float bestCost[EXACT_BLK / 64], bestPos[EXACT_BLK / 64];
    __shared__ uint32_t bestKey[EXACT_BLK / 64];
    const uint32_t node = taskNodes[blockIdx.x];
    const NodeDev n = nodes[node];
    const uint32_t N = n.count;
    uint32_t m = 1;
    while (m < 2 * N) m <<= 1;                                // padded event count (power of two)
    const uint32_t per = (m + EXACT_BLK - 1) / EXACT_BLK;     // events per thread in the scans
    float myCost = INFINITY, myPos = 0.0f;
    uint32_t myKey = 0xFFFFFFFFu;                              // axis << 30 | event << 1 | right
    for (int a = 0; a < 3; ++a) {
        if (!(n.hi[a] > n.lo[a])) continue;
        // events: key = ordered(position) << 32 | type << 30 (0 end, 1 planar, 2 start)
        for (uint32_t i = threadIdx.x; i < m; i += EXACT_BLK) ev[i] = ~0ull;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < N; i += EXACT_BLK) {
            const Ref r = refs[n.begin + i];
            const float lo = axisOf(r.mn, a), hi = axisOf(r.mx, a);
            if (lo == hi) {
                ev[2 * i] = (unsigned long long)ordered(lo) << 32 | 1ull << 30;
            } else {
                ev[2 * i] = (unsigned long long)ordered(lo) << 32 | 2ull << 30;
                ev[2 * i + 1] = (unsigned long long)ordered(hi) << 32;
            }
        }
        __syncthreads();
        for (uint32_t k = 2; k <= m; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = threadIdx.x; i < m; i += EXACT_BLK) {
                    const uint32_t l = i ^ j;
                    if (l > i) {
                        const unsigned long long x = ev[i], y = ev[l];
                        if (((i & k) == 0) == (x > y)) { ev[i] = y; ev[l] = x; }
                    }
                }
                __syncthreads();
            }
        // exclusive scans of (start | planar) and (end | planar) over events
        const uint32_t e0 = threadIdx.x * per;
        uint32_t sa = 0, sb = 0;
        for (uint32_t e = e0; e < min(m, e0 + per); ++e) {
            const unsigned long long x = ev[e];
            if (x == ~0ull) continue;
            const uint32_t ty = (uint32_t)(x >> 30) & 3u;
            sa += ty != 0u;
            sb += ty != 2u;
        }
        scanA[threadIdx.x] = sa;
        scanB[threadIdx.x] = sb;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t ra = 0, rb = 0;
            for (int t = 0; t < EXACT_BLK; ++t) {
                const uint32_t xa = scanA[t], xb = scanB[t];
                scanA[t] = ra;
                scanB[t] = rb;
                ra += xa;
                rb += xb;
            }
        }
        __syncthreads();
        uint32_t pa = scanA[threadIdx.x], pb = scanB[threadIdx.x];
        for (uint32_t e = e0; e < min(m, e0 + per); ++e) {
            const unsigned long long x = ev[e];
            if (x == ~0ull) break;
            const uint32_t ty = (uint32_t)(x >> 30) & 3u;
            const uint32_t pos = (uint32_t)(x >> 32);
            if (e == 0 || (uint32_t)(ev[e - 1] >> 32) != pos) {
                // first event at this position: count the group's ends and planars
                uint32_t pe = 0, pp = 0;
                for (uint32_t f = e; f < m && ev[f] != ~0ull && (uint32_t)(ev[f] >> 32) == pos; ++f) {
                    const uint32_t t2 = (uint32_t)(ev[f] >> 30) & 3u;
                    pe += t2 == 0u;
                    pp += t2 == 1u;
                }
                const float p = unordered(pos);
                if (p > n.lo[a] && p < n.hi[a]) {
                    const uint32_t nL = pa, nR = N - pb - pe - pp;
                    const float cl = sah_cost(n.lo, n.hi, a, p, nL + pp, nR, travCost, queryCost, emptyBonus);
                    const float cr = sah_cost(n.lo, n.hi, a, p, nL, nR + pp, travCost, queryCost, emptyBonus);
                    const uint32_t key = (uint32_t)a << 30 | e << 1;
                    if (cl < myCost || (cl == myCost && key < myKey)) { myCost = cl; myKey = key; myPos = p; }
                    if (cr < myCost || (cr == myCost && (key | 1u) < myKey)) { myCost = cr; myKey = key | 1u; myPos = p; }
                }
            }
            pa += ty != 0u;
            pb += ty != 2u;
        }
        __syncthreads();
    }
    // block minimum of (cost, key); the position travels with it
    for (int o = 32; o > 0; o >>= 1) {
        const float c2 = __shfl_down(myCost, o), p2 = __shfl_down(myPos, o);
        const uint32_t k2 = __shfl_down(myKey, o);
        if (c2 < myCost || (c2 == myCost && k2 < myKey)) { myCost = c2; myKey = k2; myPos = p2; }
    }
    if ((threadIdx.x & 63) == 0) {
        bestCost[threadIdx.x >> 6] = myCost;
        bestKey[threadIdx.x >> 6] = myKey;
        bestPos[threadIdx.x >> 6] = myPos;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float c = INFINITY, pos = 0.0f;
        uint32_t k = 0xFFFFFFFFu;
        for (int w = 0; w < EXACT_BLK / 64; ++w)
            if (bestCost[w] < c || (bestCost[w] == c && bestKey[w] < k)) { c = bestCost[w]; k = bestKey[w]; pos = bestPos[w]; }
        Decision d{-1, 0.0f, INFINITY, 1u};
        if (k != 0xFFFFFFFFu && c < INFINITY) d = Decision{(int)(k >> 30), pos, c, (k & 1u) ? 0u : 1u};
        out[node] = d;
    }
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

struct HostNode { uint32_t begin, count, out, depth, bad; float lo[3], hi[3]; };
// what the retraction pass needs of every node of the tree (box, references)
struct NodeInfo { float lo[3], hi[3]; uint32_t count; };

inline float bitsToFloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

// Retraction (m_retract, gkdtree.h:739-742 and 1910-1922; host/kdtree.cpp
// build): bottom up, a split whose subtree costs no less than a leaf of the
// node's references becomes that leaf (the unique primitives of its
// leaves).  Then the tree is re-laid out breadth first (children adjacent,
// KDNode encoding).  Returns the number of retracted splits.
uint32_t retract_and_compact(std::vector<mtsg_kdnode> &nodes, const std::vector<NodeInfo> &info, std::vector<uint32_t> &idx,
                             const mtsg_kd_build_params &P, uint32_t &leaves, uint32_t &depthOut) {
    const size_t n = nodes.size();
    std::vector<float> cost(n, 0.0f);
    std::vector<uint8_t> collapse(n, 0);
    auto isLeaf = [&](size_t i) { return (nodes[i].combined & 0x80000000u) != 0; };
    auto leftOf = [&](size_t i) { return i + (nodes[i].combined >> 2); };
    // post-order over the tree
    std::vector<std::pair<uint32_t, bool>> st{{0u, false}};
    uint32_t retracted = 0;
    while (!st.empty()) {
        auto [i, expanded] = st.back();
        st.pop_back();
        if (isLeaf(i)) { cost[i] = P.query_cost * (float)info[i].count; continue; }
        const uint32_t l = (uint32_t)leftOf(i);
        if (!expanded) {
            st.push_back({i, true});
            st.push_back({l, false});
            st.push_back({l + 1, false});
            continue;
        }
        const NodeInfo &b = info[i];
        const int axis = (int)(nodes[i].combined & 3u);
        const float pos = bitsToFloat(nodes[i].data);
        const float e[3] = {b.hi[0] - b.lo[0], b.hi[1] - b.lo[1], b.hi[2] - b.lo[2]};
        const float tmp = e[0] * e[1] + e[1] * e[2] + e[0] * e[2];
        const float inv = tmp > 0 ? 1.0f / tmp : 0.0f;
        const int a1 = (axis + 1) % 3, a2 = (axis + 2) % 3;
        const float t0 = e[a1] * e[a2] * inv, t1 = (e[a1] + e[a2]) * inv;
        const float pL = t0 + t1 * (pos - b.lo[axis]), pR = t0 + t1 * (b.hi[axis] - pos);
        const float finalCost = P.traversal_cost + (pL * cost[l] + pR * cost[l + 1]);
        const float leafCost = P.query_cost * (float)b.count;
        if (finalCost < leafCost) {
            cost[i] = finalCost;
        } else {
            cost[i] = leafCost;
            collapse[i] = 1;
            ++retracted;
        }
    }
    // breadth-first re-layout
    std::vector<mtsg_kdnode> out(1);
    std::vector<uint32_t> outIdx;
    outIdx.reserve(idx.size());
    leaves = 0;
    depthOut = 0;
    struct Q { uint32_t old, slot, depth; };
    std::vector<Q> q{{0u, 0u, 0u}};
    std::vector<uint32_t> ids;
    for (size_t h = 0; h < q.size(); ++h) {
        const Q c = q[h];
        depthOut = std::max(depthOut, c.depth);
        if (isLeaf(c.old) || collapse[c.old]) {
            ids.clear();
            // the primitives of the (sub)tree's leaves, unique and ascending
            std::vector<uint32_t> sub{c.old};
            while (!sub.empty()) {
                const uint32_t k = sub.back();
                sub.pop_back();
                if (isLeaf(k)) {
                    const uint32_t s0 = nodes[k].combined & 0x7FFFFFFFu, e0 = nodes[k].data;
                    ids.insert(ids.end(), idx.begin() + s0, idx.begin() + e0);
                } else {
                    const uint32_t l = (uint32_t)leftOf(k);
                    sub.push_back(l);
                    sub.push_back(l + 1);
                }
            }
            if (!isLeaf(c.old)) {
                std::sort(ids.begin(), ids.end());
                ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
            }
            out[c.slot].combined = 0x80000000u | (uint32_t)outIdx.size();
            outIdx.insert(outIdx.end(), ids.begin(), ids.end());
            out[c.slot].data = (uint32_t)outIdx.size();
            ++leaves;
            continue;
        }
        const uint32_t left = (uint32_t)out.size();
        out.resize(out.size() + 2);
        out[c.slot].combined = (nodes[c.old].combined & 3u) | ((left - c.slot) << 2);
        out[c.slot].data = nodes[c.old].data;
        const uint32_t ol = (uint32_t)leftOf(c.old);
        q.push_back({ol, left, c.depth + 1});
        q.push_back({ol + 1, left + 1, c.depth + 1});
    }
    nodes.swap(out);
    idx.swap(outIdx);
    return retracted;
}

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
    if (nLive) level.push_back(HostNode{0, nLive, 0, 0, 0, {lo[0], lo[1], lo[2]}, {hi[0], hi[1], hi[2]}});
    std::vector<NodeInfo> info(1, NodeInfo{{lo[0], lo[1], lo[2]}, {hi[0], hi[1], hi[2]}, nLive});
    uint32_t nRefs = nLive, nIndices = 0, depthReached = 0;
    std::vector<NodeDev> nd;
    std::vector<Task> tasks;
    std::vector<Decision> dec;
    std::vector<Plan> plans;
    std::vector<uint32_t> counts, exactNodes;
    DevBuf dExact;
    if (hipFuncSetAttribute((const void *)k_exact, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(2 * EXACT_MAX * sizeof(unsigned long long))) != hipSuccess)
        return fail("k_exact shared memory");
    while (!level.empty()) {
        const uint32_t nN = (uint32_t)level.size();
        nd.resize(nN);
        tasks.clear();
        exactNodes.clear();
        uint32_t exactMaxCount = 0;
        for (uint32_t i = 0; i < nN; ++i) {
            const HostNode &h = level[i];
            nd[i] = NodeDev{h.begin, h.count, {h.lo[0], h.lo[1], h.lo[2]}, {h.hi[0], h.hi[1], h.hi[2]}};
            depthReached = std::max(depthReached, h.depth);
            if (h.count <= (uint32_t)P.stop_prims || (int)h.depth >= maxDepth) continue;   // leaf without a sweep
            if (h.count <= EXACT_MAX) {
                exactNodes.push_back(i);
                exactMaxCount = std::max(exactMaxCount, h.count);
                continue;
            }
            for (uint32_t b = h.begin; b < h.begin + h.count; b += CHUNK) tasks.push_back(Task{i, b, std::min(b + CHUNK, h.begin + h.count), 0});
        }
        if (!dNodes.reserve(nN * sizeof(NodeDev)) || !dBins.reserve((size_t)nN * BIN_WORDS * 4) || !dDec.reserve(nN * sizeof(Decision)) ||
            !dPlans.reserve(nN * sizeof(Plan)) || !dCnt.reserve((size_t)nN * 2 * 4) || !dTasks.reserve(std::max<size_t>(1, tasks.size()) * sizeof(Task)))
            return fail("out of device memory");
        if (hipMemcpy(dNodes.p, nd.data(), nN * sizeof(NodeDev), hipMemcpyHostToDevice) != hipSuccess) return fail("upload");
        dec.assign(nN, Decision{-1, 0.0f, INFINITY, 1u});
        if (hipMemcpy(dDec.p, dec.data(), nN * sizeof(Decision), hipMemcpyHostToDevice) != hipSuccess) return fail("upload");
        if (!exactNodes.empty()) {
            if (!dExact.reserve(exactNodes.size() * sizeof(uint32_t)) ||
                hipMemcpy(dExact.p, exactNodes.data(), exactNodes.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess)
                return fail("upload");
            uint32_t m = 1;
            while (m < 2 * exactMaxCount) m <<= 1;
            hipLaunchKernelGGL(k_exact, dim3((uint32_t)exactNodes.size()), dim3(EXACT_BLK), m * sizeof(unsigned long long), 0,
                               dRefs.as<Ref>(), dNodes.as<NodeDev>(), dExact.as<uint32_t>(), dDec.as<Decision>(), P.traversal_cost,
                               P.query_cost, P.empty_space_bonus);
            if (hipGetLastError() != hipSuccess) return fail("k_exact launch");
        }
        if (!tasks.empty()) {
            if (hipMemset(dBins.p, 0, (size_t)nN * BIN_WORDS * 4) != hipSuccess ||
                hipMemcpy(dTasks.p, tasks.data(), tasks.size() * sizeof(Task), hipMemcpyHostToDevice) != hipSuccess)
                return fail("upload");
            hipLaunchKernelGGL(k_bin, dim3((uint32_t)tasks.size()), dim3(BLK), 0, 0, dRefs.as<Ref>(), dNodes.as<NodeDev>(), dTasks.as<Task>(),
                               dBins.as<uint32_t>());
            hipLaunchKernelGGL(k_sah, dim3((nN + BLK - 1) / BLK), dim3(BLK), 0, 0, dNodes.as<NodeDev>(), nN, dBins.as<uint32_t>(),
                               dDec.as<Decision>(), P.traversal_cost, P.query_cost, P.empty_space_bonus);
        }
        if ((!tasks.empty() || !exactNodes.empty()) &&
            hipMemcpy(dec.data(), dDec.p, nN * sizeof(Decision), hipMemcpyDeviceToHost) != hipSuccess)
            return fail("download");
        // leaf decisions
        // (buildTree's leaf / bad-refine decisions, gkdtree.h:1818-1850, as
        // host/kdtree.cpp: a split no cheaper than the leaf is still taken up
        // to MAX_BAD_REFINES times on a path, the retraction pass below
        // undoes the ones that did not pay off)
        plans.assign(nN, Plan{-1, 0.0f, 0, 0, 0, 1u, {0, 0}});
        std::vector<uint32_t> badOf(nN, 0);
        for (uint32_t i = 0; i < nN; ++i) {
            const HostNode &h = level[i];
            badOf[i] = h.bad;
            if (h.count <= (uint32_t)P.stop_prims || (int)h.depth >= maxDepth || dec[i].axis < 0) continue;
            const float leafCost = P.query_cost * (float)h.count;
            if (!(dec[i].cost < leafCost)) {
                if ((dec[i].cost > 4 * leafCost && h.count < 16) || (int)h.bad >= MAX_BAD_REFINES) continue;
                ++badOf[i];
            }
            plans[i].axis = dec[i].axis;
            plans[i].split = dec[i].split;
            plans[i].planarLeft = dec[i].planarLeft;
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
            info.resize(nodes.size());
            uint32_t splitBits;
            memcpy(&splitBits, &p.split, 4);
            nodes[h.out].combined = (uint32_t)p.axis | ((left - h.out) << 2);
            nodes[h.out].data = splitBits;
            p.child0 = (uint32_t)next.size();
            p.out0 = nextRefs;
            p.out1 = nextRefs + counts[2 * i];
            HostNode L{p.out0, counts[2 * i], left, h.depth + 1, badOf[i], {h.lo[0], h.lo[1], h.lo[2]}, {h.hi[0], h.hi[1], h.hi[2]}};
            HostNode R{p.out1, counts[2 * i + 1], left + 1, h.depth + 1, badOf[i], {h.lo[0], h.lo[1], h.lo[2]}, {h.hi[0], h.hi[1], h.hi[2]}};
            L.hi[p.axis] = p.split;
            R.lo[p.axis] = p.split;
            info[left] = NodeInfo{{L.lo[0], L.lo[1], L.lo[2]}, {L.hi[0], L.hi[1], L.hi[2]}, L.count};
            info[left + 1] = NodeInfo{{R.lo[0], R.lo[1], R.lo[2]}, {R.hi[0], R.hi[1], R.hi[2]}, R.count};
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
    std::vector<uint32_t> idx(nIndices);
    if (nIndices && hipMemcpy(idx.data(), dIdx.p, (size_t)nIndices * 4, hipMemcpyDeviceToHost) != hipSuccess) return fail("download");
    if (hipDeviceSynchronize() != hipSuccess) return fail("kernel failure");
    uint32_t nLeavesOut = nLeaves;
    if (nLive) retract_and_compact(nodes, info, idx, P, nLeavesOut, depthReached);
    out->n_nodes = (uint32_t)nodes.size();
    out->n_indices = (uint32_t)idx.size();
    out->nodes = (mtsg_kdnode *)malloc(nodes.size() * sizeof(mtsg_kdnode));
    out->indices = (uint32_t *)malloc(std::max<size_t>(1, idx.size()) * sizeof(uint32_t));
    if (!out->nodes || !out->indices) { mtsg_kd_free(out); mtsg::set_last_error("mtsg_kd_build: out of host memory"); return MTSG_ERR_OOM; }
    memcpy(out->nodes, nodes.data(), nodes.size() * sizeof(mtsg_kdnode));
    if (!idx.empty()) memcpy(out->indices, idx.data(), idx.size() * sizeof(uint32_t));
    // the enlarged tree AABB (MTS_KD_AABB_EPSILON, gkdtree.h:1213-1220), as host/kdtree.cpp
    const float eps = 1e-3f;
    for (int k = 0; k < 3; ++k) {
        const float ext = hi[k] - lo[k];
        out->aabb_min[k] = lo[k] - ext * eps - eps;
        out->aabb_max[k] = hi[k] + (hi[k] - out->aabb_min[k]) * eps + eps;
    }
    out->max_depth = depthReached;
    out->leaves = nLeavesOut;
    out->ms_build = std::chrono::duration<double, std::milli>(clock::now() - t0).count();
    return MTSG_OK;
}

// Refit: a tree's topology and split planes kept, its leaves refilled from the
// primitives' current bounds (deforming or moving geometry between frames, a
// rebuild without the SAH search).  The references are pushed down the given
// tree level by level with the build's own classification (k_count /
// k_scatter: straddling triangles clipped to each child box, Mitsuba's perfect
// splits), planar references in a split plane going left; every primitive
// therefore lands in every leaf its clipped box overlaps, so the tree answers
// exactly, at the SAH cost of the old planes.  Leaf ranges are re-laid out
// breadth first in the build's index order; inner nodes keep their words.
int mtsg_kd_refit(int device, const mtsg_scene_desc *scene, const float *prim_bounds, const mtsg_kd_tree *tree,
                  mtsg_kd_tree *out) {
    using clock = std::chrono::steady_clock;
    const uint32_t n_prims = scene ? scene->n_prims : 0;
    if (!out || !scene || !tree || !tree->nodes || tree->n_nodes == 0 || (n_prims && !prim_bounds) ||
        (scene->n_triangles && (!scene->vtx_pos || !scene->tri_idx)) || scene->n_triangles > n_prims) {
        mtsg::set_last_error("mtsg_kd_refit: invalid arguments");
        return MTSG_ERR_INVALID;
    }
    // the input tree must be well formed: children inside the array, acyclic
    // (each node reached once), breadth-first child pairs as the build writes
    {
        std::vector<uint8_t> seen(tree->n_nodes, 0);
        std::vector<uint32_t> st{0u};
        seen[0] = 1;
        while (!st.empty()) {
            const uint32_t i = st.back();
            st.pop_back();
            const mtsg_kdnode &N = tree->nodes[i];
            if (N.combined & 0x80000000u) continue;
            const uint64_t l = (uint64_t)i + ((N.combined & ~(3u | 0x40000000u)) >> 2);
            if ((N.combined & 3u) == 3u || l <= i || l + 1 >= tree->n_nodes || seen[l] || seen[l + 1]) {
                mtsg::set_last_error("mtsg_kd_refit: malformed tree");
                return MTSG_ERR_INVALID;
            }
            seen[l] = seen[l + 1] = 1;
            st.push_back((uint32_t)l);
            st.push_back((uint32_t)l + 1);
        }
    }
    memset(out, 0, sizeof(*out));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        mtsg::set_last_error("mtsg_kd_refit: no such device");
        return MTSG_ERR_NODEVICE;
    }
    if (hipSetDevice(device) != hipSuccess) { mtsg::set_last_error("hipSetDevice failed"); return MTSG_ERR_DEVICE; }
    const auto t0 = clock::now();
    auto fail = [&](const char *what) {
        mtsg::set_last_error(std::string("mtsg_kd_refit: ") + what);
        return MTSG_ERR_DEVICE;
    };
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
    if (nLive == 0)
        for (int k = 0; k < 3; ++k) { lo[k] = 0; hi[k] = 0; }
    std::vector<mtsg_kdnode> nodes(tree->nodes, tree->nodes + tree->n_nodes);
    DevBuf dRefs, dNext, dNodes, dPlans, dCnt, dIdx, dRanges, dVtx, dTri;
    size_t capRefs = std::max<size_t>(1024, (size_t)nLive * 2);
    size_t capIdx = capRefs;
    if (!dRefs.reserve(capRefs * sizeof(Ref)) || !dNext.reserve(capRefs * sizeof(Ref)) || !dIdx.reserve(capIdx * sizeof(uint32_t)))
        return fail("out of device memory");
    if (nLive && hipMemcpy(dRefs.p, refs0.data(), (size_t)nLive * sizeof(Ref), hipMemcpyHostToDevice) != hipSuccess) return fail("upload");
    Geo geo{nullptr, nullptr, scene->n_triangles};
    if (scene->n_triangles) {
        std::vector<float4> v(scene->n_vertices);
        std::vector<uint4> t(scene->n_triangles);
        for (uint32_t i = 0; i < scene->n_vertices; ++i)
            v[i] = make_float4(scene->vtx_pos[3 * i], scene->vtx_pos[3 * i + 1], scene->vtx_pos[3 * i + 2], 0.f);
        for (uint32_t i = 0; i < scene->n_triangles; ++i) {
            t[i] = make_uint4(scene->tri_idx[3 * i], scene->tri_idx[3 * i + 1], scene->tri_idx[3 * i + 2], 0u);
            if (t[i].x >= scene->n_vertices || t[i].y >= scene->n_vertices || t[i].z >= scene->n_vertices) {
                mtsg::set_last_error("mtsg_kd_refit: triangle index out of range");
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
    level.push_back(HostNode{0, nLive, 0, 0, 0, {lo[0], lo[1], lo[2]}, {hi[0], hi[1], hi[2]}});
    std::vector<uint2> leafRanges;
    std::vector<NodeDev> nd;
    std::vector<Plan> plans;
    std::vector<uint32_t> counts;
    uint32_t nRefs = nLive, nIndices = 0, depthReached = 0;
    while (!level.empty()) {
        const uint32_t nN = (uint32_t)level.size();
        nd.resize(nN);
        plans.assign(nN, Plan{-1, 0.0f, 0, 0, 0, 1u, {0, 0}});
        for (uint32_t i = 0; i < nN; ++i) {
            const HostNode &h = level[i];
            nd[i] = NodeDev{h.begin, h.count, {h.lo[0], h.lo[1], h.lo[2]}, {h.hi[0], h.hi[1], h.hi[2]}};
            depthReached = std::max(depthReached, h.depth);
            const mtsg_kdnode &N = nodes[h.out];
            if (!(N.combined & 0x80000000u)) {
                plans[i].axis = (int)(N.combined & 3u);
                plans[i].split = bitsToFloat(N.data);
            }
        }
        if (!dNodes.reserve(nN * sizeof(NodeDev)) || !dPlans.reserve(nN * sizeof(Plan)) || !dCnt.reserve((size_t)nN * 2 * 4))
            return fail("out of device memory");
        if (hipMemcpy(dNodes.p, nd.data(), nN * sizeof(NodeDev), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(dPlans.p, plans.data(), nN * sizeof(Plan), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemset(dCnt.p, 0, (size_t)nN * 2 * 4) != hipSuccess)
            return fail("upload");
        if (nRefs)
            hipLaunchKernelGGL(k_count, dim3((nRefs + BLK - 1) / BLK), dim3(BLK), 0, 0, dRefs.as<Ref>(), nRefs, dPlans.as<Plan>(),
                               dNodes.as<NodeDev>(), geo, dCnt.as<uint32_t>());
        counts.resize((size_t)nN * 2);
        if (hipMemcpy(counts.data(), dCnt.p, counts.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return fail("download");
        std::vector<HostNode> next;
        uint32_t nextRefs = 0;
        for (uint32_t i = 0; i < nN; ++i) {
            const HostNode &h = level[i];
            Plan &p = plans[i];
            mtsg_kdnode &N = nodes[h.out];
            if (p.axis < 0) {
                p.out0 = nIndices;
                N.combined = 0x80000000u | nIndices;
                N.data = nIndices + h.count;
                leafRanges.push_back(make_uint2(nIndices, nIndices + h.count));
                nIndices += h.count;
                continue;
            }
            const uint32_t left = h.out + ((N.combined & ~(3u | 0x40000000u)) >> 2);
            p.child0 = (uint32_t)next.size();
            p.out0 = nextRefs;
            p.out1 = nextRefs + counts[2 * i];
            HostNode L{p.out0, counts[2 * i], left, h.depth + 1, 0, {h.lo[0], h.lo[1], h.lo[2]}, {h.hi[0], h.hi[1], h.hi[2]}};
            HostNode R{p.out1, counts[2 * i + 1], left + 1, h.depth + 1, 0, {h.lo[0], h.lo[1], h.lo[2]}, {h.hi[0], h.hi[1], h.hi[2]}};
            L.hi[p.axis] = p.split;
            R.lo[p.axis] = p.split;
            next.push_back(L);
            next.push_back(R);
            nextRefs += counts[2 * i] + counts[2 * i + 1];
        }
        if (nextRefs > capRefs) {
            const size_t cap = (size_t)nextRefs * 3 / 2;
            DevBuf grown;
            if (!grown.reserve(cap * sizeof(Ref)) ||
                (nRefs && hipMemcpy(grown.p, dRefs.p, (size_t)nRefs * sizeof(Ref), hipMemcpyDeviceToDevice) != hipSuccess))
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
        if (nRefs)
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
    std::vector<uint32_t> idx(nIndices);
    if (nIndices && hipMemcpy(idx.data(), dIdx.p, (size_t)nIndices * 4, hipMemcpyDeviceToHost) != hipSuccess) return fail("download");
    if (hipDeviceSynchronize() != hipSuccess) return fail("kernel failure");
    out->n_nodes = (uint32_t)nodes.size();
    out->n_indices = (uint32_t)idx.size();
    out->nodes = (mtsg_kdnode *)malloc(nodes.size() * sizeof(mtsg_kdnode));
    out->indices = (uint32_t *)malloc(std::max<size_t>(1, idx.size()) * sizeof(uint32_t));
    if (!out->nodes || !out->indices) { mtsg_kd_free(out); mtsg::set_last_error("mtsg_kd_refit: out of host memory"); return MTSG_ERR_OOM; }
    memcpy(out->nodes, nodes.data(), nodes.size() * sizeof(mtsg_kdnode));
    if (!idx.empty()) memcpy(out->indices, idx.data(), idx.size() * sizeof(uint32_t));
    const float eps = 1e-3f;   // the enlarged AABB of the build (gkdtree.h:1213-1220)
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
