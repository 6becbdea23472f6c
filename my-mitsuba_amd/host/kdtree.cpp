// SAH kd-tree construction (host preprocessing, excluded from the metric
// exactly as in Mitsuba, src/librender/renderjob.cpp:102,113).
//
// Follows GenericKDTree's cost model and termination rules
// (include/mitsuba/render/gkdtree.h:734-744 parameters, :1792-1950 min-max
// binning, :1954-2400 exact sweep, :1797-1842 leaf/bad-refine criteria,
// sahkdtree3.h:39-84 SurfaceAreaHeuristic3) with perfect-split clipping of
// triangles (Triangle::getClippedAABB) and retraction of splits whose
// subtree ends up costlier than a leaf (m_retract, gkdtree.h:739-742,
// 1895-1922; createLeafAfterRetraction :1665-1699).  Indirection nodes are
// not implemented: any valid kd-tree yields the same closest hits, so the
// traversal kernels only rely on the node encoding (gkdtree.h:452-600), not
// on Mitsuba's exact split choices.
#include <atomic>
#include <chrono>
#include <cstring>
#include <future>
#include <mutex>
#include <thread>

#include "scene.h"

namespace mtsh {
namespace {

struct BPrim {
    uint32_t id;
    float lo[3], hi[3];
};

struct Sub {                         // independently built subtree
    std::vector<mtsg_kdnode> nodes;
    std::vector<uint32_t> indices;
    uint32_t maxDepth = 0;
    size_t leaves = 0, nonEmpty = 0, retracted = 0;
};

struct Split {
    int axis = -1;
    float pos = 0;
    float cost = INFINITY;
    bool planarLeft = true;
};

struct Builder {
    const PrimSource &src;
    KDBuildParams P;
    int maxDepth;
    size_t parallelCut;

    Builder(const PrimSource &s, const KDBuildParams &p, int md, size_t cut)
        : src(s), P(p), maxDepth(md), parallelCut(cut) {}

    static float areaOf(const float lo[3], const float hi[3]) {
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }

    // SurfaceAreaHeuristic3 probabilities of the two children
    // (sahkdtree3.h:39-84, TreeConstructionHeuristic::operator())
    static void probs(const AABB &box, int axis, float pos, float &pL, float &pR) {
        V3 ext = box.extents();
        float tmp = ext.x * ext.y + ext.y * ext.z + ext.x * ext.z;
        float inv = tmp > 0 ? 1.0f / tmp : 0.0f;
        int a1 = (axis + 1) % 3, a2 = (axis + 2) % 3;
        float t0 = ext[a1] * ext[a2] * inv, t1 = (ext[a1] + ext[a2]) * inv;
        pL = t0 + t1 * (pos - box.mn[axis]);
        pR = t0 + t1 * (box.mx[axis] - pos);
    }

    // SurfaceAreaHeuristic3 as a cost for split (axis, pos) of box
    float cost(const AABB &box, int axis, float pos, size_t nL, size_t nR) const {
        V3 ext = box.extents();
        float tmp = ext.x * ext.y + ext.y * ext.z + ext.x * ext.z;
        if (tmp <= 0) return INFINITY;
        float inv = 1.0f / tmp;
        int a1 = (axis + 1) % 3, a2 = (axis + 2) % 3;
        float t0 = ext[a1] * ext[a2] * inv;
        float t1 = (ext[a1] + ext[a2]) * inv;
        float pL = t0 + t1 * (pos - box.mn[axis]);
        float pR = t0 + t1 * (box.mx[axis] - pos);
        float c = P.traversalCost + P.queryCost * (pL * nL + pR * nR);
        if (nL == 0 || nR == 0) c *= P.emptySpaceBonus;
        return c;
    }

    Split findExact(const AABB &box, const std::vector<BPrim> &prims) const {
        Split best;
        size_t N = prims.size();
        struct Ev { float p; int type; };  // 0 end, 1 planar, 2 start
        std::vector<Ev> ev;
        ev.reserve(2 * N);
        for (int axis = 0; axis < 3; ++axis) {
            if (box.mx[axis] <= box.mn[axis]) continue;
            ev.clear();
            for (const BPrim &p : prims) {
                if (p.lo[axis] == p.hi[axis]) ev.push_back({p.lo[axis], 1});
                else { ev.push_back({p.lo[axis], 2}); ev.push_back({p.hi[axis], 0}); }
            }
            std::sort(ev.begin(), ev.end(), [](const Ev &a, const Ev &b) {
                return a.p < b.p || (a.p == b.p && a.type < b.type);
            });
            size_t nL = 0, nP = 0, nR = N;
            for (size_t i = 0; i < ev.size();) {
                float pos = ev[i].p;
                size_t pe = 0, pp = 0, ps = 0;
                while (i < ev.size() && ev[i].p == pos && ev[i].type == 0) { ++pe; ++i; }
                while (i < ev.size() && ev[i].p == pos && ev[i].type == 1) { ++pp; ++i; }
                while (i < ev.size() && ev[i].p == pos && ev[i].type == 2) { ++ps; ++i; }
                nP = pp;
                nR -= pp + pe;
                if (pos > box.mn[axis] && pos < box.mx[axis]) {
                    float cl = cost(box, axis, pos, nL + nP, nR);
                    float cr = cost(box, axis, pos, nL, nR + nP);
                    if (cl < best.cost) { best.cost = cl; best.axis = axis; best.pos = pos; best.planarLeft = true; }
                    if (cr < best.cost) { best.cost = cr; best.axis = axis; best.pos = pos; best.planarLeft = false; }
                }
                nL += ps + pp;
                nP = 0;
            }
        }
        return best;
    }

    Split findBinned(const AABB &box, const std::vector<BPrim> &prims) const {
        Split best;
        const int B = P.minMaxBins;
        std::vector<uint32_t> mins(B), maxs(B);
        for (int axis = 0; axis < 3; ++axis) {
            float lo = box.mn[axis], hi = box.mx[axis];
            if (hi <= lo) continue;
            float w = (hi - lo) / B, invW = B / (hi - lo);
            std::fill(mins.begin(), mins.end(), 0);
            std::fill(maxs.begin(), maxs.end(), 0);
            for (const BPrim &p : prims) {
                int a = std::min(B - 1, std::max(0, (int)((p.lo[axis] - lo) * invW)));
                int b = std::min(B - 1, std::max(0, (int)((p.hi[axis] - lo) * invW)));
                mins[a]++;
                maxs[b]++;
            }
            size_t nL = 0, nR = prims.size();
            for (int k = 1; k < B; ++k) {
                nL += mins[k - 1];
                nR -= maxs[k - 1];
                float pos = lo + w * k;
                float c = cost(box, axis, pos, nL, nR);
                if (c < best.cost) { best.cost = c; best.axis = axis; best.pos = pos; best.planarLeft = true; }
            }
        }
        return best;
    }

    void clipInto(const BPrim &p, const AABB &childBox, std::vector<BPrim> &out) const {
        bool inside = true;
        for (int a = 0; a < 3; ++a)
            if (p.lo[a] < childBox.mn[a] || p.hi[a] > childBox.mx[a]) inside = false;
        if (inside || !P.clip) {
            BPrim q = p;
            for (int a = 0; a < 3; ++a) { q.lo[a] = std::max(q.lo[a], childBox.mn[a]); q.hi[a] = std::min(q.hi[a], childBox.mx[a]); }
            out.push_back(q);
            return;
        }
        AABB c = src.clippedBounds(p.id, childBox);
        BPrim q;
        q.id = p.id;
        if (c.valid()) {
            for (int a = 0; a < 3; ++a) { q.lo[a] = c.mn[a]; q.hi[a] = c.mx[a]; }
        } else {
            // numerical corner case: keep the conservative overlap box
            for (int a = 0; a < 3; ++a) { q.lo[a] = std::max(p.lo[a], childBox.mn[a]); q.hi[a] = std::min(p.hi[a], childBox.mx[a]); }
            if (q.lo[0] > q.hi[0] || q.lo[1] > q.hi[1] || q.lo[2] > q.hi[2]) return;
        }
        out.push_back(q);
    }

    void makeLeaf(Sub &s, uint32_t slot, const std::vector<BPrim> &prims, int depth) {
        uint32_t start = (uint32_t)s.indices.size();
        for (const BPrim &p : prims) s.indices.push_back(p.id);
        s.nodes[slot].combined = 0x80000000u | start;
        s.nodes[slot].data = start + (uint32_t)prims.size();
        s.maxDepth = std::max<uint32_t>(s.maxDepth, depth);
        s.leaves++;
        if (!prims.empty()) s.nonEmpty++;
    }

    struct Job {
        AABB box;
        std::vector<BPrim> prims;
        int depth, badRefines;
        uint32_t slot;   // node slot in the parent Sub
        Sub result;
    };

    // Build subtree rooted at s.nodes[slot]; large nodes become jobs when
    // `jobs` is non-null.  Returns the subtree's SAH cost (buildTreeMinMax /
    // buildTree return values, gkdtree.h:1792-1923); a split whose final cost
    // is not below the leaf cost is retracted into a leaf of the node's
    // primitives (gkdtree.h:1910-1922).  Subtrees deferred to parallel jobs
    // report their split estimate and are never retracted (nodes of that size
    // always pay for their split).
    float build(Sub &s, uint32_t slot, const AABB &box, std::vector<BPrim> &prims, int depth,
                int badRefines, std::vector<std::unique_ptr<Job>> *jobs) {
        size_t N = prims.size();
        float leafCost = (float)N * P.queryCost;
        if ((int)N <= P.stopPrims || depth >= maxDepth) { makeLeaf(s, slot, prims, depth); return leafCost; }
        if (jobs && N <= parallelCut) {
            auto j = std::make_unique<Job>();
            j->box = box; j->prims = std::move(prims); j->depth = depth; j->badRefines = badRefines; j->slot = slot;
            jobs->push_back(std::move(j));
            return leafCost;
        }
        Split sp = N <= (size_t)P.exactSweepLimit ? findExact(box, prims) : findBinned(box, prims);
        if (sp.axis < 0) { makeLeaf(s, slot, prims, depth); return leafCost; }
        if (sp.cost >= leafCost) {
            if ((sp.cost > 4 * leafCost && N < 16) || badRefines >= P.maxBadRefines) { makeLeaf(s, slot, prims, depth); return leafCost; }
            ++badRefines;
        }
        AABB lb = box, rb = box;
        lb.mx[sp.axis] = sp.pos;
        rb.mn[sp.axis] = sp.pos;
        std::vector<BPrim> L, R;
        L.reserve(N / 2 + 16);
        R.reserve(N / 2 + 16);
        int ax = sp.axis;
        for (const BPrim &p : prims) {
            if (p.lo[ax] == p.hi[ax] && p.lo[ax] == sp.pos) {
                (sp.planarLeft ? L : R).push_back(p);
            } else {
                bool goL = p.lo[ax] < sp.pos, goR = p.hi[ax] > sp.pos;
                if (goL && goR) { clipInto(p, lb, L); clipInto(p, rb, R); }
                else if (goL) L.push_back(p);
                else R.push_back(p);
            }
        }
        std::vector<BPrim>().swap(prims);
        const size_t jobsBefore = jobs ? jobs->size() : 0;
        const uint32_t c = (uint32_t)s.nodes.size();
        const size_t indexStart = s.indices.size(), leavesBefore = s.leaves, nonEmptyBefore = s.nonEmpty;
        const uint32_t depthBefore = s.maxDepth;
        s.nodes.push_back({0, 0});
        s.nodes.push_back({0, 0});
        uint32_t rel = c - slot;
        uint32_t split;
        memcpy(&split, &sp.pos, 4);
        s.nodes[slot].combined = (uint32_t)ax | (rel << 2);
        s.nodes[slot].data = split;
        const float leftCost = build(s, c, lb, L, depth + 1, badRefines, jobs);
        const float rightCost = build(s, c + 1, rb, R, depth + 1, badRefines, jobs);
        float pL, pR;
        probs(box, ax, sp.pos, pL, pR);
        const float finalCost = P.traversalCost + (pL * leftCost + pR * rightCost);
        const bool deferred = jobs && jobs->size() != jobsBefore;
        if (!P.retract || deferred || finalCost < leafCost) return finalCost;
        // retraction: tear up the subtree, one leaf with its unique primitives
        std::vector<uint32_t> ids(s.indices.begin() + indexStart, s.indices.end());
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
        s.nodes.resize(c);
        s.indices.resize(indexStart);
        s.leaves = leavesBefore;
        s.nonEmpty = nonEmptyBefore;
        s.maxDepth = depthBefore;
        s.retracted++;
        std::vector<BPrim> leaf(ids.size());
        for (size_t i = 0; i < ids.size(); ++i) leaf[i].id = ids[i];
        makeLeaf(s, slot, leaf, depth);
        return leafCost;
    }
};

}  // namespace

void buildKDTree(const PrimSource &src, const KDBuildParams &params, KDTree &out) {
    auto t0 = std::chrono::steady_clock::now();
    size_t N = src.count();
    out = KDTree();
    AABB box;
    std::vector<BPrim> prims;
    prims.reserve(N);
    for (size_t i = 0; i < N; ++i) {
        AABB b = src.bounds(i);
        if (!b.valid()) continue;
        BPrim p;
        p.id = (uint32_t)i;
        for (int a = 0; a < 3; ++a) { p.lo[a] = b.mn[a]; p.hi[a] = b.mx[a]; }
        prims.push_back(p);
        box.expand(b);
    }
    if (prims.empty()) {
        box.mn = V3(0.0f); box.mx = V3(0.0f);
    }
    int maxDepth = params.maxDepth > 0 ? params.maxDepth
                                       : (int)(8 + 1.3f * std::log2((float)std::max<size_t>(N, 1)) + 0.5f);
    maxDepth = std::min(maxDepth, 48);   // MTS_KD_MAXDEPTH (gkdtree.h:37)
    unsigned threads = params.threads > 0 ? (unsigned)params.threads : std::max(1u, std::thread::hardware_concurrency());
    size_t cut = std::max<size_t>(4096, prims.size() / (8 * threads));
    Builder b(src, params, maxDepth, cut);

    Sub top;
    top.nodes.push_back({0, 0});
    std::vector<std::unique_ptr<Builder::Job>> jobs;
    b.build(top, 0, box, prims, 0, 0, threads > 1 ? &jobs : nullptr);

    // run subtree jobs in parallel (largest first)
    std::sort(jobs.begin(), jobs.end(), [](const auto &x, const auto &y) { return x->prims.size() > y->prims.size(); });
    std::atomic<size_t> next{0};
    std::vector<std::thread> pool;
    std::mutex errMu;
    std::string errMsg;
    for (unsigned t = 0; t < std::min<size_t>(threads, jobs.size()); ++t)
        pool.emplace_back([&]() {
            try {
                for (;;) {
                    size_t j = next.fetch_add(1);
                    if (j >= jobs.size()) break;
                    auto &job = *jobs[j];
                    job.result.nodes.push_back({0, 0});
                    b.build(job.result, 0, job.box, job.prims, job.depth, job.badRefines, nullptr);
                }
            } catch (const std::exception &e) {
                std::lock_guard<std::mutex> g(errMu);
                errMsg = e.what();
            }
        });
    for (auto &t : pool) t.join();
    if (!errMsg.empty()) throw std::runtime_error(errMsg);

    // stitch: subtree root goes to its reserved slot, the rest is appended
    out.nodes = std::move(top.nodes);
    out.indices = std::move(top.indices);
    out.maxDepth = top.maxDepth;
    out.leafCount = top.leaves;
    out.nonEmptyLeaves = top.nonEmpty;
    out.retractedSplits = top.retracted;
    for (auto &jp : jobs) {
        Sub &s = jp->result;
        uint32_t base = (uint32_t)out.nodes.size();
        uint32_t ibase = (uint32_t)out.indices.size();
        out.indices.insert(out.indices.end(), s.indices.begin(), s.indices.end());
        auto fix = [&](mtsg_kdnode n) {
            if (n.combined & 0x80000000u) {
                uint32_t st = (n.combined & 0x7FFFFFFFu) + ibase;
                n.data += ibase;
                n.combined = 0x80000000u | st;
            }
            return n;
        };
        for (size_t k = 1; k < s.nodes.size(); ++k) out.nodes.push_back(fix(s.nodes[k]));
        mtsg_kdnode root = fix(s.nodes[0]);
        if (!(root.combined & 0x80000000u)) {
            uint32_t childSub = root.combined >> 2;             // index in s (root at 0)
            uint32_t childFinal = base + childSub - 1;
            uint32_t rel = childFinal - jp->slot;
            if (rel > (1u << 28) - 1) throw std::runtime_error("kd-tree too large for relative offsets");
            root.combined = (root.combined & 3u) | (rel << 2);
        }
        out.nodes[jp->slot] = root;
        out.maxDepth = std::max(out.maxDepth, s.maxDepth);
        out.leafCount += s.leaves;
        out.nonEmptyLeaves += s.nonEmpty;
        out.retractedSplits += s.retracted;
    }
    if (out.nodes.size() >= (1u << 28)) throw std::runtime_error("kd-tree has too many nodes");

    // SAH cost of the final tree (informational)
    out.tightAABB = box;
    AABB e = box;
    const float eps = 1e-3f;   // MTS_KD_AABB_EPSILON, gkdtree.h:1213-1220
    V3 ext = e.mx - e.mn;
    e.mn = e.mn - ext * eps - V3(eps);
    e.mx = e.mx + (e.mx - e.mn) * eps + V3(eps);
    out.aabb = e;
    out.buildSeconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace mtsh
