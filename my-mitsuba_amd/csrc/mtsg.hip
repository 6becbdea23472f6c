// mtsg.hip -- MI355X (gfx950, CDNA4) wavefront unidirectional path tracer
// behind the C-ABI in include/mtsg.h.
//
// Replaces, for the `path` plugin, the reference's per-sample CPU loop
//   SamplingIntegrator::renderBlock   src/librender/integrator.cpp:144-197
//   MIPathTracer::Li                  src/integrators/path/path.cpp:119-294
//   ShapeKDTree::rayIntersect         src/librender/skdtree.cpp:112-226
//   SAHKDTree3D::rayIntersectHavran   include/mitsuba/render/sahkdtree3.h:178-308
//   TriAccel::rayIntersect            include/mitsuba/render/triaccel.h:96-158
//   diffuse / roughconductor / dielectric sample, eval, pdf
//   AreaLight + Scene::sampleEmitterDirect / pdfEmitterDirect
//   ImageBlock::put                   include/mitsuba/render/imageblock.h:124-204
// with a wavefront of SoA path states in HBM:
//   k_camera -> [ k_trace_closest -> k_shade -> k_trace_shadow ] x bounces -> k_splat
// Active paths are compacted into queues with wave-aggregated atomics
// (__ballot / __popcll / mbcnt on 64-lane waves); the kd-tree traversal
// keeps a short stack in LDS (kd-restart on overflow); the film is splatted
// per 16x16 tile into LDS and flushed with one float atomic per texel.
// No MFMA: the path has no dense contraction.  See DESIGN.md.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>
#include <chrono>
#include <functional>

#include "../../include/mtsg.h"
#include "device_math.h"
#include "envmap.h"
#include "sampler.h"

#include "kernels.h"

namespace {

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
thread_local std::string g_err;

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess) {                                                        \
            g_err = std::string(#expr) + ": " + hipGetErrorString(_e);                 \
            return _e == hipErrorOutOfMemory ? MTSG_ERR_OOM : MTSG_ERR_DEVICE;         \
        }                                                                              \
    } while (0)

template <class T>
int upload(const T *src, size_t n, T **dst) {
    *dst = nullptr;
    if (n == 0) return MTSG_OK;
    HIP_TRY(hipMalloc((void **)dst, n * sizeof(T)));
    HIP_TRY(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
    return MTSG_OK;
}

}  // namespace

struct mtsg_scene {
    int device = 0;
    mtsg_tile_fn tileFn = nullptr;   // tile completion (mtsg_set_tile_callback)
    void *tileUser = nullptr;
    hipStream_t stream = nullptr;
    DevScene ds{};
    DevCamera cam{};
    std::vector<void *> allocs;
    // batch buffers
    uint32_t capacity = 0;         // paths per batch (per lane)
    uint32_t requestedBatch = 0;   // paths in flight over all lanes
    int lanes = MTSG_LANES;        // concurrent batches (streams) of a render
    int stagger = 0;               // bounces between the starts of consecutive lanes
    int lanesAlloc = 0;            // lanes with path state allocated
    hipStream_t lstream[MTSG_MAX_LANES] = {};   // lstream[0] == stream
    // mtsg_set_tile_list: the deal keys a render call takes (empty: tile_stride / tile_offset)
    std::vector<int32_t> tileKeys;
    int32_t *tileKeysDev = nullptr;
    size_t tileKeysCap = 0;
    DevPaths LP[MTSG_MAX_LANES]{};
    std::vector<void *> batchAllocs;
    uint32_t *hostCnt = nullptr;   // pinned copy of the queue counters (2 per lane)
    int cuCount = 0;
    int traceGrid = 0, shadeGrid = 0, traceGridInst = 0, finishGrid = 0, finishGridMats = 0;
    // tail mode: once a bounce starts with fewer than finishPaths paths, k_finish
    // carries them through their remaining bounces in one launch (0: off)
    uint32_t finishPaths = 0;
    // a tail-kernel wave shades once 16 of its busy lanes wait to (or none traces):
    // r06, with the 4-wave material kernels, C5 tail 18.3 -> 13.4 ms, C3 0.66 ->
    // 0.58, two-level 1.16 -> 0.99 against 1 (profiles/r06_finish_threshold.txt)
    uint32_t finishShadeMin = 16;
    uint32_t flags = 0;
    int samplerType = MTSG_SAMPLER_INDEPENDENT, samplerDim = 4;
    int qmcInv[2][3] = {{0, 0, 0}, {0, 0, 0}};
    int traceMode = 0;            // 0: refill at 16 idle lanes (measured best), 1: at 32
    // camera ray differentials (DevScene::cam_diffs / cam_env_diffs): stored
    // in the path state for filtered textures (or MTSG_OPT_CAMERA_DIFFS 1),
    // else recomputed at bounce 0 for environment misses
    bool texDiffs = false, hasEnvmap = false, storeCamDiffs = false;
    int rayOrder = 0;             // MTSG_OPT_RAY_ORDER: 1 = bounce rays sorted per window by direction (k_sortwin;
                                  // measured r06: C3 trace +6.7 ms, profiles/r06_ray_order.txt)
    float *dumpL = nullptr;
    std::atomic<int> cancel{0};
    bool knobs = false;   // traversal test overrides set (mtsg_set_test_knobs): KNOBS kernels, no tail mode
    mtsg_stats stats{};
    std::vector<hipEvent_t> evPool;
    size_t evUsed = 0;
    std::vector<std::pair<int, size_t>> timed;   // (kind, event index)
    std::vector<unsigned long long> stragglers;  // MTSG_FLAG_COUNT: slow-ray records
    unsigned long long *waveTimes = nullptr;     // MTSG_FLAG_WAVETIME: [launch][wave][WT_WORDS]
    uint32_t wtLaunches = 0;
    bool extBsdfs = false;   // conductor / plastic / twosided records or textures present (k_shade<..., true>)
    int mats = MATS_ALL;     // material classes of the scene's records (k_shade<..., MATS>)
    bool shadeGeneric = false;   // MTSG_OPT_SHADE_GENERIC: the all-materials kernel (A/B tests)
    uint32_t nTextures = 0;
    const uint32_t *sobolM = nullptr;        // sobol sampler tables (device)
    const uint64_t *sobolVdc = nullptr, *sobolVdcInv = nullptr;
    uint64_t sobolScramble = 0;
};

namespace {

int set_device(mtsg_scene *s) {
    HIP_TRY(hipSetDevice(s->device));
    return MTSG_OK;
}

void free_batch(mtsg_scene *s) {
    for (void *p : s->batchAllocs) hipFree(p);
    s->batchAllocs.clear();
    s->capacity = 0;
    s->lanesAlloc = 0;
}

int ensure_batch(mtsg_scene *s, uint32_t paths, int lanes) {
    if (s->capacity >= paths && s->lanesAlloc >= lanes) return MTSG_OK;
    paths = std::max(paths, s->capacity);
    lanes = std::max(lanes, s->lanesAlloc);
    free_batch(s);
    auto alloc = [&](size_t bytes, void **p) -> int {
        HIP_TRY(hipMalloc(p, bytes));
        s->batchAllocs.push_back(*p);
        return MTSG_OK;
    };
    size_t n = paths;
    int rc = MTSG_OK;
    for (int l = 0; l < lanes; ++l) {
    DevPaths &P = s->LP[l];
#define A(field, T) if ((rc = alloc(n * sizeof(T), (void **)&P.field)) != MTSG_OK) return rc
    A(ray_o, float4); A(ray_d, float4); A(T, float4); A(aux, float4); A(Lp, float4); A(meta, uint4);
    A(n_ray_o, float4); A(n_ray_d, float4); A(n_T, float4); A(n_aux, float4); A(n_Lp, float4); A(n_meta, uint4);
    A(hit, float4); A(L, float4); A(sh_o, float4); A(sh_d, float4); A(sh_c, float4);
    if (s->ds.inst) { A(hitInst, uint32_t); } else P.hitInst = nullptr;
    A(tie, uint32_t);
    A(orderBuf, uint32_t);
    P.order = nullptr;
#undef A
    if ((rc = alloc(CNT_WORDS * sizeof(uint32_t), (void **)&P.cnt)) != MTSG_OK) return rc;
    if ((rc = alloc(CTR_WORDS * sizeof(unsigned long long), (void **)&P.ctr)) != MTSG_OK) return rc;
    HIP_TRY(hipMemset(P.ctr, 0, CTR_WORDS * sizeof(unsigned long long)));
    }
    s->capacity = paths;
    s->lanesAlloc = lanes;
    return MTSG_OK;
}

enum { K_CAMERA = 0, K_CLOSEST, K_SHADOW, K_SHADE, K_SPLAT, K_FINISH, K_SORT };

// the survivors k_shade compacted into n_* are the next bounce's paths
void swap_bounce(DevPaths &P) {
    std::swap(P.ray_o, P.n_ray_o);
    std::swap(P.ray_d, P.n_ray_d);
    std::swap(P.T, P.n_T);
    std::swap(P.aux, P.n_aux);
    std::swap(P.Lp, P.n_Lp);
    std::swap(P.meta, P.n_meta);
}

hipEvent_t next_event(mtsg_scene *s) {
    if (s->evUsed == s->evPool.size()) {
        hipEvent_t e;
        hipEventCreate(&e);
        s->evPool.push_back(e);
    }
    return s->evPool[s->evUsed++];
}

// bracket a launch with events when timing is enabled
template <class F>
void timed_launch(mtsg_scene *s, int kind, hipStream_t st, F f) {
    if (!(s->flags & MTSG_FLAG_TIMING)) { f(); return; }
    size_t i0 = s->evUsed;
    hipEventRecord(next_event(s), st);
    f();
    hipEventRecord(next_event(s), st);
    s->timed.emplace_back(kind, i0);
}

// One traversal launch over a work list (see k_trace_s): closest rays cIn,
// shadow rays sIn.  traceMode 1 refills lanes at 32 idle lanes instead of 16
// (MTSG_TRACE_MODE, for measurement).
template <bool COUNT>
void launch_trace_c(mtsg_scene *s, const DevPaths &P, int cIn, int sIn, uint32_t n, hipStream_t st) {
    dim3 g(s->traceGrid), blk(TRACE_BLOCK);
    unsigned long long *wt = nullptr;
    if ((s->flags & MTSG_FLAG_WAVETIME) && s->waveTimes && s->wtLaunches < WT_MAX_LAUNCHES && !s->ds.inst)
        wt = s->waveTimes + (size_t)WT_WORDS * s->traceGrid * s->wtLaunches++;
    // the KNOBS instantiations read the stack caps and restart limits the
    // scene was created with (test overrides); the COUNT pass ignores them
    // closest rays that met an exact tie: traced again with the mailbox
    // (a grid a quarter of the trace grid's; two-level: the exact Havran).
    // The flat traversal retraces them inside its own launch (TIE_INLINE).
    const dim3 tg(std::max<unsigned>(1u, (unsigned)s->traceGrid / 4u));
    if (!s->ds.inst) {   // the flat kernels: trace_flat.hip
        FlatTraceLaunch a{g, tg, st, &s->ds, &P, cIn, sIn, n, wt, COUNT, s->knobs, s->traceMode == 1,
                          MTSG_MAILBOX && cIn != -2 && !TIE_INLINE};
        launch_trace_flat(a);
        return;
    }
    if (s->knobs && !COUNT)
        hipLaunchKernelGGL((k_trace_s<false, MTSG_INST_MIN_IDLE, true, true>), dim3(s->traceGridInst), blk, 0, st, s->ds, P, cIn, sIn, n, wt);
    else hipLaunchKernelGGL((k_trace_s<COUNT, MTSG_INST_MIN_IDLE, true>), dim3(s->traceGridInst), blk, 0, st, s->ds, P, cIn, sIn, n, wt);
    if (MTSG_MAILBOX && cIn != -2) hipLaunchKernelGGL(k_tie_i, tg, blk, 0, st, s->ds, P);
}
void launch_trace(mtsg_scene *s, bool count, const DevPaths &P, int cIn, int sIn, uint32_t n, hipStream_t st) {
    if (count) launch_trace_c<true>(s, P, cIn, sIn, n, st);
    else launch_trace_c<false>(s, P, cIn, sIn, n, st);
}

// k_shade / k_finish are instantiated per sampler in smp_kernels.hip
ShadeLaunch shade_args(mtsg_scene *s, const DevIntegrator &I, const DevBatch &B, const DevPaths &P, int b, int qin, hipStream_t st,
                       dim3 grid, dim3 block) {
    ShadeLaunch a;
    a.grid = grid;
    a.block = block;
    a.stream = st;
    a.S = &s->ds;
    a.I = &I;
    a.B = &B;
    a.P = &P;
    a.bounce = b;
    a.qin = qin;
    a.nIdentity = B.nslots;
    a.hasAlpha = s->cam.has_alpha;
    a.shadeMin = s->finishShadeMin;
    a.env = s->ds.has_env != 0;
    a.ext = s->extBsdfs;
    a.inst = s->ds.inst != nullptr;
    a.mats = s->shadeGeneric ? (int)MATS_ALL : s->mats;
    return a;
}
// where bounce 0 finds the camera rays' differentials (mtsg_scene::storeCamDiffs)
void camera_diff_mode(mtsg_scene *s) {
    s->ds.cam_diffs = (s->texDiffs || (s->hasEnvmap && s->storeCamDiffs)) ? 1 : 0;
    s->ds.cam_env_diffs = (s->hasEnvmap && !s->ds.cam_diffs) ? 1 : 0;
    s->cam.diffs = s->ds.cam_diffs;
}
void launch_shade(mtsg_scene *s, const DevIntegrator &I, const DevBatch &B, const DevPaths &P, int b, int qin, hipStream_t st) {
    const ShadeLaunch a = shade_args(s, I, B, P, b, qin, st, dim3(s->shadeGrid), dim3(SHADE_BLOCK));
    switch (I.smp.type) {
        case MTSG_SAMPLER_HALTON: launch_shade_smp<MTSG_SAMPLER_HALTON>(a); break;
        case MTSG_SAMPLER_HAMMERSLEY: launch_shade_smp<MTSG_SAMPLER_HAMMERSLEY>(a); break;
        case MTSG_SAMPLER_LDSAMPLER: launch_shade_smp<MTSG_SAMPLER_LDSAMPLER>(a); break;
        case MTSG_SAMPLER_SOBOL: launch_shade_smp<MTSG_SAMPLER_SOBOL>(a); break;
        default: launch_shade_smp<MTSG_SAMPLER_INDEPENDENT>(a);
    }
}
void launch_finish(mtsg_scene *s, const DevIntegrator &I, const DevBatch &B, const DevPaths &P, int qin, hipStream_t st) {
    const bool mats = finish_uses_mats(I.smp.type, s->extBsdfs, s->ds.inst != nullptr, s->shadeGeneric ? (int)MATS_ALL : s->mats);
    const ShadeLaunch a = shade_args(s, I, B, P, 1, qin, st, dim3(mats ? s->finishGridMats : s->finishGrid), dim3(TRACE_BLOCK));
    switch (I.smp.type) {
        case MTSG_SAMPLER_HALTON: launch_finish_smp<MTSG_SAMPLER_HALTON>(a); break;
        case MTSG_SAMPLER_HAMMERSLEY: launch_finish_smp<MTSG_SAMPLER_HAMMERSLEY>(a); break;
        case MTSG_SAMPLER_LDSAMPLER: launch_finish_smp<MTSG_SAMPLER_LDSAMPLER>(a); break;
        case MTSG_SAMPLER_SOBOL: launch_finish_smp<MTSG_SAMPLER_SOBOL>(a); break;
        default: launch_finish_smp<MTSG_SAMPLER_INDEPENDENT>(a);
    }
}

// Sampler constants of a render (setFilmResolution with blocked = true over
// the film's crop size: halton.cpp:240-271, hammersley.cpp:181-200)
DevSampler make_sampler(const mtsg_scene *s, uint32_t spp) {
    DevSampler S{};
    S.type = s->samplerType;
    S.ldDim = s->samplerDim;
    while ((1u << S.ldBits) < spp) ++S.ldBits;
    S.stride = 1;
    S.primes = s->ds.qmcPrimes;
    S.off = s->ds.qmcOff;
    S.perm = s->ds.qmcPerm;
    S.sobolM = s->sobolM;
    S.vdc = s->sobolVdc;
    S.vdcInv = s->sobolVdcInv;
    S.sobolScramble = s->sobolScramble;
    S.logRes = 0;
    S.sobolRes = 1.0f;
    if (S.type == MTSG_SAMPLER_SOBOL) {
        // setFilmResolution(crop size, bucketed = true) (sobol.cpp:147-158)
        uint32_t r = 1;
        while (r < (uint32_t)std::max(s->cam.crop_w, s->cam.crop_h)) r <<= 1;
        S.sobolRes = (float)r;
        while ((1u << (S.logRes + 1)) <= r) ++S.logRes;
    }
    for (int b = 0; b < 2; ++b)
        for (int j = 0; j < 3; ++j) S.inv[b][j] = (uint16_t)s->qmcInv[b][j];
    const int crop[2] = {s->cam.crop_w, s->cam.crop_h};
    if (S.type == MTSG_SAMPLER_HALTON) {
        const uint32_t primes[2] = {2, 3};
        for (int i = 0; i < 2; ++i) {
            uint32_t value = 1, e = 0;
            while ((int)value < std::min(crop[i], 128)) { value *= primes[i]; ++e; }
            S.primePow[i] = value;
            S.primeExp[i] = e;
            S.stride *= value;
        }
        // multiplicativeInverse (halton.cpp:211-234)
        auto inv = [](int64_t a, int64_t n) {
            int64_t t = 0, nt = 1, r = n, nr = a % n;
            while (nr) { int64_t q = r / nr; std::swap(t, nt); nt -= q * t; std::swap(r, nr); nr -= q * r; }
            return (uint32_t)(t < 0 ? t + n : t);
        };
        S.multInv[0] = S.primePow[0] > 1 ? inv(S.primePow[1], S.primePow[0]) : 0;
        S.multInv[1] = S.primePow[1] > 1 ? inv(S.primePow[0], S.primePow[1]) : 0;
    } else if (S.type == MTSG_SAMPLER_HAMMERSLEY) {
        for (int i = 0; i < 2; ++i) {
            uint32_t r = 1;
            while (r < (uint32_t)crop[i]) r <<= 1;
            S.res[i] = std::min<uint32_t>(128, r);
        }
        S.logH = 0;
        while ((1u << (S.logH + 1)) <= S.res[1]) ++S.logH;
        S.factor = 1.0f / (float)((size_t)spp * S.res[0] * S.res[1]);
        S.stride = S.res[1];
    }
    return S;
}

const char *const traversal_error =
    "kd-tree traversal: a ray reached the restart limit without making progress (kernels.h kd_restart)";
// Mitsuba's Log(EError) of Halton/Hammersley (halton.cpp:343-386) and sobol (sobol.cpp:223-239)
const char *dim_error(int sampler) {
    return sampler == MTSG_SAMPLER_SOBOL
               ? "Lookup dimension exceeds the direction number table size! You may have to reduce the 'maxDepth' parameter of your integrator."
               : "Lookup dimension exceeds the prime number table size! You may have to reduce the 'maxDepth' parameter of your integrator.";
}

int validate(const mtsg_render_params *p, const mtsg_scene *s) {
    if (!p) { g_err = "null params"; return MTSG_ERR_INVALID; }
    if (p->spp == 0) { g_err = "spp must be > 0"; return MTSG_ERR_INVALID; }
    if (s->samplerType == MTSG_SAMPLER_LDSAMPLER && (p->spp & (p->spp - 1))) {
        g_err = "ldsampler: the sample count must be a power of two";
        return MTSG_ERR_INVALID;
    }
    if (p->rr_depth <= 0) { g_err = "'rrDepth' must be set to a value greater than zero!"; return MTSG_ERR_INVALID; }
    if (p->max_depth <= 0 && p->max_depth != -1) { g_err = "'maxDepth' must be set to -1 (infinite) or a value greater than zero!"; return MTSG_ERR_INVALID; }
    if (p->tile_w <= 0 || p->tile_h <= 0 || p->tile_x < 0 || p->tile_y < 0 ||
        p->tile_x + p->tile_w > s->cam.film_w || p->tile_y + p->tile_h > s->cam.film_h) {
        g_err = "tile rectangle outside the film";
        return MTSG_ERR_INVALID;
    }
    if (p->tile_stride < 0 || (p->tile_stride > 1 && (p->tile_offset < 0 || p->tile_offset >= p->tile_stride))) {
        g_err = "invalid tile_stride / tile_offset";
        return MTSG_ERR_INVALID;
    }
    if (p->integrator != MTSG_INTEGRATOR_PATH && p->integrator != MTSG_INTEGRATOR_PATH2_OM) { g_err = "unknown integrator"; return MTSG_ERR_INVALID; }
    if (p->integrator == MTSG_INTEGRATOR_PATH2_OM) {
        if (!s->ds.om) { g_err = "myPath2_OM: the scene has no occupancy maps"; return MTSG_ERR_INVALID; }
        if (s->samplerType != MTSG_SAMPLER_INDEPENDENT) { g_err = "myPath2_OM: only the independent sampler is supported"; return MTSG_ERR_INVALID; }
        if (p->max_depth < 1) { g_err = "myPath2_OM: 'maxDepthEye' must be at least 1"; return MTSG_ERR_INVALID; }
        if (p->om_strategy < MTSG_OM_STRATEGY_BSDF || p->om_strategy > MTSG_OM_STRATEGY_MIS || p->om_mis < MTSG_OM_MIS_UNIFORM ||
            p->om_mis > MTSG_OM_MIS_POWER) {
            g_err = "myPath2_OM: unknown strategy or MIS mode";
            return MTSG_ERR_INVALID;
        }
    }
    return MTSG_OK;
}

// win = 0: film is the ImageBlock of the whole rectangle + border; win > 0:
// film holds one win x win window per tile of this call (mtsg_render_device_tiles)
int render_impl(mtsg_scene *s, const mtsg_render_params *p, float *film, int win = 0) {
    int rc;
    if ((rc = validate(p, s)) != MTSG_OK) return rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    auto t0 = std::chrono::steady_clock::now();
    const bool count = (s->flags & MTSG_FLAG_COUNT) != 0;
    uint32_t maxPaths = s->requestedBatch ? s->requestedBatch : DEFAULT_BATCH_PATHS;
    if (!s->requestedBatch) {
        size_t freeB = 0, totalB = 0;
        if (hipMemGetInfo(&freeB, &totalB) == hipSuccess) {
            const size_t held = (size_t)s->capacity * s->lanesAlloc * PATH_STATE_BYTES;
            // 3/4 of the free HBM (288 GB on an MI355X: 768M paths, C5's three
            // batches of 713M); the rest stays for the scene and other users
            const size_t fit = (size_t)((freeB + held) * 0.75 / PATH_STATE_BYTES);
            maxPaths = (uint32_t)std::max<size_t>(TILE * TILE, std::min<size_t>(maxPaths, fit));
        }
    }
    if (s->dumpL && (uint64_t)p->tile_w * p->tile_h * p->spp > maxPaths) { g_err = "render_samples: tile does not fit one batch"; return MTSG_ERR_INVALID; }
    const uint32_t tilesX = (uint32_t)(p->tile_w + TILE - 1) / TILE, tilesY = (uint32_t)(p->tile_h + TILE - 1) / TILE;
    const uint32_t allTiles = tilesX * tilesY;
    const uint32_t tstride = p->tile_stride > 1 ? (uint32_t)p->tile_stride : 1u;
    const uint32_t toffset = p->tile_stride > 1 ? (uint32_t)p->tile_offset : 0u;
    const bool listed = !s->tileKeys.empty();
    const uint32_t ntiles = listed ? (uint32_t)s->tileKeys.size() : toffset < allTiles ? (allTiles - toffset + tstride - 1) / tstride : 0u;
    if (listed)
        for (int32_t k : s->tileKeys)
            if ((uint32_t)k >= allTiles) { g_err = "tile list: a deal key lies outside the rectangle's tiles"; return MTSG_ERR_INVALID; }
    // the deal key of virtual tile v, on the host
    auto hostKey = [&](int v) { return listed ? s->tileKeys[v] : (int)toffset + v * (int)tstride; };
    // Lanes: independent batches on their own streams, issued bounce by bounce
    // in lock step, so one lane's launch tail (its slowest rays) overlaps the
    // other lane's launch.  The debug and counting modes use one lane.
    const uint32_t nl = (s->dumpL || count || ntiles < 2) ? 1u : (uint32_t)s->lanes;
    const uint32_t lanePaths = std::max<uint32_t>(TILE * TILE, maxPaths / nl);
    const uint32_t sppPerBatch = std::max(1u, std::min(p->spp, lanePaths / (TILE * TILE)));
    // equal-sized batches, a multiple of the lane count: a nearly empty last
    // batch costs a full set of bounce launches (and their tails) for a
    // sliver of the work
    const uint32_t tilesMax = std::max(1u, lanePaths / (TILE * TILE * sppPerBatch));
    uint32_t nTileBatches = std::max(1u, (ntiles + tilesMax - 1) / tilesMax);
    nTileBatches = std::min(ntiles ? ntiles : 1u, (nTileBatches + nl - 1) / nl * nl);
    const uint32_t tilesPerBatch = std::max(1u, (ntiles + nTileBatches - 1) / nTileBatches);
    if ((rc = ensure_batch(s, tilesPerBatch * sppPerBatch * TILE * TILE, (int)nl)) != MTSG_OK) return rc;
    const int blockW = p->tile_w + 2 * s->cam.border, blockH = p->tile_h + 2 * s->cam.border;
    DevIntegrator I{p->max_depth, p->rr_depth, p->strict_normals, p->hide_emitters, p->spp, p->seed, (uint32_t)s->cam.film_w,
                    make_sampler(s, p->spp)};
    I.om = p->integrator == MTSG_INTEGRATOR_PATH2_OM ? 1 : 0;
    I.om_strategy = p->om_strategy;
    I.om_mis = p->om_mis;
    I.om_jitter = p->om_jitter;
    memset(&s->stats, 0, sizeof(s->stats));
    s->wtLaunches = 0;
    if ((s->flags & MTSG_FLAG_WAVETIME) && !s->waveTimes)
        HIP_TRY(hipMalloc((void **)&s->waveTimes, (size_t)WT_WORDS * s->traceGrid * WT_MAX_LAUNCHES * sizeof(unsigned long long)));
    s->evUsed = 0;
    s->timed.clear();
    // the cancel flag is consumed (cleared) when a render returns, so a
    // cancel that races with the start of a render is not lost
    if (count) HIP_TRY(hipMemsetAsync(s->LP[0].ctr, 0, CTR_WORDS * sizeof(unsigned long long), s->stream));
    // row rotation of the tile deal (include/mtsg.h): fixed at 1, as the
    // oracle, mtsg_tile_windows and mtsg.put_tile_windows assume (the round-3
    // measurement override is gone: a rank with another rotation would put
    // its tiles in the wrong places without an error)
    const int dealSkew = 1;
    // the batches of this call, tile-major
    std::vector<DevBatch> batches;
    for (uint32_t t0i = 0; t0i < ntiles; t0i += tilesPerBatch) {
        for (uint32_t s0 = 0; s0 < p->spp; s0 += sppPerBatch) {
            DevBatch B;
            B.rect_x = p->tile_x; B.rect_y = p->tile_y; B.rect_w = p->tile_w; B.rect_h = p->tile_h;
            B.tiles_x = (int)tilesX;
            B.skew = dealSkew;
            B.tile0 = (int)t0i;
            B.tstride = (int)tstride;
            B.toffset = (int)toffset;
            B.ntiles = (int)std::min(tilesPerBatch, ntiles - t0i);
            B.s0 = s0;
            B.ns = std::min(sppPerBatch, p->spp - s0);
            B.nslots = (uint32_t)B.ntiles * B.ns * TILE * TILE;
            B.keys = listed ? s->tileKeysDev : nullptr;
            batches.push_back(B);
        }
    }
    struct LaneRun {
        DevBatch B;
        int last = -1;
        int start = 0;
        bool open = false;
        bool finished = false;   // the tail kernel took over the batch's remaining bounces
        hipEvent_t cntEv[2] = {nullptr, nullptr};
    } lr[MTSG_MAX_LANES];
    int result = MTSG_OK;
    for (uint32_t l = 0; l < nl && result == MTSG_OK; ++l)
        for (int k = 0; k < 2; ++k)
            if (hipEventCreateWithFlags(&lr[l].cntEv[k], hipEventDisableTiming) != hipSuccess) { g_err = "event"; result = MTSG_ERR_DEVICE; }
    // work the caller queued on s->stream (the film memset of mtsg_render)
    // precedes every lane's first kernel
    hipEvent_t startEv = nullptr;
    if (result == MTSG_OK && nl > 1) {
        if (hipEventCreateWithFlags(&startEv, hipEventDisableTiming) != hipSuccess || hipEventRecord(startEv, s->stream) != hipSuccess) {
            g_err = "event";
            result = MTSG_ERR_DEVICE;
        }
        for (uint32_t l = 1; l < nl && result == MTSG_OK; ++l)
            if (hipStreamWaitEvent(s->lstream[l], startEv, 0) != hipSuccess) { g_err = "stream wait"; result = MTSG_ERR_DEVICE; }
    }
    // myPath2_OM shades depths 1..maxDepthEye and one more launch books the
    // emitters its last BSDF rays found
    const int maxBounces = I.om ? p->max_depth + 1 : (p->max_depth > 0 ? p->max_depth : 1 << 30);
    // tail mode (k_finish): one lane, not in the instrumented or myPath2_OM modes
    const bool useFinish = s->finishPaths > 0 && nl == 1 && !count && !I.om && !s->knobs;
    // bounce b of a lane: one trace launch over this bounce's closest rays
    // (work list qin(b), identity for b = 0) and bounce b-1's shadow rays
    // (S((b-1) & 1)), then k_shade appends the next bounce's paths to
    // qout(b) = (b & 1) ^ 1 and its shadow rays to S(b & 1)
    auto hostCnt = [&](uint32_t l, int bb) { return s->hostCnt + HOSTCNT_STRIDE * (2 * l + (bb & 1)); };
    auto account = [&](uint32_t l, int bb) {
        const uint32_t *hc = hostCnt(l, bb);
        const uint32_t consumed = bb == 0 ? lr[l].B.nslots : hc[(bb & 1) ? CNT_Q1 : CNT_Q0];
        s->stats.rays_closest += consumed;
        s->stats.rays_shadow += hc[cnt_s(bb & 1)];
        s->stats.launches_trace_closest++;
        return hc[((bb & 1) ^ 1) ? CNT_Q1 : CNT_Q0];
    };
    // every error inside the batch loop returns from `run`; the lanes are then
    // drained and the per-render events destroyed below, whatever happened
    auto run = [&]() -> int {
    for (size_t k0 = 0; k0 < batches.size(); k0 += nl) {
        if (s->cancel.load()) { g_err = "cancelled"; return MTSG_ERR_CANCELLED; }
        const uint32_t nb = (uint32_t)std::min<size_t>(nl, batches.size() - k0);
        for (uint32_t l = 0; l < nb; ++l) {
            LaneRun &L = lr[l];
            L.B = batches[k0 + l];
            L.last = -1;
            L.open = true;
            L.finished = false;
            // staggered lanes: lane l starts `stagger` bounces after lane
            // l-1, so its early, full launches overlap the other lanes'
            // late, tail-bound ones
            L.start = (int)l * s->stagger;
        }
        for (int gb = 0;; ++gb) {
            // cancel() between bounces (the whole frame is usually one batch)
            if (s->cancel.load()) { g_err = "cancelled"; return MTSG_ERR_CANCELLED; }
            bool any = false;
            for (uint32_t l = 0; l < nb; ++l) {
                LaneRun &L = lr[l];
                if (!L.open) continue;
                const int b = gb - L.start;
                if (b < 0) continue;
                DevPaths &P = s->LP[l];
                hipStream_t st = s->lstream[l];
                if (b == 0) {
                    HIP_TRY(hipMemsetAsync(P.cnt, 0, CNT_WORDS * sizeof(uint32_t), st));
                    timed_launch(s, K_CAMERA, st, [&]() {
                        hipLaunchKernelGGL(k_camera, dim3((L.B.nslots + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, s->cam, I, L.B, P);
                    });
                }
                const int qin = b == 0 ? -1 : (b & 1);
                const int qout = (b & 1) ^ 1;
                hipLaunchKernelGGL(k_reset, dim3(1), dim3(64), 0, st, P.cnt, qout, b & 1);
                // bounce rays in direction-sorted windows (k_sortwin); the
                // camera rays keep their tile order
                DevPaths PT = P;
                PT.camEnc = (b == 0 && s->ds.camCompact) ? 1u : 0u;   // bounce 0: camera rays as k_camera stores them
                if (b >= 1 && s->rayOrder == 1) {
                    timed_launch(s, K_SORT, st, [&]() {
                        hipLaunchKernelGGL(k_sortwin, dim3(s->cuCount * 2), dim3(SORT_BLOCK), 0, st, P, qin);
                    });
                    PT.order = P.orderBuf;
                }
                timed_launch(s, K_CLOSEST, st, [&]() { launch_trace(s, count, PT, qin, b == 0 ? -1 : ((b - 1) & 1), L.B.nslots, st); });
                if (useFinish && b >= 1) {
                    // the count of this bounce's paths is known once bounce b-1 is
                    // done (the GPU meanwhile runs this bounce's trace): few left ->
                    // k_finish carries them to their ends in one launch
                    HIP_TRY(hipEventSynchronize(L.cntEv[(b - 1) & 1]));
                    const uint32_t nb = account(l, b - 1);
                    if (nb < s->finishPaths) {
                        hipLaunchKernelGGL(k_reset, dim3(1), dim3(64), 0, st, P.cnt, -1, -1);
                        timed_launch(s, K_FINISH, st, [&]() { launch_finish(s, I, L.B, P, qin, st); });
                        s->stats.launches_finish++;
                        s->stats.paths_finish += nb;
                        HIP_TRY(hipMemcpyAsync(hostCnt(l, b), P.cnt, (CNT_S1 + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
                        HIP_TRY(hipEventRecord(L.cntEv[b & 1], st));
                        L.last = b;
                        L.open = false;
                        L.finished = true;
                        continue;
                    }
                }
                timed_launch(s, K_SHADE, st, [&]() { launch_shade(s, I, L.B, P, b, qin, st); });
                swap_bounce(P);
                HIP_TRY(hipMemcpyAsync(hostCnt(l, b), P.cnt, (CNT_S1 + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
                HIP_TRY(hipEventRecord(L.cntEv[b & 1], st));
                L.last = b;
                if (b + 1 >= maxBounces) L.open = false;
            }
            for (uint32_t l = 0; l < nb; ++l) {
                LaneRun &L = lr[l];
                const int b = gb - L.start;
                // lagged check: if bounce b-1 produced nothing, bounce b was empty
                // (also for a lane that launched its last bounce b just now, so
                // every bounce is booked once: b-1 here, the last one below)
                if (b >= 1 && L.last == b && !useFinish) {
                    HIP_TRY(hipEventSynchronize(L.cntEv[(b - 1) & 1]));
                    if (account(l, b - 1) == 0) L.open = false;
                }
                any |= L.open;
            }
            if (!any) break;
        }
        for (uint32_t l = 0; l < nb; ++l) {
            LaneRun &L = lr[l];
            DevPaths &P = s->LP[l];
            hipStream_t st = s->lstream[l];
            const DevBatch &B = L.B;
            if (L.last >= 0 && !L.finished) {
                // the last bounce's shadow rays
                hipLaunchKernelGGL(k_reset, dim3(1), dim3(64), 0, st, P.cnt, -1, -1);
                timed_launch(s, K_SHADOW, st, [&]() { launch_trace(s, count, P, -2, L.last & 1, 0u, st); });
                s->stats.launches_trace_shadow++;
                // the error word again, after this launch: a traversal error of
                // the last bounce's shadow rays fails the render too (the copy
                // of bounce L.last's counters was taken before this launch)
                HIP_TRY(hipMemcpyAsync(hostCnt(l, L.last) + CNT_ERR, P.cnt + CNT_ERR, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
                HIP_TRY(hipEventRecord(L.cntEv[L.last & 1], st));
            }
            timed_launch(s, K_SPLAT, st, [&]() {
                dim3 g(B.ntiles, (B.ns + SPLAT_CHUNK - 1) / SPLAT_CHUNK);
                const int K = 2 * s->cam.border + 1;
                if (K == 5 && !s->cam.has_alpha) hipLaunchKernelGGL((k_splat<5, 4>), g, dim3(BLOCK), 0, st, s->cam, I, B, P, film, blockW, blockH, win);
                else if (K == 5) hipLaunchKernelGGL((k_splat<5, 5>), g, dim3(BLOCK), 0, st, s->cam, I, B, P, film, blockW, blockH, win);
                else if (K <= 3 && !s->cam.has_alpha) hipLaunchKernelGGL((k_splat<3, 4>), g, dim3(BLOCK), 0, st, s->cam, I, B, P, film, blockW, blockH, win);
                else if (K <= 3) hipLaunchKernelGGL((k_splat<3, 5>), g, dim3(BLOCK), 0, st, s->cam, I, B, P, film, blockW, blockH, win);
                else if (!s->cam.has_alpha) hipLaunchKernelGGL((k_splat<9, 4>), g, dim3(BLOCK), 0, st, s->cam, I, B, P, film, blockW, blockH, win);
                else hipLaunchKernelGGL((k_splat<9, 5>), g, dim3(BLOCK), 0, st, s->cam, I, B, P, film, blockW, blockH, win);
            });
            s->stats.samples += (uint64_t)B.nslots;
        }
        for (uint32_t l = 0; l < nb; ++l) {
            LaneRun &L = lr[l];
            if (L.last < 0) continue;
            HIP_TRY(hipEventSynchronize(L.cntEv[L.last & 1]));
            account(l, L.last);
            // the error word is sticky within the batch: the last copy holds it
            const uint32_t err = hostCnt(l, L.last)[CNT_ERR];
            if (err & CNT_ERR_TRAVERSAL) {
                g_err = traversal_error;
                return MTSG_ERR_TRAVERSAL;
            }
            if (err) {
                g_err = dim_error(s->samplerType);
                return MTSG_ERR_INVALID;
            }
        }
        if (s->tileFn) {
            // the tiles whose last samples this batch splatted are complete
            for (uint32_t l = 0; l < nb; ++l) {
                HIP_TRY(hipStreamSynchronize(s->lstream[l]));
                const DevBatch &B = lr[l].B;
                if (B.s0 + B.ns < p->spp) continue;
                for (int tl = 0; tl < B.ntiles; ++tl) {
                    const int key = hostKey(B.tile0 + tl);
                    int tx, ty;
                    tile_of_key(key, B.tiles_x, tx, ty, B.skew);
                    const int x = tx * TILE, y = ty * TILE;
                    s->tileFn(s->tileUser, key, p->tile_x + x, p->tile_y + y, std::min(TILE, p->tile_w - x),
                              std::min(TILE, p->tile_h - y));
                }
            }
        }
        if (s->dumpL) {
            // debug: copy the batch's per-slot radiance (single batch, one lane)
            const DevBatch &B = lr[0].B;
            std::vector<float4> L(B.nslots);
            HIP_TRY(hipMemcpyAsync(L.data(), s->LP[0].L, B.nslots * sizeof(float4), hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(hipStreamSynchronize(s->stream));
            for (uint32_t slot = 0; slot < B.nslots; ++slot) {
                const uint32_t pix = slot & (TILE * TILE - 1), rest = slot >> 8;
                const uint32_t sl = rest % B.ns, tl = rest / B.ns;
                int tx, ty;
                tile_of_key(hostKey(B.tile0 + (int)tl), B.tiles_x, tx, ty, B.skew);
                int lx, ly;
                tile_pix(pix, lx, ly);
                const int x = tx * TILE + lx, y = ty * TILE + ly;
                if (x >= p->tile_w || y >= p->tile_h) continue;
                float *o = s->dumpL + (((size_t)y * p->tile_w + x) * p->spp + B.s0 + sl) * 4;
                o[0] = L[slot].x; o[1] = L[slot].y; o[2] = L[slot].z; o[3] = L[slot].w;
            }
        }
    }
    return MTSG_OK;
    };
    if (result == MTSG_OK) result = run();
    // drain every lane (also after an error or a cancel: the caller may free
    // the film as soon as this returns) and release the per-render events
    hipError_t e = hipSuccess;
    for (uint32_t l = 0; l < nl; ++l) {
        const hipError_t el = hipStreamSynchronize(s->lstream[l]);
        if (e == hipSuccess) e = el;
        for (int k = 0; k < 2; ++k)
            if (lr[l].cntEv[k]) hipEventDestroy(lr[l].cntEv[k]);
    }
    if (startEv) hipEventDestroy(startEv);
    s->cancel.store(0);
    if (e != hipSuccess) { g_err = std::string("render: ") + hipGetErrorString(e); return MTSG_ERR_DEVICE; }
    e = hipGetLastError();
    if (e != hipSuccess) { g_err = std::string("kernel launch: ") + hipGetErrorString(e); return MTSG_ERR_DEVICE; }
    if (result != MTSG_OK) return result;
    // samples actually inside the rectangle (all tiles of this call)
    if (tstride == 1 && !listed) s->stats.samples = (uint64_t)p->tile_w * p->tile_h * p->spp;
    if (s->flags & MTSG_FLAG_TIMING) {
        for (auto &te : s->timed) {
            float ms = 0;
            hipEventElapsedTime(&ms, s->evPool[te.second], s->evPool[te.second + 1]);
            switch (te.first) {
                case K_CAMERA: s->stats.ms_camera += ms; break;
                case K_CLOSEST: s->stats.ms_trace_closest += ms; break;
                case K_SHADOW: s->stats.ms_trace_shadow += ms; break;
                case K_SHADE: s->stats.ms_shade += ms; break;
                case K_SPLAT: s->stats.ms_splat += ms; break;
                case K_FINISH: s->stats.ms_finish += ms; break;
                case K_SORT: s->stats.ms_sort += ms; break;
            }
        }
    }
    if (count) {
        unsigned long long c[CTR_WORDS];
        HIP_TRY(hipMemcpy(c, s->LP[0].ctr, sizeof(c), hipMemcpyDeviceToHost));
        s->stats.nodes_visited = c[0];
        s->stats.leaf_refs = c[1];
        s->stats.tri_tests = c[2];
        s->stats.wave_node_iters = c[3];
        s->stats.wave_test_iters = c[4];
        s->stats.wave_steps = c[5];
        s->stats.wave_active_lanes = c[6];
        s->stats.shadow_nodes_visited = c[8];
        s->stats.shadow_leaf_refs = c[9];
        s->stats.shadow_tri_tests = c[10];
        s->stats.shadow_wave_node_iters = c[11];
        s->stats.shadow_wave_test_iters = c[12];
        s->stats.shadow_wave_steps = c[13];
        s->stats.shadow_wave_active_lanes = c[14];
        s->stats.iter_max_closest = c[7];
        s->stats.iter_max_shadow = c[15];
        for (int k = 0; k < 16; ++k) {
            s->stats.iter_hist_closest[k] = c[16 + k];
            s->stats.iter_hist_shadow[k] = c[32 + k];
        }
        s->stragglers.assign(c + 64, c + 64 + 8 * std::min<unsigned long long>(c[48], STRAGGLER_MAX));
        s->stats.instance_visits = c[49];
        s->stats.shadow_instance_visits = c[50];
        s->stats.instance_rejects = c[58];
        s->stats.instance_prefiltered = c[59];
        s->stats.tie_retraces = c[51];
        s->stats.guard_rays_closest = c[52];
        s->stats.guard_rays_shadow = c[53];
        s->stats.guard_steps_closest = c[54];
        s->stats.guard_steps_shadow = c[55];
        s->stats.restarts_closest = c[56];
        s->stats.restarts_shadow = c[57];
    }
    s->stats.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return MTSG_OK;
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int mtsg_device_pci_id(int device, char *buf, int len) {
    if (!buf || len < 13) { g_err = "mtsg_device_pci_id: buffer too small"; return MTSG_ERR_INVALID; }
    if (hipDeviceGetPCIBusId(buf, len, device) != hipSuccess) { g_err = "hipDeviceGetPCIBusId failed"; return MTSG_ERR_DEVICE; }
    return MTSG_OK;
}

int mtsg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int gfx950 = 0;
    for (int i = 0; i < n; ++i) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, i) == hipSuccess && strncmp(prop.gcnArchName, "gfx950", 6) == 0) ++gfx950;
    }
    return gfx950;
}

int mtsg_scene_create(const mtsg_scene_desc *d, int device, mtsg_scene **out) {
    if (!d || !out) { g_err = "null argument"; return MTSG_ERR_INVALID; }
    *out = nullptr;
    if (d->abi_version != MTSG_ABI_VERSION) { g_err = "ABI version mismatch"; return MTSG_ERR_INVALID; }
    if (d->n_prims != d->n_triangles + d->n_rects + d->n_instances || d->n_nodes == 0 || d->n_emitters == 0) {
        g_err = "inconsistent scene description";
        return MTSG_ERR_INVALID;
    }
    if (d->camera.border > MAX_BORDER) { g_err = "reconstruction filter radius too large (border > 4)"; return MTSG_ERR_INVALID; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        g_err = "no such HIP device";
        return MTSG_ERR_NODEVICE;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        g_err = std::string("device is not gfx950: ") + prop.gcnArchName;
        return MTSG_ERR_NODEVICE;
    }
    auto *s = new mtsg_scene();
    s->device = device;
    auto fail = [&](int rc) { mtsg_scene_destroy(s); return rc; };
    if (hipSetDevice(device) != hipSuccess) { g_err = "hipSetDevice failed"; delete s; return MTSG_ERR_DEVICE; }
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) { g_err = "stream"; delete s; return MTSG_ERR_DEVICE; }
    s->cuCount = prop.multiProcessorCount;
    // ---- convert + upload (host-side SoA -> device layout)
    std::vector<float4> vpos(d->n_vertices), vnrm(d->n_vertices);
    for (uint32_t i = 0; i < d->n_vertices; ++i) {
        vpos[i] = make_float4(d->vtx_pos[3 * i], d->vtx_pos[3 * i + 1], d->vtx_pos[3 * i + 2], 0.f);
        vnrm[i] = make_float4(d->vtx_nrm[3 * i], d->vtx_nrm[3 * i + 1], d->vtx_nrm[3 * i + 2], 0.f);
    }
    std::vector<uint4> tidx(d->n_triangles);
    for (uint32_t t = 0; t < d->n_triangles; ++t)
        tidx[t] = make_uint4(d->tri_idx[3 * t], d->tri_idx[3 * t + 1], d->tri_idx[3 * t + 2], 0);
    for (uint32_t sh = 0; sh < d->n_shapes; ++sh)
        if (d->shapes[sh].type == MTSG_SHAPE_MESH)
            for (uint32_t t = 0; t < d->shapes[sh].tri_count; ++t) tidx[d->shapes[sh].tri_begin + t].w = sh;
    std::vector<float4> shrec((size_t)d->n_triangles * 6);
    for (uint32_t t = 0; t < d->n_triangles; ++t) {
        const uint4 ti = tidx[t];
        if (ti.x >= d->n_vertices || ti.y >= d->n_vertices || ti.z >= d->n_vertices || ti.w >= d->n_shapes) {
            g_err = "triangle index out of range";
            return fail(MTSG_ERR_INVALID);
        }
        const float *P = d->vtx_pos, *N = d->vtx_nrm;
        float f[24];
        for (int k = 0; k < 3; ++k) {
            f[k] = P[3 * ti.x + k]; f[3 + k] = P[3 * ti.y + k]; f[6 + k] = P[3 * ti.z + k];
            f[9 + k] = N[3 * ti.x + k]; f[12 + k] = N[3 * ti.y + k]; f[15 + k] = N[3 * ti.z + k];
            f[18 + k] = d->tri_dpdu[3 * t + k];
        }
        const mtsg_shape &sh = d->shapes[ti.w];
        uint32_t u[3] = {ti.w, (uint32_t)sh.bsdf | (sh.face_normals ? 0x80000000u : 0u), (uint32_t)sh.emitter};
        memcpy(f + 21, u, sizeof(u));
        memcpy(&shrec[6 * (size_t)t], f, sizeof(f));
    }
    int rc;
    DevScene &ds = s->ds;
    auto up = [&](auto *src, size_t n, auto **dst) {
        int r = upload(src, n, dst);
        if (r == MTSG_OK && *dst) s->allocs.push_back((void *)*dst);
        return r;
    };
    // ---- device kd-tree layout from Mitsuba's KDNode array (same splits and
    // leaves, re-laid out): sibling pairs (host only, the input of the
    // two-level blocks) + leaf-ordered TriAccel copies.  The top-level tree
    // and every shape group's tree (two-level instancing) share both arrays.
    std::vector<uint4> pairs;
    std::vector<float4> triL;
    pairs.reserve(d->n_nodes / 2 + 1);
    triL.reserve((size_t)d->n_indices * 3);
    bool layoutOk = true;
    const mtsg_kdnode *tNodes = d->nodes;
    const uint32_t *tIdx = d->indices;
    uint32_t tNodeCount = d->n_nodes, tIdxCount = d->n_indices;
    std::function<uint2(uint32_t, int)> convert = [&](uint32_t ni, int depth) -> uint2 {
        if (depth > 64 || ni >= tNodeCount) { layoutOk = false; return make_uint2(0x80000000u, 0u); }
        const mtsg_kdnode &N = tNodes[ni];
        if (N.combined & 0x80000000u) {
            const uint32_t start = (uint32_t)(triL.size() / 3);
            for (uint32_t e = N.combined & 0x7FFFFFFFu; e < N.data; ++e) {
                const uint32_t p = e < tIdxCount ? tIdx[e] : 0xFFFFFFFFu;
                if (p >= d->n_prims) { layoutOk = false; break; }
                mtsg_triaccel ta = d->triaccel[p];
                if (ta.k == MTSG_TRIACCEL_SHAPE && ta.shape_index < d->n_shapes &&
                    d->shapes[ta.shape_index].type == MTSG_SHAPE_INSTANCE) {
                    if (ta.prim_index >= d->n_instances) { layoutOk = false; break; }
                    ta.k = KINST;
                    // the instance's world box in the record's free words
                    // (n_u n_v n_d = min, a_u a_v b_nu = max): the group box's
                    // corners through to_world in double, widened by 1e-4 of
                    // its size and position and rounded outward, so the
                    // traversal's prefilter (kernels.h inst_box) never drops an
                    // entry the exact group-space clip would take
                    const mtsg_instance &I = d->instances[ta.prim_index];
                    if (I.group >= d->n_groups) { layoutOk = false; break; }
                    const mtsg_group &G = d->groups[I.group];
                    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
                    for (int c = 0; c < 8; ++c) {
                        const double q[3] = {(c & 1) ? G.aabb_max[0] : G.aabb_min[0], (c & 2) ? G.aabb_max[1] : G.aabb_min[1],
                                             (c & 4) ? G.aabb_max[2] : G.aabb_min[2]};
                        for (int a = 0; a < 3; ++a) {
                            const float *W = I.to_world + 4 * a;
                            const double w = (double)W[0] * q[0] + (double)W[1] * q[1] + (double)W[2] * q[2] + (double)W[3];
                            lo[a] = std::min(lo[a], w);
                            hi[a] = std::max(hi[a], w);
                        }
                    }
                    double ext = 0, mag = 0;
                    for (int a = 0; a < 3; ++a) {
                        ext = std::max(ext, hi[a] - lo[a]);
                        mag = std::max(mag, std::max(std::fabs(lo[a]), std::fabs(hi[a])));
                    }
                    const double m = 1e-4 * (ext + mag) + 1e-30;
                    float bmin[3], bmax[3];
                    for (int a = 0; a < 3; ++a) {
                        bmin[a] = std::nextafter((float)(lo[a] - m), -INFINITY);
                        bmax[a] = std::nextafter((float)(hi[a] + m), INFINITY);
                    }
                    if (!std::isfinite(bmin[0] + bmin[1] + bmin[2] + bmax[0] + bmax[1] + bmax[2])) {
                        // a degenerate or unbounded transform: a box that takes every ray
                        for (int a = 0; a < 3; ++a) { bmin[a] = -INFINITY; bmax[a] = INFINITY; }
                    }
                    ta.n_u = bmin[0]; ta.n_v = bmin[1]; ta.n_d = bmin[2];
                    ta.a_u = bmax[0]; ta.a_v = bmax[1]; ta.b_nu = bmax[2];
                }
                // the TriAccel index (Mitsuba's mailbox key, kernels.h
                // mailbox_step) in place of the shape index
                ta.shape_index = p;
                const float4 *t = (const float4 *)&ta;
                triL.push_back(t[0]); triL.push_back(t[1]); triL.push_back(t[2]);
            }
            return make_uint2(0x80000000u | start, (uint32_t)(triL.size() / 3));
        }
        const uint32_t left = ni + ((N.combined & ~(3u | 0x40000000u)) >> 2);
        const uint32_t pi = (uint32_t)pairs.size();
        pairs.push_back(make_uint4(0, 0, 0, 0));
        const uint2 L = convert(left, depth + 1);
        const uint2 R = convert(left + 1, depth + 1);
        pairs[pi] = make_uint4(L.x, L.y, R.x, R.y);
        return make_uint2((N.combined & 3u) | (pi << 2), N.data);
    };
    const uint2 root = convert(0, 0);
    std::vector<uint2> groupRoots(d->n_groups);
    if (d->n_instances && (!d->instances || !d->groups || !d->group_nodes || !d->group_indices)) layoutOk = false;
    for (uint32_t g = 0; g < d->n_groups && layoutOk; ++g) {
        const mtsg_group &G = d->groups[g];
        if ((uint64_t)G.node_offset + G.n_nodes > d->n_group_nodes || (uint64_t)G.index_offset + G.n_indices > d->n_group_indices ||
            G.n_nodes == 0) { layoutOk = false; break; }
        tNodes = d->group_nodes + G.node_offset;
        tIdx = d->group_indices + G.index_offset;
        tNodeCount = G.n_nodes;
        tIdxCount = G.n_indices;
        groupRoots[g] = convert(0, 0);
    }
    for (uint32_t i = 0; i < d->n_instances && layoutOk; ++i)
        if (d->instances[i].group >= d->n_groups) layoutOk = false;
    if (!layoutOk || pairs.size() >= (1u << 29) || triL.size() / 3 >= (1u << 30)) {
        g_err = "malformed or oversized kd-tree";
        return fail(MTSG_ERR_INVALID);
    }
    // ---- two-level blocks from the binary pair layout
    std::vector<uint4> blocks;
    blocks.reserve(pairs.size() * 2 + 8);
    // the scene root's block and the blocks of its (up to four) grandchildren
    // come first, blocks 0-4: the top four levels of the tree in 320 B (the
    // MTSG_LDS_TOP variant stages them in LDS)
    std::unordered_map<uint32_t, uint32_t> preBlock;
    auto reserveBlock = [&](uint32_t pair) {
        preBlock[pair] = (uint32_t)(blocks.size() / 4);
        blocks.resize(blocks.size() + 4, make_uint4(0, 0, 0, 0));
    };
    if (!(root.x & 0x80000000u)) {
        reserveBlock(root.x >> 2);
        const uint4 pr = pairs[root.x >> 2];
        for (const uint2 c : {make_uint2(pr.x, pr.y), make_uint2(pr.z, pr.w)}) {
            if (c.x & 0x80000000u) continue;
            const uint4 gp = pairs[c.x >> 2];
            for (const uint2 g : {make_uint2(gp.x, gp.y), make_uint2(gp.z, gp.w)})
                if (!(g.x & 0x80000000u)) reserveBlock(g.x >> 2);
        }
    }
    std::function<uint2(uint2, bool, uint32_t)> conv2 = [&](uint2 w, bool root, uint32_t slot) -> uint2 {
        if (w.x & 0x80000000u) return w;                       // leaf: unchanged
        const uint4 pr = pairs[w.x >> 2];
        const uint2 L = make_uint2(pr.x, pr.y), R = make_uint2(pr.z, pr.w);
        if (root) {
            uint32_t b;
            const auto pre = preBlock.find(w.x >> 2);
            if (pre != preBlock.end()) {
                b = pre->second;
            } else {
                b = (uint32_t)(blocks.size() / 4);
                blocks.resize(blocks.size() + 4, make_uint4(0, 0, 0, 0));
            }
            const uint2 nL = conv2(L, false, 4 * b + 1);
            const uint2 nR = conv2(R, false, 4 * b + 2);
            blocks[4 * b] = make_uint4(nL.x, nL.y, nR.x, nR.y);
            return make_uint2((w.x & 3u) | (b << 3), w.y);
        }
        // pair-only node: its children are block roots (or leaves)
        const uint2 nL = conv2(L, true, 0), nR = conv2(R, true, 0);
        blocks[slot] = make_uint4(nL.x, nL.y, nR.x, nR.y);
        return make_uint2((w.x & 3u) | 4u | (slot << 3), w.y);
    };
    const uint2 root2 = conv2(root, true, 0);
    for (auto &gr : groupRoots) gr = conv2(gr, true, 0);
    blocks.resize(blocks.size() + 4, make_uint4(0, 0, 0, 0));   // slack for the 3-slot fetch of the last slot
    if (blocks.size() < 20) blocks.resize(20, make_uint4(0, 0, 0, 0));   // blocks 0-4 are always readable
    if (blocks.size() >= (1u << 29)) { g_err = "kd-tree too large for the two-level layout"; return fail(MTSG_ERR_INVALID); }
    if (triL.empty()) triL.resize(3, make_float4(0, 0, 0, 0));
    uint4 *dblocks; float4 *dtriL; float4 *dvpos, *dvnrm, *dshrec; uint4 *dtidx;
    mtsg_rect *rects; mtsg_shape *shapes; mtsg_bsdf *bsdfs; mtsg_emitter *emitters; float *ecdf, *etcdf;
    if ((rc = up(triL.data(), triL.size(), &dtriL)) ||
        (rc = up(blocks.data(), blocks.size(), &dblocks)) ||
        (rc = up(vpos.data(), vpos.size(), &dvpos)) || (rc = up(vnrm.data(), vnrm.size(), &dvnrm)) ||
        (rc = up(tidx.data(), tidx.size(), &dtidx)) ||
        (rc = up(shrec.data(), shrec.size(), &dshrec)) ||
        (rc = up(d->rects, d->n_rects, &rects)) || (rc = up(d->shapes, d->n_shapes, &shapes)) ||
        (rc = up(d->bsdfs, d->n_bsdfs, &bsdfs)) || (rc = up(d->emitters, d->n_emitters, &emitters)) ||
        (rc = up(d->emitter_cdf, d->n_emitters + 1, &ecdf)) ||
        (rc = up(d->emitter_tri_cdf, d->n_emitter_tri_cdf, &etcdf)))
        return fail(rc);
    ds.blocks = dblocks; ds.root2 = root2;
    ds.triL = dtriL; ds.vpos = dvpos; ds.vnrm = dvnrm;
    {
        // to_object rows of every rectangle, 48 B each (DevScene::rectM)
        std::vector<float4> rm((size_t)3 * std::max<uint32_t>(d->n_rects, 1u), make_float4(0, 0, 0, 0));
        for (uint32_t i = 0; i < d->n_rects; ++i)
            for (int k = 0; k < 3; ++k) {
                const float *m = d->rects[i].to_object + 4 * k;
                rm[3 * i + k] = make_float4(m[0], m[1], m[2], m[3]);
            }
        // per rectangle its shading data, per emitter its rectangle's rows
        // (DevScene::rectSh / emitRect)
        if (d->n_bsdfs >= 0xFFFFu || d->n_emitters >= 0xFFFEu) { g_err = "too many BSDFs or emitters"; return fail(MTSG_ERR_INVALID); }
        std::vector<float4> rs((size_t)2 * std::max<uint32_t>(d->n_rects, 1u), make_float4(0, 0, 0, 0));
        for (uint32_t i = 0; i < d->n_rects; ++i) {
            const mtsg_rect &R = d->rects[i];
            if (R.shape_index >= d->n_shapes) { g_err = "rectangle with an invalid shape index"; return fail(MTSG_ERR_INVALID); }
            const mtsg_shape &sh = d->shapes[R.shape_index];
            uint32_t be = ((uint32_t)sh.bsdf & 0xFFFFu) | (uint32_t)(sh.emitter + 1) << 16, si = R.shape_index;
            float bef, sif;
            memcpy(&bef, &be, 4);
            memcpy(&sif, &si, 4);
            rs[2 * i] = make_float4(R.frame_n[0], R.frame_n[1], R.frame_n[2], sif);
            rs[2 * i + 1] = make_float4(R.dpdu[0], R.dpdu[1], R.dpdu[2], bef);
        }
        std::vector<float4> er((size_t)4 * std::max<uint32_t>(d->n_emitters, 1u), make_float4(0, 0, 0, 0));
        for (uint32_t e = 0; e < d->n_emitters; ++e) {
            const int32_t sidx = d->emitters[e].shape;
            uint32_t type = (uint32_t)MTSG_SHAPE_MESH + 100u;   // not a shape emitter (environment)
            if (sidx >= 0 && (uint32_t)sidx < d->n_shapes) {
                const mtsg_shape &sh = d->shapes[sidx];
                type = (uint32_t)sh.type;
                if (sh.type == MTSG_SHAPE_RECT && sh.rect < d->n_rects) {
                    const mtsg_rect &R = d->rects[sh.rect];
                    for (int k = 0; k < 3; ++k)
                        er[4 * e + k] = make_float4(R.to_world[4 * k], R.to_world[4 * k + 1], R.to_world[4 * k + 2], R.to_world[4 * k + 3]);
                    er[4 * e + 3] = make_float4(R.frame_n[0], R.frame_n[1], R.frame_n[2], 0.f);
                }
            }
            memcpy(&er[4 * e + 3].w, &type, 4);
        }
        float4 *drm, *drs, *der;
        if ((rc = up(rm.data(), rm.size(), &drm)) || (rc = up(rs.data(), rs.size(), &drs)) || (rc = up(er.data(), er.size(), &der)))
            return fail(rc);
        ds.rectM = drm;
        ds.rectSh = drs;
        ds.emitRect = der;
    }
    ds.tidx = dtidx; ds.shrec = dshrec; ds.rects = rects; ds.shapes = shapes; ds.bsdfs = bsdfs;
    ds.emitters = emitters; ds.emitter_cdf = ecdf; ds.emitter_tri_cdf = etcdf;
    ds.inst = nullptr;
    if (d->n_instances) {
        std::vector<float4> in((size_t)8 * d->n_instances);
        for (uint32_t i = 0; i < d->n_instances; ++i) {
            const mtsg_instance &I = d->instances[i];
            const mtsg_group &G = d->groups[I.group];
            const float *L = I.to_local, *W = I.to_world;
            float4 *o = &in[8 * (size_t)i];
            for (int r = 0; r < 3; ++r) {
                o[r] = make_float4(L[4 * r], L[4 * r + 1], L[4 * r + 2], L[4 * r + 3]);
                o[3 + r] = make_float4(W[4 * r], W[4 * r + 1], W[4 * r + 2], W[4 * r + 3]);
            }
            const uint2 gr = groupRoots[I.group];
            float r0, r1;
            memcpy(&r0, &gr.x, 4);
            memcpy(&r1, &gr.y, 4);
            o[6] = make_float4(G.aabb_min[0], G.aabb_min[1], G.aabb_min[2], r0);
            o[7] = make_float4(G.aabb_max[0], G.aabb_max[1], G.aabb_max[2], r1);
        }
        float4 *dinst;
        if ((rc = up(in.data(), in.size(), &dinst))) return fail(rc);
        ds.inst = dinst;
    }
    // traversal stacks and the kd-restart guard (kernels.h kd_restart): the
    // compile-time defaults; only mtsg_set_test_knobs (tests) changes them
    ds.capFlat = SHORT_STACK;
    ds.capGrp = INNER_STACK;
    ds.capTop = OUTER_STACK;
    ds.rstGuard = RST_GUARD;
    ds.rstMax = RST_MAX;
    ds.rstMaxC = RST_MAX;
    ds.instPrefilter = 1;
    s->knobs = false;
    // two-level tie keys (kernels.h spec_iter_i): the TriAccel key count as
    // the per-instance stride, so keys of different (primitive, instance)
    // pairs never coincide; scenes too large for 32-bit keys fall back to an
    // odd multiplier (a bijection per instance; pairs across instances can
    // then collide, which only hides a tie of two such primitives)
    ds.instKeyStride = (uint64_t)d->n_prims * ((uint64_t)d->n_instances + 1) <= 0xFFFFFFFFull ? d->n_prims : 0x9E3779B1u;
    // environment emitter tables (envmap.h)
    ds.has_env = d->has_envmap ? 1 : 0;
    s->mats = 0;
    for (uint32_t i = 0; i < d->n_bsdfs; ++i) {
        const mtsg_bsdf &b = d->bsdfs[i];
        if (b.type == MTSG_BSDF_CONDUCTOR || b.type == MTSG_BSDF_PLASTIC || b.type == MTSG_BSDF_ROUGHDIELECTRIC ||
            b.type == MTSG_BSDF_ROUGHPLASTIC || b.twosided)
            s->extBsdfs = true;
        // the material classes the non-extended shading kernel must hold
        if (b.type == MTSG_BSDF_DIFFUSE) s->mats |= MAT_DIFFUSE;
        else if (b.type == MTSG_BSDF_ROUGHCONDUCTOR) s->mats |= b.distribution == MTSG_MF_GGX ? MAT_RC_GGX : MAT_RC_OTHER;
        else if (b.type == MTSG_BSDF_DIELECTRIC) s->mats |= MAT_DIELECTRIC;
        else s->mats |= MATS_ALL;
        if (b.twosided && (b.back < 0 || (uint32_t)b.back >= d->n_bsdfs)) {
            g_err = "bsdf " + std::to_string(i) + ": twosided back record out of range";
            return fail(MTSG_ERR_INVALID);
        }
    }
    ds.env = DevEnv{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (d->has_envmap) {
        const mtsg_envmap &E = d->envmap;
        const mtsg_mipmap &EM = E.mip;
        if (EM.levels <= 0 || EM.levels > MTSG_ENVMAP_MAX_LEVELS || !d->env_texels || !d->env_cdf_rows || !d->env_cdf_cols ||
            !d->env_row_weights || E.emitter < 0 || (uint32_t)E.emitter >= d->n_emitters) {
            g_err = "inconsistent environment map description";
            return fail(MTSG_ERR_INVALID);
        }
        size_t need = 0;
        for (int l = 0; l < EM.levels; ++l)
            need = std::max(need, (size_t)EM.level_offset[l] + 3 * (size_t)EM.level_w[l] * EM.level_h[l]);
        if (need > d->n_env_texels) { g_err = "environment map texel array too small"; return fail(MTSG_ERR_INVALID); }
        mtsg_envmap *dE; float *dt, *dr, *dc, *dw;
        uint32_t *dgr, *dgc;
        const int W = EM.level_w[0], H = EM.level_h[0];
        // guide tables of the CDF searches (envmap.h env_sample_reuse_guided):
        // entry g = std::lower_bound of g / ENV_GUIDE over the size + 1 entries
        auto guides = [](const float *cdf, uint32_t size, uint32_t *out) {
            for (uint32_t g = 0; g <= ENV_GUIDE; ++g)
                out[g] = (uint32_t)(std::lower_bound(cdf, cdf + size + 1, (float)g / (float)ENV_GUIDE) - cdf);
        };
        std::vector<uint32_t> gr(ENV_GUIDE + 1), gc((size_t)(ENV_GUIDE + 1) * H);
        guides(d->env_cdf_rows, (uint32_t)H, gr.data());
        for (int y = 0; y < H; ++y) guides(d->env_cdf_cols + (size_t)y * (W + 1), (uint32_t)W, gc.data() + (size_t)y * (ENV_GUIDE + 1));
        if ((rc = up(&E, 1, &dE)) || (rc = up(d->env_texels, d->n_env_texels, &dt)) ||
            (rc = up(d->env_cdf_rows, (size_t)H + 1, &dr)) || (rc = up(d->env_cdf_cols, (size_t)(W + 1) * H, &dc)) ||
            (rc = up(d->env_row_weights, (size_t)H, &dw)) || (rc = up(gr.data(), gr.size(), &dgr)) ||
            (rc = up(gc.data(), gc.size(), &dgc)))
            return fail(rc);
        ds.env = DevEnv{dE, dt, dr, dc, dw, dgr, dgc};
    }
    // bitmap textures (mipmap.h) and the per-triangle records of their lookups
    ds.textures = nullptr; ds.tex_texels = nullptr; ds.ttex = nullptr;
    bool texDiffs = false;
    for (uint32_t i = 0; i < d->n_bsdfs; ++i)
        if (d->bsdfs[i].texture < 0 || (uint32_t)d->bsdfs[i].texture > d->n_textures) {
            g_err = "bsdf " + std::to_string(i) + ": texture index out of range";
            return fail(MTSG_ERR_INVALID);
        }
    if (d->n_textures) {
        if (!d->textures || !d->tex_texels || (d->n_triangles && (!d->tri_uv || !d->tri_dpdv))) {
            g_err = "inconsistent texture description";
            return fail(MTSG_ERR_INVALID);
        }
        for (uint32_t i = 0; i < d->n_textures; ++i) {
            const mtsg_mipmap &M = d->textures[i].mip;
            bool ok = M.levels > 0 && M.levels <= MTSG_MIPMAP_MAX_LEVELS && M.filter >= MTSG_MIP_NEAREST && M.filter <= MTSG_MIP_EWA &&
                      M.wrap_u >= MTSG_WRAP_CLAMP && M.wrap_u <= MTSG_WRAP_ONE && M.wrap_v >= MTSG_WRAP_CLAMP && M.wrap_v <= MTSG_WRAP_ONE;
            for (int l = 0; ok && l < M.levels; ++l)
                ok = M.level_w[l] > 0 && M.level_h[l] > 0 &&
                     (size_t)M.level_offset[l] + 3 * (size_t)M.level_w[l] * M.level_h[l] <= d->n_tex_texels;
            if (!ok) { g_err = "texture " + std::to_string(i) + ": malformed MIP map"; return fail(MTSG_ERR_INVALID); }
            texDiffs |= M.filter == MTSG_MIP_TRILINEAR || M.filter == MTSG_MIP_EWA;
        }
        std::vector<float4> tt((size_t)3 * std::max(1u, d->n_triangles), make_float4(0, 0, 0, 0));
        for (uint32_t t = 0; t < d->n_triangles; ++t) {
            const float *uv = d->tri_uv + 6 * (size_t)t, *dv = d->tri_dpdv + 3 * (size_t)t;
            tt[3 * t] = make_float4(uv[0], uv[1], uv[2], uv[3]);
            tt[3 * t + 1] = make_float4(uv[4], uv[5], dv[0], dv[1]);
            tt[3 * t + 2] = make_float4(dv[2], 0.f, 0.f, 0.f);
        }
        mtsg_texture *dtex; float *dtt; float4 *dttex;
        if ((rc = up(d->textures, d->n_textures, &dtex)) || (rc = up(d->tex_texels, d->n_tex_texels, &dtt)) ||
            (rc = up(tt.data(), tt.size(), &dttex)))
            return fail(rc);
        ds.textures = dtex; ds.tex_texels = dtt; ds.ttex = dttex;
        s->nTextures = d->n_textures;
        s->extBsdfs = true;   // texture lookups live in the extended shade kernel
    }
    s->texDiffs = texDiffs;
    s->hasEnvmap = d->has_envmap != 0;
    // myPath2_OM occupancy maps (om.cpp)
    ds.om = nullptr; ds.om_bits = nullptr;
    if (d->om) {
        if (!d->om_bits) { g_err = "occupancy maps without their bits"; return fail(MTSG_ERR_INVALID); }
        mtsg_om *dom; uint32_t *dbits;
        if ((rc = up(d->om, 1, &dom)) ||
            (rc = up(d->om_bits, (size_t)MTSG_OM_COUNT * MTSG_OM_SIZE * MTSG_OM_SIZE * (MTSG_OM_SIZE / 32), &dbits)))
            return fail(rc);
        ds.om = dom; ds.om_bits = dbits;
    }
    ds.n_emitters = d->n_emitters;
    ds.n_tri = d->n_triangles;
    ds.n_bsdfs = d->n_bsdfs;
    for (int k = 0; k < 3; ++k) { ds.bmin[k] = d->aabb_min[k]; ds.bmax[k] = d->aabb_max[k]; }
    DevCamera &c = s->cam;
    const mtsg_camera &hc = d->camera;
    memcpy(c.s2c, hc.sample_to_camera, sizeof(c.s2c));
    memcpy(c.c2w, hc.camera_to_world, sizeof(c.c2w));
    c.near_clip = hc.near_clip; c.far_clip = hc.far_clip; c.inv_res_x = hc.inv_res_x; c.inv_res_y = hc.inv_res_y;
    c.film_w = hc.film_w; c.film_h = hc.film_h;
    c.filter_radius = hc.filter_radius; c.filter_scale = hc.filter_scale; c.border = hc.border;
    c.has_alpha = hc.has_alpha;
    memcpy(c.filter_values, hc.filter_values, sizeof(c.filter_values));
    memcpy(c.dx, hc.dx, sizeof(c.dx));
    memcpy(c.dy, hc.dy, sizeof(c.dy));
    c.crop_w = hc.crop_w; c.crop_h = hc.crop_h;
    ds.camO[0] = c.c2w[3]; ds.camO[1] = c.c2w[7]; ds.camO[2] = c.c2w[11];
    ds.camNear = c.near_clip; ds.camFar = c.far_clip;
    ds.camCompact = ds.inst ? 0 : 1;
    c.compact = ds.camCompact;
    camera_diff_mode(s);
    // the camera on the device too: bounce 0 recomputes a missing camera ray's
    // differentials from it (DevScene::cam_env_diffs)
    {
        DevCamera *dc;
        if ((rc = up(&s->cam, 1, &dc))) return fail(rc);
        ds.camDev = dc;
    }
    // sampler and its quasi-Monte Carlo tables
    s->samplerType = d->sampler.type;
    s->samplerDim = d->sampler.dimension;
    if (s->samplerType < MTSG_SAMPLER_INDEPENDENT || s->samplerType > MTSG_SAMPLER_SOBOL) {
        g_err = "unknown sampler type";
        return fail(MTSG_ERR_INVALID);
    }
    if (s->samplerType == MTSG_SAMPLER_HALTON || s->samplerType == MTSG_SAMPLER_HAMMERSLEY) {
        if (!d->qmc_primes || !d->qmc_perm_offset) { g_err = "sampler: missing QMC tables"; return fail(MTSG_ERR_INVALID); }
        uint32_t *dp, *doff;
        if ((rc = up(d->qmc_primes, MTSG_QMC_PRIMES, &dp)) || (rc = up(d->qmc_perm_offset, MTSG_QMC_PRIMES, &doff)))
            return fail(rc);
        s->ds.qmcPrimes = dp;
        s->ds.qmcOff = doff;
        if (d->qmc_perm) {
            const size_t n = (size_t)d->qmc_perm_offset[MTSG_QMC_PRIMES - 1] + d->qmc_primes[MTSG_QMC_PRIMES - 1];
            uint16_t *dperm;
            if ((rc = up(d->qmc_perm, n, &dperm))) return fail(rc);
            s->ds.qmcPerm = dperm;
            // inverse permutations of the first two bases (faure.cpp:74-78)
            for (int b = 0; b < 2; ++b)
                for (uint32_t j = 0; j < d->qmc_primes[b]; ++j) s->qmcInv[b][d->qmc_perm[d->qmc_perm_offset[b] + j]] = (int)j;
        }
    }
    if (s->samplerType == MTSG_SAMPLER_SOBOL) {
        if (!d->sobol_matrices || !d->sobol_vdc || !d->sobol_vdc_inv) { g_err = "sampler: missing sobol tables"; return fail(MTSG_ERR_INVALID); }
        uint32_t r = 1, m = 0;
        while (r < (uint32_t)std::max(d->camera.crop_w, d->camera.crop_h)) r <<= 1;
        while ((1u << (m + 1)) <= r) ++m;
        if (m > 1 && (m > d->sobol_vdc_inv_rows || m > d->sobol_vdc_rows + 1)) { g_err = "sobol: film too large for the look_up tables"; return fail(MTSG_ERR_INVALID); }
        uint32_t *dm;
        uint64_t *dv, *dvi;
        if ((rc = up(d->sobol_matrices, (size_t)MTSG_SOBOL_DIMS * MTSG_SOBOL_COLUMNS, &dm)) ||
            (rc = up(d->sobol_vdc, (size_t)d->sobol_vdc_rows * MTSG_SOBOL_COLUMNS + MTSG_SOBOL_COLUMNS, &dv)) ||
            (rc = up(d->sobol_vdc_inv, (size_t)d->sobol_vdc_inv_rows * MTSG_SOBOL_COLUMNS, &dvi)))
            return fail(rc);
        s->sobolM = dm;
        s->sobolVdc = dv;
        s->sobolVdcInv = dvi;
        s->sobolScramble = d->sobol_scramble;
    }
    // persistent grids from the occupancy query
    int perCU = 0;
    if ((perCU = trace_flat_blocks_per_cu()) <= 0) perCU = 8;
    s->traceGrid = s->cuCount * perCU;
    perCU = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, (const void *)k_trace_s<false, MTSG_INST_MIN_IDLE, true>, TRACE_BLOCK, 0) != hipSuccess ||
        perCU <= 0)
        perCU = 4;
    s->traceGridInst = s->cuCount * perCU;
#ifndef MTSG_SHADE_WG_PER_CU
#define MTSG_SHADE_WG_PER_CU 64   // k_shade workgroups of 256 per CU, 4 resident (r05_shade_launch.txt: 8 -> 64, C3 shade -5%)
#endif
    s->shadeGrid = s->cuCount * MTSG_SHADE_WG_PER_CU * 256 / SHADE_BLOCK;
    perCU = 0;
    if ((perCU = finish_blocks_per_cu(false)) <= 0) perCU = 3;
    s->finishGrid = s->cuCount * perCU;
    if ((perCU = finish_blocks_per_cu(true)) <= 0) perCU = 3;
    s->finishGridMats = s->cuCount * perCU;
    // two-level traversal: the per-lane save slots of its grid (kernels.h save_vec)
    s->ds.instSave = nullptr;
    if (s->ds.inst && !MTSG_INST_REGSAVE) {
        uint4 *save = nullptr;
        // slots for the larger of the two grids that switch levels (k_trace_s, k_finish)
        const size_t lanes = (size_t)std::max(s->traceGridInst, s->finishGrid) * TRACE_BLOCK;
        if (hipMalloc((void **)&save, (size_t)SAVE_VECS * lanes * sizeof(uint4)) != hipSuccess) {
            g_err = "out of device memory (instance save slots)";
            return fail(MTSG_ERR_OOM);
        }
        s->allocs.push_back(save);
        s->ds.instSave = save;
    }
    s->finishPaths = MTSG_DEFAULT_FINISH_PATHS;
    s->lstream[0] = s->stream;
    for (int l = 1; l < MTSG_MAX_LANES; ++l)
        if (hipStreamCreateWithFlags(&s->lstream[l], hipStreamNonBlocking) != hipSuccess) { g_err = "stream"; return fail(MTSG_ERR_DEVICE); }
    if (hipHostMalloc((void **)&s->hostCnt, 2 * MTSG_MAX_LANES * HOSTCNT_STRIDE * sizeof(uint32_t)) != hipSuccess) { g_err = "pinned alloc"; return fail(MTSG_ERR_OOM); }
    *out = s;
    return MTSG_OK;
}

int mtsg_set_batch_paths(mtsg_scene *s, uint32_t paths) {
    if (!s || paths < TILE * TILE) { g_err = "batch must hold at least 256 paths"; return MTSG_ERR_INVALID; }
    s->requestedBatch = paths;
    return MTSG_OK;
}

int mtsg_set_test_knobs(mtsg_scene *s, const mtsg_test_knobs *k) {
    if (!s) return MTSG_ERR_INVALID;
    DevScene &ds = s->ds;
    ds.capFlat = SHORT_STACK;
    ds.capGrp = INNER_STACK;
    ds.capTop = OUTER_STACK;
    ds.rstGuard = RST_GUARD;
    ds.rstMax = RST_MAX;
    if (k) {
        if (k->stack_cap > 0) {
            const uint32_t cap = (uint32_t)k->stack_cap;
            ds.capFlat = std::min(ds.capFlat, cap);
            ds.capGrp = std::min(ds.capGrp, cap);
            ds.capTop = std::min(ds.capTop, cap);
        }
        if (k->restart_guard >= 0) ds.rstGuard = (uint32_t)k->restart_guard;
        if (k->restart_limit >= 0) ds.rstMax = std::min<uint32_t>(RST_MAX, (uint32_t)k->restart_limit);
    }
    ds.rstMaxC = (k && k->limit_shadow_only) ? RST_MAX : ds.rstMax;
    ds.instPrefilter = (k && k->no_instance_prefilter) ? 0u : 1u;
    // any change selects the KNOBS kernel instantiations (the production
    // kernels keep their compile-time constants) and turns the tail kernel off
    s->knobs = ds.capFlat != (uint32_t)SHORT_STACK || ds.capGrp != (uint32_t)INNER_STACK || ds.capTop != (uint32_t)OUTER_STACK ||
               ds.rstGuard != RST_GUARD || ds.rstMax != RST_MAX || ds.rstMaxC != RST_MAX || !ds.instPrefilter;
    return MTSG_OK;
}

int mtsg_set_finish_paths(mtsg_scene *s, uint32_t paths) {
    if (!s) return MTSG_ERR_INVALID;
    s->finishPaths = paths;
    return MTSG_OK;
}

int mtsg_set_option(mtsg_scene *s, int32_t key, int64_t value) {
    if (!s) { g_err = "null scene"; return MTSG_ERR_INVALID; }
    switch (key) {
        case MTSG_OPT_TRACE_REFILL:
            if (value != 16 && value != 32) { g_err = "MTSG_OPT_TRACE_REFILL: 16 or 32 idle lanes"; return MTSG_ERR_INVALID; }
            s->traceMode = value == 32 ? 1 : 0;
            return MTSG_OK;
        case MTSG_OPT_FINISH_SHADE_MIN:
            if (value < 1 || value > 64) { g_err = "MTSG_OPT_FINISH_SHADE_MIN: 1..64 lanes"; return MTSG_ERR_INVALID; }
            s->finishShadeMin = (uint32_t)value;
            return MTSG_OK;
        case MTSG_OPT_LANES:
            if (value < 1 || value > MTSG_MAX_LANES) { g_err = "MTSG_OPT_LANES: 1..4 concurrent batches"; return MTSG_ERR_INVALID; }
            s->lanes = (int)value;
            return MTSG_OK;
        case MTSG_OPT_STAGGER:
            if (value < 0 || value > 16) { g_err = "MTSG_OPT_STAGGER: 0..16 bounces"; return MTSG_ERR_INVALID; }
            s->stagger = (int)value;
            return MTSG_OK;
        case MTSG_OPT_SHADE_GENERIC:
            s->shadeGeneric = value != 0;
            return MTSG_OK;
        case MTSG_OPT_RAY_ORDER:
            if (value < 0 || value > 1) { g_err = "MTSG_OPT_RAY_ORDER: 0 (append order) or 1 (direction-sorted windows)"; return MTSG_ERR_INVALID; }
            s->rayOrder = (int)value;
            return MTSG_OK;
        case MTSG_OPT_CAMERA_DIFFS:
            if (value < 0 || value > 1) { g_err = "MTSG_OPT_CAMERA_DIFFS: 0 (recomputed on a miss) or 1 (stored)"; return MTSG_ERR_INVALID; }
            s->storeCamDiffs = value != 0;
            camera_diff_mode(s);
            return MTSG_OK;
        default:
            g_err = "unknown option key " + std::to_string(key);
            return MTSG_ERR_INVALID;
    }
}

int mtsg_set_flags(mtsg_scene *s, uint32_t flags) {
    if (!s) return MTSG_ERR_INVALID;
    s->flags = flags;
    return MTSG_OK;
}

int mtsg_get_stats(mtsg_scene *s, mtsg_stats *out) {
    if (!s || !out) return MTSG_ERR_INVALID;
    *out = s->stats;
    return MTSG_OK;
}

int mtsg_debug_wavetimes(mtsg_scene *s, uint64_t *out, uint32_t max_launches, uint32_t *waves) {
    if (!s || !waves || (!out && max_launches)) return MTSG_ERR_INVALID;
    *waves = (uint32_t)s->traceGrid;
    const uint32_t n = std::min(max_launches, s->wtLaunches);
    if (n && s->waveTimes &&
        hipMemcpy(out, s->waveTimes, (size_t)WT_WORDS * s->traceGrid * n * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        return MTSG_ERR_DEVICE;
    return (int)s->wtLaunches;
}

int mtsg_debug_stragglers(mtsg_scene *s, float *out, uint32_t max_rays) {
    if (!s || (!out && max_rays)) return MTSG_ERR_INVALID;
    const uint32_t n = (uint32_t)(s->stragglers.size() / 8);
    for (uint32_t k = 0; k < std::min(n, max_rays); ++k) {
        const unsigned long long *w = &s->stragglers[8 * k];
        float *o = out + 12 * k;
        for (int j = 0; j < 6; ++j) {
            const uint32_t bits = (uint32_t)w[j];
            memcpy(&o[j], &bits, 4);
        }
        const uint32_t w6 = (uint32_t)w[6], w7 = (uint32_t)w[7];
        o[6] = (float)(w6 & 0x7FFFFFFFu);
        o[7] = (float)(w6 >> 31);
        o[8] = (float)(w7 & 4095u);
        o[9] = (float)((w7 >> 12) & 4095u);
        o[10] = (float)(w7 >> 24);
        o[11] = 0.0f;
    }
    return (int)n;
}

int mtsg_set_tile_callback(mtsg_scene *s, mtsg_tile_fn fn, void *user) {
    if (!s) return MTSG_ERR_INVALID;
    s->tileFn = fn;
    s->tileUser = user;
    return MTSG_OK;
}

void mtsg_cancel_clear(mtsg_scene *s) {
    if (s) s->cancel.store(0);
}

void mtsg_cancel(mtsg_scene *s) {
    if (s) s->cancel.store(1);
}

int mtsg_device_alloc(mtsg_scene *s, size_t bytes, void **out) {
    if (!s || !out) return MTSG_ERR_INVALID;
    int rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    HIP_TRY(hipMalloc(out, bytes));
    return MTSG_OK;
}
int mtsg_device_free(mtsg_scene *s, void *ptr) {
    if (!s) return MTSG_ERR_INVALID;
    int rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    HIP_TRY(hipFree(ptr));
    return MTSG_OK;
}
int mtsg_device_memset(mtsg_scene *s, void *ptr, size_t bytes) {
    if (!s) return MTSG_ERR_INVALID;
    int rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    HIP_TRY(hipMemsetAsync(ptr, 0, bytes, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MTSG_OK;
}
int mtsg_device_to_host(mtsg_scene *s, void *dst, const void *src, size_t bytes) {
    if (!s) return MTSG_ERR_INVALID;
    int rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return MTSG_OK;
}

int mtsg_render_device(mtsg_scene *s, const mtsg_render_params *p, float *film) {
    if (!s || !film) { g_err = "null argument"; return MTSG_ERR_INVALID; }
    return render_impl(s, p, film);
}

static uint32_t tile_count(const mtsg_scene *s, const mtsg_render_params *p) {
    if (!s->tileKeys.empty()) return (uint32_t)s->tileKeys.size();
    const uint32_t allTiles = (uint32_t)((p->tile_w + TILE - 1) / TILE) * (uint32_t)((p->tile_h + TILE - 1) / TILE);
    const uint32_t tstride = p->tile_stride > 1 ? (uint32_t)p->tile_stride : 1u;
    const uint32_t toffset = p->tile_stride > 1 ? (uint32_t)p->tile_offset : 0u;
    return toffset < allTiles ? (allTiles - toffset + tstride - 1) / tstride : 0u;
}

int mtsg_tile_windows(mtsg_scene *s, const mtsg_render_params *p, uint32_t *ntiles, int32_t *window) {
    if (!s || !ntiles || !window) { g_err = "null argument"; return MTSG_ERR_INVALID; }
    int rc;
    if ((rc = validate(p, s)) != MTSG_OK) return rc;
    *ntiles = tile_count(s, p);
    *window = TILE + 2 * s->cam.border;
    return MTSG_OK;
}

int mtsg_set_tile_list(mtsg_scene *s, const int32_t *keys, uint32_t n) {
    if (!s || (n && !keys)) { g_err = "null argument"; return MTSG_ERR_INVALID; }
    std::vector<int32_t> k(keys, keys + n), sorted(k);
    std::sort(sorted.begin(), sorted.end());
    for (uint32_t i = 0; i < n; ++i)
        if (sorted[i] < 0 || (i && sorted[i] == sorted[i - 1])) {
            g_err = "tile list: deal keys must be distinct and non-negative";
            return MTSG_ERR_INVALID;
        }
    int rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    if (n > s->tileKeysCap) {
        if (s->tileKeysDev) hipFree(s->tileKeysDev);
        s->tileKeysDev = nullptr;
        s->tileKeysCap = 0;
        HIP_TRY(hipMalloc((void **)&s->tileKeysDev, n * sizeof(int32_t)));
        s->tileKeysCap = n;
    }
    if (n) HIP_TRY(hipMemcpy(s->tileKeysDev, k.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
    s->tileKeys.swap(k);
    return MTSG_OK;
}

int mtsg_render_device_tiles(mtsg_scene *s, const mtsg_render_params *p, float *windows) {
    if (!s || !windows) { g_err = "null argument"; return MTSG_ERR_INVALID; }
    return render_impl(s, p, windows, TILE + 2 * s->cam.border);
}

int mtsg_render(mtsg_scene *s, const mtsg_render_params *p, float *rgbaw_out) {
    if (!s || !rgbaw_out) { g_err = "null argument"; return MTSG_ERR_INVALID; }
    int rc;
    if ((rc = validate(p, s)) != MTSG_OK) return rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    const size_t bytes = (size_t)(p->tile_w + 2 * s->cam.border) * (p->tile_h + 2 * s->cam.border) * 5 * sizeof(float);
    float *film = nullptr;
    HIP_TRY(hipMalloc((void **)&film, bytes));
    hipError_t e = hipMemsetAsync(film, 0, bytes, s->stream);
    if (e != hipSuccess) { hipFree(film); g_err = hipGetErrorString(e); return MTSG_ERR_DEVICE; }
    rc = render_impl(s, p, film);
    if (rc == MTSG_OK) {
        e = hipMemcpy(rgbaw_out, film, bytes, hipMemcpyDeviceToHost);
        if (e != hipSuccess) { g_err = hipGetErrorString(e); rc = MTSG_ERR_DEVICE; }
    }
    hipFree(film);
    return rc;
}

int mtsg_render_samples(mtsg_scene *s, const mtsg_render_params *p, float *L_out) {
    if (!s || !L_out) { g_err = "null argument"; return MTSG_ERR_INVALID; }
    s->dumpL = L_out;
    int rc = mtsg_render(s, p, std::vector<float>((size_t)(p->tile_w + 2 * s->cam.border) * (p->tile_h + 2 * s->cam.border) * 5).data());
    s->dumpL = nullptr;
    return rc;
}

// Ray queries run the production traversal kernel (the one the integrator
// launches, selected by traceMode) over a work list of n rays.
static int trace_rays(mtsg_scene *s, uint32_t n, const float *rays, float *t, float *u, float *v, uint32_t *prim,
                      uint8_t *occ, bool shadow) {
    if (!s || (!rays && n)) return MTSG_ERR_INVALID;
    if (n == 0) return MTSG_OK;
    int rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    std::vector<float4> a(n), b(n), c(shadow ? n : 0);
    for (uint32_t i = 0; i < n; ++i) {
        const float *r = rays + 8 * (size_t)i;   // o.xyz, d.xyz, mint, maxt
        if (shadow) {
            a[i] = make_float4(r[0], r[1], r[2], r[7]);
            b[i] = make_float4(r[3], r[4], r[5], r[6]);
            uint32_t tgt = 0x80000000u | i;
            float ft;
            memcpy(&ft, &tgt, 4);
            c[i] = make_float4(1.f, 0.f, 0.f, ft);   // unoccluded -> L[i].x = 1
        } else {
            a[i] = make_float4(r[0], r[1], r[2], r[6]);
            b[i] = make_float4(r[3], r[4], r[5], r[7]);
        }
    }
    std::vector<float4> out(n, make_float4(INFINITY, 0.f, 0.f, 0.f));
    if (!shadow) {
        const uint32_t miss = 0xFFFFFFFFu;
        for (auto &o : out) memcpy(&o.w, &miss, 4);
    } else {
        for (auto &o : out) o = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    DevPaths D{};
    std::vector<void *> mem;
    auto cleanup = [&]() { for (void *m : mem) hipFree(m); };
    const size_t f4 = (size_t)n * sizeof(float4);
    auto alloc = [&](void **ptr, size_t bytes, const void *src) -> hipError_t {
        hipError_t e = hipMalloc(ptr, bytes);
        if (e != hipSuccess) return e;
        mem.push_back(*ptr);
        return src ? hipMemcpy(*ptr, src, bytes, hipMemcpyHostToDevice) : hipMemset(*ptr, 0, bytes);
    };
    float4 **pa = shadow ? &D.sh_o : &D.ray_o, **pb = shadow ? &D.sh_d : &D.ray_d, **po = shadow ? &D.L : &D.hit;
    hipError_t e = alloc((void **)pa, f4, a.data());
    if (e == hipSuccess) e = alloc((void **)pb, f4, b.data());
    if (e == hipSuccess) e = alloc((void **)po, f4, out.data());
    if (e == hipSuccess && shadow) e = alloc((void **)&D.sh_c, f4, c.data());
    if (e == hipSuccess && s->ds.inst) e = alloc((void **)&D.hitInst, (size_t)n * sizeof(uint32_t), nullptr);
    if (e == hipSuccess && !shadow) e = alloc((void **)&D.tie, (size_t)n * sizeof(uint32_t), nullptr);
    if (e == hipSuccess) e = alloc((void **)&D.cnt, CNT_WORDS * sizeof(uint32_t), nullptr);
    if (e == hipSuccess) e = alloc((void **)&D.ctr, CTR_WORDS * sizeof(unsigned long long), nullptr);
    if (e == hipSuccess && shadow) e = hipMemcpy(D.cnt + CNT_S0, &n, sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) { g_err = hipGetErrorString(e); cleanup(); return MTSG_ERR_DEVICE; }
    if (shadow) launch_trace(s, false, D, -2, 0, 0u, s->stream);
    else launch_trace(s, false, D, -1, -1, n, s->stream);
    e = hipStreamSynchronize(s->stream);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out.data(), *po, f4, hipMemcpyDeviceToHost);
    uint32_t err = 0;
    if (e == hipSuccess) e = hipMemcpy(&err, D.cnt + CNT_ERR, sizeof(uint32_t), hipMemcpyDeviceToHost);
    cleanup();
    if (e != hipSuccess) { g_err = hipGetErrorString(e); return MTSG_ERR_DEVICE; }
    if (err & CNT_ERR_TRAVERSAL) { g_err = traversal_error; return MTSG_ERR_TRAVERSAL; }
    for (uint32_t i = 0; i < n; ++i) {
        if (shadow) {
            occ[i] = out[i].x == 0.f ? 1 : 0;
        } else {
            uint32_t pb2;
            memcpy(&pb2, &out[i].w, 4);
            prim[i] = pb2;   // triangle index, 0x80000000 | rectangle index, or ~0 (miss)
            t[i] = out[i].x; u[i] = out[i].y; v[i] = out[i].z;
        }
    }
    return MTSG_OK;
}

int mtsg_env_eval(mtsg_scene *s, uint32_t n, const float *dirs, const float *rx, const float *ry, float *out) {
    if (!s || (!dirs && n) || (!out && n) || ((rx == nullptr) != (ry == nullptr))) { g_err = "invalid arguments"; return MTSG_ERR_INVALID; }
    if (!s->ds.has_env) { g_err = "scene has no environment emitter"; return MTSG_ERR_INVALID; }
    if (n == 0) return MTSG_OK;
    int rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    const size_t bytes = (size_t)n * 3 * sizeof(float);
    float *dd = nullptr, *dx = nullptr, *dy = nullptr, *dout = nullptr;
    auto cleanup = [&]() { hipFree(dd); hipFree(dx); hipFree(dy); hipFree(dout); };
    hipError_t e = hipMalloc((void **)&dd, bytes);
    if (e == hipSuccess) e = hipMalloc((void **)&dout, bytes);
    if (e == hipSuccess && rx) e = hipMalloc((void **)&dx, bytes);
    if (e == hipSuccess && ry) e = hipMalloc((void **)&dy, bytes);
    if (e == hipSuccess) e = hipMemcpy(dd, dirs, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && rx) e = hipMemcpy(dx, rx, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && ry) e = hipMemcpy(dy, ry, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_env_eval, dim3((n + 255) / 256), dim3(256), 0, s->stream, s->ds, dd, dx, dy, n, dout);
        e = hipStreamSynchronize(s->stream);
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
    cleanup();
    if (e != hipSuccess) { g_err = hipGetErrorString(e); return MTSG_ERR_DEVICE; }
    return MTSG_OK;
}

int mtsg_tex_eval(mtsg_scene *s, int tex, uint32_t n, const float *uv, const float *duv, float *out) {
    if (!s || (!uv && n) || (!out && n)) { g_err = "invalid arguments"; return MTSG_ERR_INVALID; }
    if (tex < 0 || (uint32_t)tex >= s->nTextures) { g_err = "texture index out of range"; return MTSG_ERR_INVALID; }
    if (n == 0) return MTSG_OK;
    int rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    float *duv_d = nullptr, *dd = nullptr, *dout = nullptr;
    auto cleanup = [&]() { hipFree(duv_d); hipFree(dd); hipFree(dout); };
    hipError_t e = hipMalloc((void **)&dd, (size_t)n * 2 * sizeof(float));
    if (e == hipSuccess) e = hipMalloc((void **)&dout, (size_t)n * 3 * sizeof(float));
    if (e == hipSuccess && duv) e = hipMalloc((void **)&duv_d, (size_t)n * 4 * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(dd, uv, (size_t)n * 2 * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess && duv) e = hipMemcpy(duv_d, duv, (size_t)n * 4 * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_tex_eval, dim3((n + 255) / 256), dim3(256), 0, s->stream, s->ds, tex, dd, duv_d, n, dout);
        e = hipStreamSynchronize(s->stream);
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * 3 * sizeof(float), hipMemcpyDeviceToHost);
    cleanup();
    if (e != hipSuccess) { g_err = hipGetErrorString(e); return MTSG_ERR_DEVICE; }
    return MTSG_OK;
}

int mtsg_om_query(mtsg_scene *s, uint32_t n, const float *dirs, const float *o1, const float *o2, int32_t *ids, int32_t *vis) {
    if (!s || (n && (!dirs || !o1 || !o2 || !ids || !vis))) { g_err = "invalid arguments"; return MTSG_ERR_INVALID; }
    if (!s->ds.om) { g_err = "scene has no occupancy maps"; return MTSG_ERR_INVALID; }
    if (n == 0) return MTSG_OK;
    int rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    const size_t fb = (size_t)n * 3 * sizeof(float), ib = (size_t)n * sizeof(int32_t);
    float *dd = nullptr, *d1 = nullptr, *d2 = nullptr;
    int32_t *di = nullptr, *dv = nullptr;
    auto cleanup = [&]() { hipFree(dd); hipFree(d1); hipFree(d2); hipFree(di); hipFree(dv); };
    hipError_t e = hipMalloc((void **)&dd, fb);
    if (e == hipSuccess) e = hipMalloc((void **)&d1, fb);
    if (e == hipSuccess) e = hipMalloc((void **)&d2, fb);
    if (e == hipSuccess) e = hipMalloc((void **)&di, ib);
    if (e == hipSuccess) e = hipMalloc((void **)&dv, ib);
    if (e == hipSuccess) e = hipMemcpy(dd, dirs, fb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d1, o1, fb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d2, o2, fb, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_om_query, dim3((n + 255) / 256), dim3(256), 0, s->stream, s->ds, dd, d1, d2, n, di, dv);
        e = hipStreamSynchronize(s->stream);
    }
    if (e == hipSuccess) e = hipMemcpy(ids, di, ib, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(vis, dv, ib, hipMemcpyDeviceToHost);
    cleanup();
    if (e != hipSuccess) { g_err = hipGetErrorString(e); return MTSG_ERR_DEVICE; }
    return MTSG_OK;
}

}  // extern "C"

namespace mtsg {
void set_last_error(const std::string &e) { g_err = e; }   // kdbuild.hip
}

namespace {
__global__ void k_sampler_draws(DevIntegrator I, int x, int y, uint32_t s, uint32_t n, const int32_t *kinds, float *out,
                                int *err) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    PathSampler p = path_sampler(I, x, y, s, 0, 0);
    for (uint32_t i = 0; i < n; ++i) {
        const int t = I.smp.type;
        if (kinds[i] == 2) {
            float a, b;
            if (t == MTSG_SAMPLER_HALTON) next2D<MTSG_SAMPLER_HALTON>(I, p, a, b);
            else if (t == MTSG_SAMPLER_HAMMERSLEY) next2D<MTSG_SAMPLER_HAMMERSLEY>(I, p, a, b);
            else if (t == MTSG_SAMPLER_LDSAMPLER) next2D<MTSG_SAMPLER_LDSAMPLER>(I, p, a, b);
            else if (t == MTSG_SAMPLER_SOBOL) next2D<MTSG_SAMPLER_SOBOL>(I, p, a, b);
            else next2D<MTSG_SAMPLER_INDEPENDENT>(I, p, a, b);
            *out++ = a;
            *out++ = b;
        } else {
            float a;
            if (t == MTSG_SAMPLER_HALTON) a = next1D<MTSG_SAMPLER_HALTON>(I, p);
            else if (t == MTSG_SAMPLER_HAMMERSLEY) a = next1D<MTSG_SAMPLER_HAMMERSLEY>(I, p);
            else if (t == MTSG_SAMPLER_LDSAMPLER) a = next1D<MTSG_SAMPLER_LDSAMPLER>(I, p);
            else if (t == MTSG_SAMPLER_SOBOL) a = next1D<MTSG_SAMPLER_SOBOL>(I, p);
            else a = next1D<MTSG_SAMPLER_INDEPENDENT>(I, p);
            *out++ = a;
        }
    }
    *err = p.dimError ? 1 : 0;
}
}  // namespace

extern "C" {

int mtsg_sampler_draws(mtsg_scene *s, const mtsg_render_params *p, int x, int y, uint32_t si, uint32_t n,
                       const int32_t *kinds, float *out) {
    if (!s || !p || (n && (!kinds || !out)) || p->spp == 0) { g_err = "invalid arguments"; return MTSG_ERR_INVALID; }
    if (n == 0) return MTSG_OK;
    int rc;
    if ((rc = set_device(s)) != MTSG_OK) return rc;
    uint32_t nOut = 0;
    for (uint32_t i = 0; i < n; ++i) nOut += kinds[i] == 2 ? 2 : 1;
    DevIntegrator I{p->max_depth, p->rr_depth, p->strict_normals, p->hide_emitters, p->spp, p->seed,
                    (uint32_t)s->cam.film_w, make_sampler(s, p->spp)};
    int32_t *dk = nullptr;
    float *dout = nullptr;
    int *derr = nullptr;
    auto cleanup = [&]() { hipFree(dk); hipFree(dout); hipFree(derr); };
    hipError_t e = hipMalloc((void **)&dk, n * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&dout, nOut * sizeof(float));
    if (e == hipSuccess) e = hipMalloc((void **)&derr, sizeof(int));
    if (e == hipSuccess) e = hipMemcpy(dk, kinds, n * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_sampler_draws, dim3(1), dim3(64), 0, s->stream, I, x, y, si, n, dk, dout, derr);
        e = hipStreamSynchronize(s->stream);
    }
    int err = 0;
    if (e == hipSuccess) e = hipMemcpy(out, dout, nOut * sizeof(float), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(&err, derr, sizeof(int), hipMemcpyDeviceToHost);
    cleanup();
    if (e != hipSuccess) { g_err = hipGetErrorString(e); return MTSG_ERR_DEVICE; }
    if (err) {
        g_err = dim_error(s->samplerType);
        return MTSG_ERR_INVALID;
    }
    return MTSG_OK;
}

int mtsg_trace_closest(mtsg_scene *s, uint32_t n, const float *rays, float *t, float *u, float *v, uint32_t *prim) {
    return trace_rays(s, n, rays, t, u, v, prim, nullptr, false);
}

int mtsg_trace_shadow(mtsg_scene *s, uint32_t n, const float *rays, uint8_t *occluded) {
    return trace_rays(s, n, rays, nullptr, nullptr, nullptr, nullptr, occluded, true);
}

void mtsg_scene_destroy(mtsg_scene *s) {
    if (!s) return;
    hipSetDevice(s->device);
    if (s->stream) hipStreamSynchronize(s->stream);
    free_batch(s);
    for (void *p : s->allocs) hipFree(p);
    for (hipEvent_t e : s->evPool) hipEventDestroy(e);
    if (s->hostCnt) hipHostFree(s->hostCnt);
    if (s->waveTimes) hipFree(s->waveTimes);
    for (int l = 1; l < MTSG_MAX_LANES; ++l)
        if (s->lstream[l]) hipStreamDestroy(s->lstream[l]);
    if (s->stream) hipStreamDestroy(s->stream);
    if (s->tileKeysDev) hipFree(s->tileKeysDev);
    delete s;
}

void mtsg_last_error(char *buf, size_t size) {
    if (!buf || !size) return;
    strncpy(buf, g_err.c_str(), size - 1);
    buf[size - 1] = 0;
}

}  // extern "C"
