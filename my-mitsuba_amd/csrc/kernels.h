// kernels.h -- device code of the MI355X wavefront path tracer (see mtsg.hip).
// Included by mtsg.hip (host side, traversal, camera, splat) and by
// smp_kernels.hip, which is compiled once per sampler and instantiates the
// shading kernels (k_shade, k_finish) for it: the translation units build in
// parallel.  Device functions live in an anonymous namespace (each unit has
// its own copy); the launch-interface structs and the per-sampler launchers
// have external linkage in namespace mtsg.
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "../../include/mtsg.h"
#include "device_math.h"
#include "envmap.h"
#include "sampler.h"

namespace mtsg {

// ---------------------------------------------------------------------------
// device-side scene and path state
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// device-side scene and path state
// ---------------------------------------------------------------------------
struct DevCamera;
struct DevScene {
    // device kd-tree (built from Mitsuba's KDNode array at upload: same splits
    // and leaves, re-laid out as two-level blocks).  A block root's 64-B block
    // holds {children pair, left child's pair, right child's pair, pad}, so one
    // fetch descends two levels.  Node words (8 B):
    //   leaf            1 << 31 | start, end   (range of triL records)
    //   block root      axis | block << 3, split
    //   pair-only node  axis | 4 | slot << 3, split  (slot = 4 * block + 1|2, uint4 units)
    const uint4 *__restrict__ blocks;
    uint2 root2;
    const float4 *__restrict__ triL;       // TriAccel records in leaf order (3 float4 each)
    const float4 *__restrict__ vpos;       // xyz
    const float4 *__restrict__ vnrm;       // xyz
    const uint4 *__restrict__ tidx;        // i0, i1, i2, shape
    // per-triangle shading record, 6 float4 (96 B, one contiguous fetch per hit):
    //   p0 p1 p2 | n0 n1 n2 | dpdu | shape, bsdf | faceNormals << 31, emitter
    const float4 *__restrict__ shrec;
    const mtsg_rect *__restrict__ rects;
    // per rectangle its to_object rows as 3 float4 (48 B, the size of a
    // TriAccel record): MTSG_RECT_PEND reads them through the primitive slot
    const float4 *__restrict__ rectM;
    // per rectangle its shading data, 2 float4 (one fetch per hit instead of
    // the rectangle, then its shape): {frame_n, shape}, {dpdu, bsdf | (emitter + 1) << 16}
    const float4 *__restrict__ rectSh;
    // per emitter 4 float4: a rectangle's to_world rows, then {frame_n, shape
    // type}; the sampling of a rectangle emitter reads only these
    const float4 *__restrict__ emitRect;
    const mtsg_shape *__restrict__ shapes;
    const mtsg_bsdf *__restrict__ bsdfs;
    const mtsg_emitter *__restrict__ emitters;
    const float *__restrict__ emitter_cdf;
    const float *__restrict__ emitter_tri_cdf;
    uint32_t n_emitters, n_tri, n_bsdfs;
    float bmin[3], bmax[3];
    int has_env;
    DevEnv env;
    // halton / hammersley tables (sampler.h); nullptr for the other samplers
    const uint32_t *qmcPrimes, *qmcOff;
    const uint16_t *qmcPerm;
    // two-level instancing (instance.cpp:115-160): per instance 8 float4 =
    // to_local rows 0-2, to_world rows 0-2, {group AABB min, root word 0},
    // {group AABB max, root word 1}; the group trees live in `blocks` / `triL`
    // beside the top-level tree.  nullptr: no instances.
    const float4 *__restrict__ inst;
    // bitmap textures (mipmap.h): headers, texels, and per triangle 3 float4
    // {uv0, uv1 | uv2, dpdv.xy | dpdv.z} for the lookups; nullptr: none
    const mtsg_texture *__restrict__ textures;
    const float *__restrict__ tex_texels;
    const float4 *__restrict__ ttex;
    int cam_diffs;        // bounce 0 carries the camera's ray differentials in T / aux
                          // (filtered texture lookups; MTSG_OPT_CAMERA_DIFFS 1)
    // environment scenes otherwise: a camera ray that misses recomputes its
    // differentials at bounce 0 from the camera (camera_differentials), so
    // k_camera writes and bounce 0 reads 32 B less per path (round 6)
    int cam_env_diffs;
    const DevCamera *__restrict__ camDev;
    float camO[3], camNear, camFar;   // the camera's origin and clip distances (load_closest_ray)
    int camCompact;   // k_camera stores ray_d = (direction, 1/z) only (flat scenes: load_closest_ray)
    // two-level traversal: per-lane save slots of the top-level state
    // (SAVE_VECS uint4 per lane of the traversal grid); nullptr: no instances
    uint4 *__restrict__ instSave;
    // myPath2_OM occupancy maps (om.cpp; nullptr unless that integrator)
    const mtsg_om *__restrict__ om;
    const uint32_t *__restrict__ om_bits;
    // traversal stacks in use (<= SHORT_STACK / INNER_STACK / OUTER_STACK;
    // smaller only to exercise the restart guard) and the restart guard:
    // from restart rstGuard of a ray (per level) on, a restart starts one ulp
    // beyond its exit distance; restart rstMax (rstMaxC for closest-hit
    // rays) ends the ray with SB_ERR
    uint32_t capFlat, capGrp, capTop, rstGuard, rstMax, rstMaxC;
    uint32_t instPrefilter;   // test knob: 0 = the two-level world-box prefilter off (KNOBS kernels only)
    // two-level exact-tie keys: key + (instance + 1) * instKeyStride, where
    // the stride is the number of TriAccel keys when keys x (instances + 1)
    // fit 32 bits (one key per (primitive, instance) pair, no collisions)
    uint32_t instKeyStride;
};

struct DevCamera {
    float s2c[16];
    float c2w[12];
    float near_clip, far_clip, inv_res_x, inv_res_y;
    int film_w, film_h;
    float filter_radius, filter_scale;
    int border, has_alpha;
    float filter_values[32];
    float dx[3], dy[3];   // near-plane differentials (perspective.cpp:160-170)
    int diffs;            // store primary-ray differentials (environment / filtered texture lookups)
    int compact;          // store ray_d = (direction, 1/z) only (DevScene::camCompact)
    int crop_w, crop_h;   // the sampler's space partition (setFilmResolution)
};

struct DevIntegrator {
    int max_depth, rr_depth, strict_normals, hide_emitters;
    uint32_t spp, seed;
    uint32_t film_w;   // sample id = (y * film_w + x) * spp + s
    DevSampler smp;
    int om, om_strategy, om_mis, om_jitter;   // myPath2_OM (mtsg_render_params)
};

// wavefront batch: tiles [tile0, tile0 + ntiles) x samples [s0, s0 + ns)
struct DevBatch {
    int rect_x, rect_y, rect_w, rect_h;   // render rectangle (film coords)
    int tiles_x;                          // tiles per row of the rectangle
    int tile0, ntiles;                    // virtual tile range of this batch
    int tstride, toffset;                 // deal key = toffset + virtual * tstride (tile_of_key)
    int skew;                             // deal: row ty rotated by ty * skew tiles (always 1)
    uint32_t s0, ns;
    uint32_t nslots;
    const int32_t *keys;                  // mtsg_set_tile_list: deal key of virtual tile v = keys[v] (device); null: arithmetic
};
// deal key of virtual tile v of a call
__host__ __device__ inline int batch_key(const DevBatch &B, int v) { return B.keys ? B.keys[v] : B.toffset + v * B.tstride; }

// Multi-GPU tile deal (mtsg_render_params.tile_stride / tile_offset): tile
// (tx, ty) of the rectangle's tile grid has the deal key ty * tiles_x +
// (tx - ty) mod tiles_x, and a call renders the tiles whose key % stride ==
// offset.  Rotating row ty by ty tiles turns the column stripes that a plain
// row-major deal gives when the stride divides tiles_x (C3: 80 tiles per row,
// 2/4/8 ranks) into diagonal stripes, so every rank's share samples every
// column of the frame: the eight 1/8 C3 shares were 22.1-23.2 ms apart as
// columns (round 3, profiles/r03_bench_c4_e8.json).
__host__ __device__ inline void tile_of_key(int key, int tiles_x, int &tx, int &ty, int skew = 1) {
    ty = key / tiles_x;
    tx = (key % tiles_x + (ty * skew) % tiles_x) % tiles_x;
}

// Path state.  The paths of a bounce are stored densely by their position in
// that bounce's work list (the camera's slot order at bounce 0, then the order
// in which k_shade appended the surviving paths), so every kernel streams its
// state with coalesced 16-B accesses instead of gathering it through a queue of
// slot indices.  k_shade writes the survivors into the n_* arrays at their new
// position; the host swaps the two sets after each bounce.  Only the final
// radiance is kept per sample slot (L, written when a path terminates).
struct DevPaths {
    float4 *ray_o;    // o.xyz, mint
    float4 *ray_d;    // d.xyz, maxt
    float4 *T;        // throughput rgb, eta        (bounce 0: x-differential direction)
    float4 *aux;      // refN.xyz of the previous vertex, bsdf pdf (bounce 0: y-differential)
    float4 *Lp;       // radiance so far, alpha
    uint4 *meta;      // depth | flags, next RNG dimension, sample slot, 0
    float4 *n_ray_o, *n_ray_d, *n_T, *n_aux, *n_Lp;   // next bounce (compacted)
    uint4 *n_meta;
    float4 *hit;      // t, u, v, prim (bits) of ray i
    uint32_t *hitInst;   // instance of hit i (0xFFFFFFFF: none); two-level scenes only
    uint32_t *tie;       // closest rays of a trace launch that met an exact tie (cnt[CNT_TIE] of them)
    float4 *L;        // per sample slot: final radiance, alpha (k_splat input)
    float4 *sh_o;     // shadow ray i: origin, maxt
    float4 *sh_d;     // direction, mint
    float4 *sh_c;     // NEE contribution, target (bits): next-bounce position, or 1 << 31 | slot
    uint32_t *cnt;    // counters, each on its own 256-B line (see CNT_*)
    unsigned long long *ctr;  // traversal counters (nodes, refs, tests)
    // closest rays of a trace launch in ray order (k_sortwin): work-list entry
    // i is the ray at position order[i]; nullptr: entry i is position i
    uint32_t *order;
    uint32_t *orderBuf;   // the buffer k_sortwin fills (one entry per path)
    // 1 while the closest rays are bounce 0's camera rays of a flat scene,
    // which k_camera stores as ray_d = (direction, 1/z) only: their origin is
    // the camera's and mint / maxt are near / far clip x 1/z (load_closest_ray,
    // DevScene::camCompact; round 6)
    uint32_t camEnc = 0;
};

// arguments of the per-sampler shading launchers (smp_kernels.hip)
struct ShadeLaunch {
    dim3 grid, block;
    hipStream_t stream;
    const DevScene *S;
    const DevIntegrator *I;
    const DevBatch *B;
    const DevPaths *P;
    int bounce, qin;
    uint32_t nIdentity;
    int hasAlpha;
    uint32_t shadeMin;   // k_finish
    bool env, ext, inst;   // inst: two-level instancing (k_finish<.., INST>)
    int mats;              // the scene's material classes (MAT_*), or MATS_ALL
};
template <int SMP> void launch_shade_smp(const ShadeLaunch &a);
template <int SMP> void launch_finish_smp(const ShadeLaunch &a);
#define MTSG_DECLARE_LAUNCHERS(SMP) \
    template <> void launch_shade_smp<SMP>(const ShadeLaunch &a); \
    template <> void launch_finish_smp<SMP>(const ShadeLaunch &a);
MTSG_DECLARE_LAUNCHERS(MTSG_SAMPLER_INDEPENDENT)
MTSG_DECLARE_LAUNCHERS(MTSG_SAMPLER_HALTON)
MTSG_DECLARE_LAUNCHERS(MTSG_SAMPLER_HAMMERSLEY)
MTSG_DECLARE_LAUNCHERS(MTSG_SAMPLER_LDSAMPLER)
MTSG_DECLARE_LAUNCHERS(MTSG_SAMPLER_SOBOL)
int finish_blocks_per_cu(bool mats);   // k_finish workgroups per CU (occupancy query)
// the flat traversal and its tie retrace (trace_flat.hip, its own translation
// unit and scheduler flags): one launch over a work list, then k_tie if `tie`
struct FlatTraceLaunch {
    dim3 grid, tieGrid;
    hipStream_t stream;
    const DevScene *S;
    const DevPaths *P;
    int cIn, sIn;
    uint32_t n;
    unsigned long long *wt;
    bool count, knobs, refill32, tie;
};
void launch_trace_flat(const FlatTraceLaunch &a);
int trace_flat_blocks_per_cu();   // k_trace_s<false, 16> workgroups per CU (occupancy query)

}  // namespace mtsg

using namespace mtsg;

namespace {
constexpr uint32_t KINST = 4u;   // leaf-ordered TriAccel copy of an instance primitive: k = 4



// a path's sampler at sample s of film pixel (x, y), `dim` dimensions and
// `n2` 2D requests into the path
DEV PathSampler path_sampler(const DevIntegrator &I, int x, int y, uint32_t s, uint32_t dim, uint32_t n2) {
    const uint64_t pix = (uint64_t)y * (uint64_t)I.film_w + (uint64_t)x;
    PathSampler p{counterKey(I.seed, pix * I.spp + s), dim, n2, s, x, y, false, 0ull};
    if (I.smp.type == MTSG_SAMPLER_SOBOL) p.qidx = sobol_index(I.smp, s, x, y);
    return p;
}
DEV uint64_t pixel_index(const DevIntegrator &I, const PathSampler &p) {
    return (uint64_t)p.y * (uint64_t)I.film_w + (uint64_t)p.x;
}
template <int KIND>
DEV float next1D(const DevIntegrator &I, PathSampler &p) {
    return smp_next1D<KIND>(I.smp, p, I.seed, pixel_index(I, p), I.spp);
}
template <int KIND>
DEV void next2D(const DevIntegrator &I, PathSampler &p, float &a, float &b) {
    smp_next2D<KIND>(I.smp, p, I.seed, pixel_index(I, p), I.spp, a, b);
}
// the camera's pixel jitter: the first 2D request of a sample (the sampler is
// a run-time choice here; k_shade is instantiated per sampler)
DEV void camera_jitter(const DevIntegrator &I, int x, int y, uint32_t s, float &a, float &b) {
    PathSampler p = path_sampler(I, x, y, s, 0, 0);
    switch (I.smp.type) {
        case MTSG_SAMPLER_HALTON: next2D<MTSG_SAMPLER_HALTON>(I, p, a, b); break;
        case MTSG_SAMPLER_HAMMERSLEY: next2D<MTSG_SAMPLER_HAMMERSLEY>(I, p, a, b); break;
        case MTSG_SAMPLER_LDSAMPLER: next2D<MTSG_SAMPLER_LDSAMPLER>(I, p, a, b); break;
        case MTSG_SAMPLER_SOBOL: next2D<MTSG_SAMPLER_SOBOL>(I, p, a, b); break;
        default: next2D<MTSG_SAMPLER_INDEPENDENT>(I, p, a, b); break;
    }
}
// (the same for a caller that knows the sampler: the shading kernels)
template <int SMP>
DEV void camera_jitter_smp(const DevIntegrator &I, int x, int y, uint32_t s, float &a, float &b) {
    PathSampler p = path_sampler(I, x, y, s, 0, 0);
    next2D<SMP>(I, p, a, b);
}


enum : uint32_t { F_SCATTERED = 1u << 16, F_DELTA = 1u << 17 };


// queue / fetch counters live on separate 256-byte lines: a single
// contended address serialises at ~11 ns per atomic (MI355X_MICROARCH.md,
// row "dequeue"), and counters sharing a line would serialise together
constexpr int XGROUPS = 8;                  // XCDs: blocks b and b + 8 share one
// Q0/Q1: paths of the next bounce (ping-pong); S0/S1: shadow rays of a bounce
// (ping-pong: bounce b appends to S(b & 1) while its trace reads S((b-1) & 1))
constexpr int CNT_Q0 = 0, CNT_Q1 = 64, CNT_S0 = 128, CNT_S1 = 192;
constexpr int CNT_ERR = 96;   // sticky error flags (CNT_ERR_*)
constexpr int CNT_TIE = 224;  // entries of P.tie (k_trace_s appends, k_tie reads)
constexpr uint32_t CNT_ERR_QMC_DIM = 1u, CNT_ERR_TRAVERSAL = 2u;
constexpr int CNT_FETCH = 256;                           // XGROUPS counters, 32 words apart
constexpr int CNT_WORDS = CNT_FETCH + 32 * XGROUPS;
constexpr int HOSTCNT_STRIDE = 256;
// traversal counters (MTSG_FLAG_COUNT): [0,7) closest, [8,15) shadow (see
// flush_counts), 7 / 15 the maximum iterations per ray, [16,32) / [32,48)
// histograms of floor(log2(iterations per ray)); [48] the number of captured
// stragglers (rays of >= STRAGGLER_ITERS iterations), [64, 64 + 8 * 64) their
// records (o.xyz, d.xyz, iterations, shadow as float / integer bits)
constexpr int CTR_WORDS = 64 + 8 * 64;
constexpr uint32_t STRAGGLER_ITERS = 300, STRAGGLER_MAX = 64;
constexpr uint32_t WT_MAX_LAUNCHES = 64;   // MTSG_FLAG_WAVETIME launches recorded per render
// MTSG_FLAG_WAVETIME words per wave: start, exit, time the work list was found
// empty, loop iterations after that
constexpr uint32_t WT_WORDS = 4;
#ifndef MTSG_WT_DRAIN
#define MTSG_WT_DRAIN 0   // record words 2-3 (diagnostic builds: the bookkeeping costs ~4% in the hot loop)
#endif
constexpr bool WT_DRAIN = MTSG_WT_DRAIN;
__host__ __device__ constexpr int cnt_s(int k) { return k ? CNT_S1 : CNT_S0; }
DEV int cnt_q(int q) { return q ? CNT_Q1 : CNT_Q0; }

constexpr int TILE = 16;                    // splat tile edge (256 pixels)
constexpr int BLOCK = 256;
#ifndef MTSG_SHADE_BLOCK
#define MTSG_SHADE_BLOCK 256
#endif
constexpr int SHADE_BLOCK = MTSG_SHADE_BLOCK;   // k_shade workgroup size
constexpr int TRACE_BLOCK = 64;             // one wave per workgroup for traversal
// Paths per wavefront batch (272 B of state per path; 2^28 paths = 73 GB
// of the 288 GB HBM, capped at 60% of free device memory at run time).
// Every traversal launch ends with a tail of ~0.5-0.8 ms while its longest
// rays finish, and late bounces hold few paths, so the batch should be as
// large as the frame -- measured on the 1M-triangle scene (Msamples/s):
// 4M paths 421, 16M 672, 32M 803, 64M 884, 128M 934, whole frame 960.
// 3 * 2^28 paths = 225 GB of path state at most (r04: 2^29, C5 in 4 batches
// instead of 8: +2.5%; r06: C5 in 3 batches of 713M paths, 200 GB, instead of
// 4: +1.1%, profiles/r06_c5_batches.txt -- every batch pays its own tail of
// small bounce launches); capped by the free HBM (render_impl)
constexpr uint32_t DEFAULT_BATCH_PATHS = 3u << 28;
#define MTSG_MAX_LANES 4
#ifndef MTSG_LANES
#define MTSG_LANES 1
#endif
constexpr size_t PATH_STATE_BYTES = 280;    // bytes per path slot (DevPaths: 2 x 96 dense + hit, L, 3 x shadow, tie, order)
#ifndef MTSG_SHORT_STACK
#define MTSG_SHORT_STACK 6   // 6 x 12 B x 64 lanes = 4.6 KB LDS/wave -> 8 waves/SIMD (8: 6.5, 12: 4.2)
#endif
constexpr int SHORT_STACK = MTSG_SHORT_STACK;   // LDS short stack entries per lane
// two-level traversal (kernels.h spec_iter_i): the top level's stack, and the
// group level's own, as deep as the flat traversal's: 6 x 12 B + 2 x 12 B per
// lane = 6 KB per wave, 6.6 waves/SIMD (the kernel runs 6, register bound).
// 6 entries measured 1.2% faster than 5 on C3-two-level (r03 variants gs6).
constexpr int OUTER_STACK = 2;
#ifndef MTSG_INNER_STACK
#define MTSG_INNER_STACK 6
#endif
constexpr int INNER_STACK = MTSG_INNER_STACK;
// the compact speculative traversal is sized for 8 waves per SIMD (64 VGPRs)
#ifndef MTSG_SPEC_WAVES
#define MTSG_SPEC_WAVES 8
#endif
#define SPEC_ATTR __launch_bounds__(TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(MTSG_SPEC_WAVES)))
// the two-level kernel runs 6 waves/SIMD: at 7 (72 VGPRs) the compiler spills
// 20 B/lane to scratch; with the registers of 6 (80) it does not, and C3
// renders 13% faster (1043 vs 920 Msamples/s, round 3).  Its LDS (group stack
// + top-level stack, 6 KB/wave) allows 6.6 waves/SIMD.
#ifndef MTSG_INST_WAVES
#define MTSG_INST_WAVES 6
#endif
// streaming (non-temporal) access to the per-path SoA state: the state of a
// 32M-path batch is GBs per bounce and would otherwise evict the kd-tree from
// the 256 MB Infinity Cache (experiment switch MTSG_NT)
#ifndef MTSG_NT
#define MTSG_NT 1
#endif
typedef float nf4 __attribute__((ext_vector_type(4)));
DEV float4 ldS(const float4 *p) {
#if MTSG_NT
    const nf4 v = __builtin_nontemporal_load((const nf4 *)p);
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
DEV void stS(float4 *p, const float4 &v) {
#if MTSG_NT
    __builtin_nontemporal_store((nf4){v.x, v.y, v.z, v.w}, (nf4 *)p);
#else
    *p = v;
#endif
}
typedef uint32_t nu4 __attribute__((ext_vector_type(4)));
DEV uint4 ldS(const uint4 *p) {
#if MTSG_NT
    const nu4 v = __builtin_nontemporal_load((const nu4 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
DEV void stS(uint4 *p, const uint4 &v) {
#if MTSG_NT
    __builtin_nontemporal_store((nu4){v.x, v.y, v.z, v.w}, (nu4 *)p);
#else
    *p = v;
#endif
}

// ---------------------------------------------------------------------------
// wave helpers (64 lanes)
// ---------------------------------------------------------------------------
DEV uint32_t lane_id() { return __lane_id(); }

// ---------------------------------------------------------------------------
// primitive tests
// ---------------------------------------------------------------------------
// TriAccel::rayIntersect (triaccel.h:96-158)
DEV bool tri_test(const float4 f0, const float4 f1, const float4 f2, float3 o, float3 d, float mint, float maxt,
                  float &u, float &v, float &t) {
    // no FMA contraction: bit-identical t, u, v to the oracle (and Mitsuba's SSE2 build)
#pragma clang fp contract(off)
    const uint32_t k = __float_as_uint(f0.x);
    // (u, v, k) = (1,2,0) | (2,0,1) | (0,1,2): a rotation of (x, y, z) by k, so
    // two compares and two selects per component (k >= 3 never hits)
    const bool k0 = k == 0u, k1 = k == 1u;
    const float o_k = k0 ? o.x : (k1 ? o.y : o.z), d_k = k0 ? d.x : (k1 ? d.y : d.z);
    const float o_u = k0 ? o.y : (k1 ? o.z : o.x), d_u = k0 ? d.y : (k1 ? d.z : d.x);
    const float o_v = k0 ? o.z : (k1 ? o.x : o.y), d_v = k0 ? d.z : (k1 ? d.x : d.y);
    const float n_u = f0.y, n_v = f0.z, n_d = f0.w;
    // branch-free on purpose: with an early `t` rejection the compiler sinks
    // the loads of f1/f2 behind it, turning one 48-byte fetch into two or
    // three dependent memory round trips per primitive
    t = (n_d - o_u * n_u - o_v * n_v - o_k) / (d_u * n_u + d_v * n_v + d_k);
    const float hu = o_u + t * d_u - f1.x;
    const float hv = o_v + t * d_v - f1.y;
    u = hv * f1.z + hu * f1.w;
    v = hu * f2.x + hv * f2.y;
    return (t >= mint) & (t <= maxt) & (u >= 0) & (v >= 0) & (u + v <= 1.0f) & (k < 3);
}

// Rectangle::rayIntersect (rectangle.cpp:115-139)
DEV bool rect_test_m(const float *m, float3 wo, float3 wd, float mint, float maxt, float &t, float &lx, float &ly) {
#pragma clang fp contract(off)
    float3 o = mk3(m[0] * wo.x + m[1] * wo.y + m[2] * wo.z + m[3], m[4] * wo.x + m[5] * wo.y + m[6] * wo.z + m[7],
                   m[8] * wo.x + m[9] * wo.y + m[10] * wo.z + m[11]);
    float3 d = mk3(m[0] * wd.x + m[1] * wd.y + m[2] * wd.z, m[4] * wd.x + m[5] * wd.y + m[6] * wd.z,
                   m[8] * wd.x + m[9] * wd.y + m[10] * wd.z);
    // Rectangle::rayIntersect's early returns as one condition (no exec-mask
    // branches); t / lx / ly are written either way and read only on a hit
    const float hit = -o.z / d.z;
    const float x = o.x + d.x * hit, y = o.y + d.y * hit;
    t = hit;
    lx = x;
    ly = y;
    return (hit >= mint) & (hit <= maxt) & (fabsf(x) <= 1.0f) & (fabsf(y) <= 1.0f);
}
DEV bool rect_test(const mtsg_rect &r, float3 wo, float3 wd, float mint, float maxt, float &t, float &lx, float &ly) {
    return rect_test_m(r.to_object, wo, wd, mint, maxt, t, lx, ly);
}
// the same test on to_object rows already in registers (MTSG_RECT_PEND)
DEV bool rect_test_rows(float4 r0, float4 r1, float4 r2, float3 wo, float3 wd, float mint, float maxt, float &t, float &lx,
                        float &ly) {
    const float m[12] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w};
    return rect_test_m(m, wo, wd, mint, maxt, t, lx, ly);
}

// ---------------------------------------------------------------------------
// kd-tree traversal (ShapeKDTree::rayIntersectHavran, sahkdtree3.h:246-358):
// t-interval front-to-back order with an LDS short stack and kd-restart when
// the short stack has overflowed (Horn et al. 2007).  Finds the same closest
// primitive as the Havran loop: every leaf overlapping the ray segment is
// visited until the best hit lies before the current leaf's exit distance
// (sahkdtree3.h:299-300).
// ---------------------------------------------------------------------------
// Algorithmic work (per lane) and, for the SIMD-efficiency figures, the
// wave-level iteration counts (accumulated by lane 0 only): a wave pays
// max-over-lanes of the inner-node and primitive iterations of every step.
struct TraceCounts { uint32_t nodes, refs, tests, wnodes, wtests, wsteps, wactive, restarts, inst; };   // restarts: not flushed

template <bool COUNT>
DEV void flush_counts(unsigned long long *ctr, TraceCounts c) {
    if (!COUNT) return;
    // wave reduction then one atomic per counter per wave
    unsigned long long v[7] = {c.nodes, c.refs, c.tests, c.wnodes, c.wtests, c.wsteps, c.wactive};
#pragma unroll
    for (int k = 0; k < 7; ++k)
        for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_down(v[k], off);
    if (lane_id() == 0)
#pragma unroll
        for (int k = 0; k < 7; ++k) atomicAdd(ctr + k, v[k]);
}

#ifndef MTSG_FETCH
#define MTSG_FETCH 128
#endif
constexpr uint32_t FETCH = MTSG_FETCH;
#ifndef MTSG_GUIDE
#define MTSG_GUIDE 0
#endif
#ifndef MTSG_FETCH_MIN
#define MTSG_FETCH_MIN 64
#endif
#ifndef MTSG_GUIDE_SPLIT
#define MTSG_GUIDE_SPLIT 2
#endif
constexpr bool GUIDE = MTSG_GUIDE;
constexpr uint32_t FETCH_MIN = MTSG_FETCH_MIN, GUIDE_SPLIT = MTSG_GUIDE_SPLIT;

// XCD-partitioned work fetch: the queue is cut into XGROUPS contiguous
// ranges; workgroup b draws from range b % XGROUPS first (blocks b, b + 8
// share an XCD, so coherent neighbouring rays share that XCD's L2) and then
// steals from the other ranges.  Each range has its own fetch counter on its
// own cache line (a contended word serialises at ~11 ns per atomic).
struct Fetch {
    uint32_t *ctr;
    uint32_t count;
    uint32_t group;    // range currently drained (wave-uniform)
    uint32_t tried;
    uint32_t guide;    // waves per range x GUIDE_SPLIT
    uint32_t req;      // next request size (GUIDE)
    DEV uint32_t lo(uint32_t g) const { return (uint32_t)(((uint64_t)count * g) / XGROUPS); }
    // returns false when every range is exhausted; else [base, base + n)
    DEV bool next(uint32_t want, uint32_t &base, uint32_t &n) {
        while (tried < XGROUPS) {
            const uint32_t beg = lo(group), end = lo(group + 1);
            // called with the whole wave active: lane 0 draws for it
            uint32_t off = 0;
            if (GUIDE) want = req;
            if (__lane_id() == 0) off = atomicAdd(&ctr[32 * group], want);
            off = __builtin_amdgcn_readfirstlane(off);
            if (beg + off < end) {
                base = beg + off;
                n = min(want, end - base);
                // guided self-scheduling: size the next request by what this
                // draw saw left of the range (no extra access to the
                // contended counter), so the last pools are small and the
                // waves run out of work together
                if (GUIDE) req = max(FETCH_MIN, min(FETCH, (end - base - n) / guide));
                return true;
            }
            group = (group + 1) % XGROUPS;
            ++tried;
        }
        return false;
    }
};

// unoccluded shadow ray i: its contribution goes to the path's radiance, at
// the path's position in the current bounce (the trace runs after the swap)
// or, if the path ended, to its sample's final slot
DEV void shadow_unoccluded(const DevPaths &P, uint32_t i) {
    const float4 con = ldS(&P.sh_c[i]);
    const uint32_t tgt = __float_as_uint(con.w);
    float4 *L = (tgt & 0x80000000u) ? &P.L[tgt & 0x7FFFFFFFu] : &P.Lp[tgt];
    float4 v = ldS(L);
    v.x += con.x; v.y += con.y; v.z += con.z;
    stS(L, v);
}

// Debug entry point: environment radiance along directions (rx/ry null:
// bilinear level-0 lookup; else EWA with those differential directions)
__global__ void k_env_eval(DevScene S, const float *dirs, const float *rx, const float *ry, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float3 d = mk3(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
    const bool diff = rx != nullptr;
    const float3 x = diff ? mk3(rx[3 * i], rx[3 * i + 1], rx[3 * i + 2]) : d;
    const float3 y = diff ? mk3(ry[3 * i], ry[3 * i + 1], ry[3 * i + 2]) : d;
    const float3 v = env_eval(S.env, d, diff, x, y);
    out[3 * i] = v.x; out[3 * i + 1] = v.y; out[3 * i + 2] = v.z;
}

// BitmapTexture::eval(uv) / eval(uv, d0, d1) (bitmap.cpp:431-499) of texture
// `tex`, for the parity tests (mtsg_tex_eval)
__global__ void k_tex_eval(DevScene S, int tex, const float *uv, const float *duv, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const DevMip M{&S.textures[tex].mip, S.tex_texels};
    const float u = uv[2 * i], v = uv[2 * i + 1];
    float3 r;
    if (duv) r = mip_filtered(M, u, v, duv[4 * i], duv[4 * i + 1], duv[4 * i + 2], duv[4 * i + 3]);
    else r = M.M->filter == MTSG_MIP_NEAREST ? mip_box(M, 0, u, v) : mip_bilinear(M, 0, u, v);
    out[3 * i] = r.x; out[3 * i + 1] = r.y; out[3 * i + 2] = r.z;
}

// ---------------------------------------------------------------------------
// Speculative traversal with compact per-lane state: each iteration issues
// one node fetch and one primitive fetch per lane, testing the leaf it holds
// while descending towards the next one.  Stack counters, direction signs and
// flags are packed in one word and hit records are written through on every
// hit (u, v and the primitive index are not kept live): 64 VGPRs, 8 waves/SIMD.
// ---------------------------------------------------------------------------
struct SpecRay {
    float3 o, d, inv;
    float mint, best;    // primitive-test interval (best shrinks with hits)
    float tmin, tmax;    // traversal interval of r.cur
    uint2 cur;           // traversal node (two-level encoding)
    uint32_t lfE, lfEnd; // primitive range of the held leaf
    float lfTmax;        // exit distance of the held leaf; < 0: none held
    uint32_t bits;       // see SB_*
    uint32_t mb;         // mailbox state of exact ties (mailbox_step)
    uint32_t bestKey;    // TriAccel index of the best hit (mailbox key)
    uint32_t rpend;      // MTSG_RECT_PEND: the rectangle tested in the lane's next iteration
    uint2 rroot;         // MTSG_PUSHDOWN: the node a kd-restart starts from
};
// bits: top slot of the circular short stack (0-2), entries held (3-5),
// entries dropped since the last restart (6), kd-restarts of the ray at this
// level (7-15), ray direction signs (16-18), traversal done (19), hit found
// (20), shadow ray (21), inside an instance (22), an exact tie met (23),
// a rectangle pending (25, MTSG_RECT_PEND), restart limit hit (31)
enum : uint32_t {
    SB_TOP = 7u, SB_N = 7u << 3, SB_N1 = 1u << 3, SB_DROPPED = 1u << 6, SB_STACK = 0x7Fu,
    SB_RST_SHIFT = 7, SB_RST1 = 1u << 7, SB_RST_MASK = 0x1FFu,
    SB_DNEG = 16, SB_TRAVDONE = 1u << 19, SB_FOUND = 1u << 20, SB_SHADOW = 1u << 21, SB_TIE = 1u << 23,
    SB_RPEND = 1u << 25, SB_ERR = 1u << 31
};
// the restart guard's defaults (DevScene::rstGuard / rstMax): rays of the
// scenes at hand restart 0-3 times (tools/iter_hist.py)
constexpr uint32_t RST_GUARD = 8, RST_MAX = SB_RST_MASK;

// stack capacities and restart limits of a traversal: compile-time constants
// in the production kernels (KNOBS = false), the scene's test overrides
// (DevScene::capFlat ...) in the KNOBS instantiations
struct TravLimits { uint32_t capFlat, capGrp, capTop, rstGuard, rstMax, rstMaxC; bool prefilter; };
template <bool KNOBS>
DEV TravLimits trav_limits(const DevScene &S) {
    if (KNOBS) return TravLimits{S.capFlat, S.capGrp, S.capTop, S.rstGuard, S.rstMax, S.rstMaxC, S.instPrefilter != 0};
    return TravLimits{(uint32_t)SHORT_STACK, (uint32_t)INNER_STACK, (uint32_t)OUTER_STACK, RST_GUARD, RST_MAX, RST_MAX, true};
}

// kd-restart after the stack ran empty with entries dropped (Foley &
// Sugerman's restart, at the exit distance t0 of the leaf just finished).
// It can only return to t0 when more far children are pushed at split
// planes crossed exactly at t0 than the stack holds; from the rstGuard-th
// restart of the ray on it starts one ulp beyond t0 instead (hits exactly at
// t0 in leaves not yet visited are the only thing that can be skipped), so
// t0 strictly increases, and the rstMax-th restart ends the ray with SB_ERR
// (the render then fails with MTSG_ERR_TRAVERSAL) instead of spinning.
#ifndef MTSG_RST_GUARD
#define MTSG_RST_GUARD 1   // 0: measurement variant without the guard (round-2 restart)
#endif
DEV void kd_restart(const TravLimits &L, SpecRay &r, uint32_t b, uint2 root, uint2 c) {
#if !MTSG_RST_GUARD
    {
        const bool restart = (b & SB_DROPPED) != 0;
        const float t0 = r.tmax;
        r.tmin = restart ? t0 : r.tmin;
        r.tmax = restart ? r.best : r.tmax;
        r.cur = restart ? root : c;
        r.bits = (b & ~SB_STACK) | ((!restart | !(t0 < r.best)) ? SB_TRAVDONE : 0u);
        return;
    }
#endif
    const bool restart = (b & SB_DROPPED) != 0;
    float t0 = r.tmax;
    uint32_t nb = b & ~SB_STACK;
#if MTSG_POPSEL
    // selects, no exec-mask branches
    const uint32_t nr = (b >> SB_RST_SHIFT) & SB_RST_MASK;
    const bool limit = nr >= ((b & SB_SHADOW) ? L.rstMax : L.rstMaxC);   // the limit (the counter saturates)
    nb = restart ? (limit ? (nb | SB_ERR | SB_TRAVDONE) : nb + SB_RST1) : nb;
    // the guard: nextafterf(t0, +inf) for finite t0, in integer arithmetic
    const uint32_t u = __float_as_uint(t0);
    const float tg = __uint_as_float(t0 >= 0.0f ? (u & 0x7FFFFFFFu) + 1u : u - 1u);
    t0 = (restart & (nr >= L.rstGuard)) ? tg : t0;
#else
    if (restart) {   // lanes that restart (the others finish their ray here)
        const uint32_t nr = (b >> SB_RST_SHIFT) & SB_RST_MASK;
        if (nr >= ((b & SB_SHADOW) ? L.rstMax : L.rstMaxC)) nb |= SB_ERR | SB_TRAVDONE;   // the limit (the counter saturates)
        else nb += SB_RST1;
        if (nr >= L.rstGuard) {
            // nextafterf(t0, +inf) for finite t0, in integer arithmetic
            const uint32_t u = __float_as_uint(t0);
            t0 = __uint_as_float(t0 >= 0.0f ? (u & 0x7FFFFFFFu) + 1u : u - 1u);
        }
    }
#endif
    r.tmin = restart ? t0 : r.tmin;
    r.tmax = restart ? r.best : r.tmax;
    r.cur = restart ? root : c;
    r.bits = nb | ((!restart | !(t0 < r.best)) ? SB_TRAVDONE : 0u);
}

// short stack of the compact traversal: entry k of lane i at [k * TRACE_BLOCK
// + i].  A workgroup is one wave, so the lane index is recomputed at every use
// (v_mbcnt) instead of holding a register through the traversal loop.
static_assert(TRACE_BLOCK == 64, "one wave per traversal workgroup");
__shared__ uint2 s_specNode[SHORT_STACK * TRACE_BLOCK];
__shared__ float s_specT[SHORT_STACK * TRACE_BLOCK];
#ifndef MTSG_LDS_TOP
#define MTSG_LDS_TOP 0
#endif
#if MTSG_LDS_TOP
__shared__ uint4 s_top[20];
#endif
// every kernel that runs spec_iter stages the top blocks first (variant only)
#ifndef MTSG_LDS_PAD
#define MTSG_LDS_PAD 0   // measurement: bytes of unused LDS per traversal workgroup (caps its occupancy)
#endif
#if MTSG_LDS_PAD
__shared__ uint32_t s_ldsPad[MTSG_LDS_PAD / 4];
#endif
DEV void lds_top_init(const DevScene &S) {
#if MTSG_LDS_TOP
    if (threadIdx.x < 20u) s_top[threadIdx.x] = S.blocks[threadIdx.x];
    __syncthreads();
#endif
#if MTSG_LDS_PAD
    if (threadIdx.x == 0) ((volatile uint32_t *)s_ldsPad)[(S.n_tri & 0xFFFFu) % (MTSG_LDS_PAD / 4)] = 0u;
#endif
}
// lane index, recomputed where it is used (volatile: not hoisted out of loops)
DEV uint32_t lane_here() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
// number of set bits of a wave mask below this lane
DEV uint32_t rank_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
struct SpecStack {
    DEV static uint32_t at(uint32_t k) { return k * TRACE_BLOCK + lane_here(); }
    DEV void push(uint32_t k, uint2 node, float t) const {
        const uint32_t i = at(k);
        s_specNode[i] = node;
        s_specT[i] = t;
    }
    DEV uint2 node(uint32_t k) const { return s_specNode[at(k)]; }
    DEV float t(uint32_t k) const { return s_specT[at(k)]; }
};

// constant 4-vector built at its use (keeps the compiler from holding it in
// registers across the traversal loop)
DEV float4 miss_record() {
    float4 m;
    uint32_t inf = 0x7F800000u, z = 0u, ff = 0xFFFFFFFFu;
    asm volatile("" : "+v"(inf), "+v"(z), "+v"(ff));
    m.x = __uint_as_float(inf); m.y = __uint_as_float(z); m.z = __uint_as_float(z); m.w = __uint_as_float(ff);
    return m;
}

// Ray setup: scene-AABB clip (AABB::rayIntersect, aabb.h:308-338) and the
// adaptive epsilon of ShapeKDTree::rayIntersect / rayIntersect for shadow
// rays (skdtree.cpp:112-142 / 207-226).  Returns false when the ray misses
// the scene bounds or its interval is empty.
DEV bool spec_init(const DevScene &S, float3 o, float3 d, float rayMint, float rayMaxt, bool shadow, SpecRay &r) {
    r.o = o;
    r.d = d;
    r.inv = mk3(rcp_exact(d.x), rcp_exact(d.y), rcp_exact(d.z));
    const uint32_t dneg = (d.x <= 0.0f ? 1u : 0u) | (d.y <= 0.0f ? 2u : 0u) | (d.z <= 0.0f ? 4u : 0u);
    float nearT = -INFINITY, farT = INFINITY;
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        // the two cases of aabb.h:308-338 as selects (no exec-mask branches)
        const float oi = comp(o, i), di = comp(d, i), ii = comp(r.inv, i);
        const bool par = di == 0.0f;
        const float t1 = (S.bmin[i] - oi) * ii, t2 = (S.bmax[i] - oi) * ii;
        nearT = par ? nearT : fmaxf(fminf(t1, t2), nearT);
        farT = par ? farT : fminf(fmaxf(t1, t2), farT);
        ok &= !par | ((oi >= S.bmin[i]) & (oi <= S.bmax[i]));
    }
    if (!ok || !(nearT <= farT)) return false;
    // the adaptive epsilon as a select (skdtree.cpp:112-142 / 207-226)
    float m = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    if (!shadow) m = fmaxf(m, kEpsilon);
    const float rayMinT = rayMint == kEpsilon ? rayMint * m : rayMint;
    r.mint = fmaxf(nearT, rayMinT);
    r.best = fminf(farT, rayMaxt);
    if (!(r.best > r.mint)) return false;
    r.tmin = r.mint;
    r.tmax = r.best;
    r.cur = S.root2;
    r.rroot = S.root2;
    r.lfE = r.lfEnd = 0;
    r.lfTmax = -1.0f;
    r.bits = dneg << SB_DNEG | (shadow ? SB_SHADOW : 0u);
    r.mb = 0;
    r.bestKey = 0xFFFFFFFFu;   // no best yet (a first hit exactly at a finite maxt is flagged
                              // and traced again with the mailbox: the same answer)
    return true;
}

// inner-node step with the packed short-stack counters (as kd_descend), split
// in two: spec_plan needs only the node word (axis, split), so the child to
// visit is known before the node's children are fetched; spec_take applies it.
DEV void spec_plan(const SpecRay &r, uint2 n, float &tsplit, bool &goLeft, bool &push) {
    const uint32_t axis = n.x & 3u;
    const float split = __uint_as_float(n.y);
    const bool a0 = axis == 0u, a1 = axis == 1u;
    const float ox = r.o.x, oy = r.o.y, oz = r.o.z, ix = r.inv.x, iy = r.inv.y, iz = r.inv.z;
    const float oa = a0 ? ox : (a1 ? oy : oz);
    const float ia = a0 ? ix : (a1 ? iy : iz);
    tsplit = (split - oa) * ia;
    if (tsplit != tsplit) tsplit = INFINITY;
    // bitwise, not short-circuit: no exec-mask branches for these
    const bool belowFirst = (oa < split) | ((oa == split) & (bool)((r.bits >> (SB_DNEG + axis)) & 1u));
    const bool onlyFirst = (tsplit > r.tmax) | (tsplit <= 0.0f);
    const bool goSecond = !onlyFirst & (tsplit < r.tmin);
    push = !onlyFirst & !goSecond;
    goLeft = belowFirst != goSecond;
}

// Push-down (Horn et al. 2007, "Interactive k-d tree GPU raytracing"): while
// nothing is held on the stack and nothing was dropped, a descent step that enters
// one child only leaves the ray's whole remaining segment inside that child,
// so a later kd-restart can start there instead of at the root.  It takes the
// same one-sided steps the root restart would (its interval [t0, best] lies
// inside the one the step was decided on), so the leaves and their order do
// not change; only the re-descent is shorter.
#ifndef MTSG_PUSHDOWN
#define MTSG_PUSHDOWN 0   // measured r04: C3 trace +1.6%, C5 +2.5% (2 more VGPRs and a compare per step for 0.08 restarts per ray)
#endif
DEV uint2 spec_take(SpecRay &r, const uint4 &pr, float tsplit, bool goLeft, bool push, SpecStack stk, uint32_t cap) {
    const uint2 c = goLeft ? make_uint2(pr.x, pr.y) : make_uint2(pr.z, pr.w);
#if MTSG_PUSHDOWN
    // (nothing held and nothing dropped: after drops the segment beyond the
    // popped subtrees still belongs to the restart, which keeps its node)
    if (!push && !(r.bits & (SB_N | SB_DROPPED))) r.rroot = c;
#endif
    if (push) {
        // circular short stack: a push onto a full stack drops the oldest entry
        const uint2 other = goLeft ? make_uint2(pr.z, pr.w) : make_uint2(pr.x, pr.y);
        const uint32_t b = r.bits, top = b & SB_TOP;
        stk.push(top, other, r.tmax);
        const bool full = (b & SB_N) == cap * SB_N1;
        r.bits = ((b & ~SB_TOP) | (top == cap - 1 ? 0u : top + 1u)) + (full ? SB_DROPPED - (b & SB_DROPPED) : SB_N1);
        r.tmax = tsplit;
    }
    return c;
}

// Mitsuba's mailbox on exact ties.  Its leaf loop skips a primitive still in
// the 8-entry direct-mapped mailbox (slot = TriAccel index & 7, written by
// every test: sahkdtree3.h:30-32,138-152,277-291) and accepts a hit at t <=
// the best distance, so of primitives hit at exactly the same t the winner is
// the one tested last, retests of still-boxed primitives not counting.  Only
// a tie can tell a retest from a first test (a retested primitive hits at the
// t it hit before, which can only equal the best), and the only retests that
// could change the winner are of the best and of the best it displaced at the
// same t ("prev"), so instead of the 8 entries the lane keeps which slots
// have been written since each of the two was boxed (r.mb): bits 0-7 since
// the best, 8-15 since prev, 16 prev exists, 17-19 prev's slot, 20-22 the
// best's slot; prev's identity in LDS, the best's in its hit record.  Exact for
// ties of two primitives; of three or more, a retest of the earliest one after
// the later two is accepted where Mitsuba may skip it.
// a rectangle met in a leaf is tested in the lane's next iteration, its rows
// read through the primitive slot (no dependent fetch inside an iteration):
// flat traversal (MTSG_RECT_PEND, measured r04: C3 trace -0.7%, but C5 trace
// +3%: the 4 more VGPRs and the address select cost every iteration, off) and
// two-level (MTSG_RECT_PEND_I, measured r04: 3% slower, off)
#ifndef MTSG_RECT_PEND
#define MTSG_RECT_PEND 0
#endif
#ifndef MTSG_RECT_PEND_I
#define MTSG_RECT_PEND_I 0
#endif
// batched instance entry and exit (two-level, spec_iter_i), measured r05 on
// C3 two-level: entry when >= 1/2, 1/4, 1/8, 1/16 of the busy lanes pend:
// 1064 / 1153 / 1157-1160 / 1143 vs 1119-1123 unbatched; exit batching on top
// of entry at 1/8: 1070-1085 (the exit block is cheap, the waits are not)
#ifndef MTSG_ENTER_BATCH
#define MTSG_ENTER_BATCH 8
#endif
#ifndef MTSG_POPSEL
#define MTSG_POPSEL 0   // measurement: stack pop / kd-restart as selects in the flat traversal
#endif
#ifndef MTSG_INST_MIN_IDLE
#define MTSG_INST_MIN_IDLE 16   // two-level traversal: idle lanes that trigger a refill (flat: 16)
#endif
#ifndef MTSG_EXIT_BATCH
#define MTSG_EXIT_BATCH 0
#endif
#ifndef MTSG_MAILBOX
#define MTSG_MAILBOX 1   // 0: measurement variant, the last primitive tested wins a tie
#endif
// flat traversal: a tie's retrace runs in the lane that met it, inside the
// trace launch (round 6), instead of in a k_tie launch after every trace launch
#ifndef MTSG_TIE_INLINE
#define MTSG_TIE_INLINE 0   // measured r06: C3 trace +4.4 ms (64 VGPRs at the 8-wave limit), C2 +6.4 ms, C5 +40 ms: off
#endif
constexpr bool TIE_INLINE = MTSG_TIE_INLINE;
__shared__ uint32_t s_mbPrev[TRACE_BLOCK];
// the tie branch of mailbox_step (mb: the state before this test)
DEV bool mailbox_tie(SpecRay &r, uint32_t mb, uint32_t sl, uint32_t id, const float4 *hitOut) {
    if (!(r.bits & SB_FOUND)) return true;   // a first hit exactly at the far end of the interval
    const uint32_t bs = (mb >> 20) & 7u, ps = (mb >> 17) & 7u;
    const uint32_t bestId = ((const uint32_t *)hitOut)[3];
    if (id == bestId) {
        // the best itself: skipped if boxed, else retested (same hit) and re-boxed
        r.mb = (mb & ~(1u << bs)) | (0x100u << bs);
        return false;
    }
    if ((mb & 0x10000u) && id == s_mbPrev[lane_here()] && !(mb & (0x100u << ps))) {
        r.mb = mb;   // prev, still boxed
        return false;
    }
    // tested for the first time or evicted: the tie winner; the best it
    // displaces becomes prev (boxed unless its slot was written since)
    s_mbPrev[lane_here()] = bestId;
    r.mb = sl << 20 | bs << 17 | 0x10000u | ((mb & 0xFFu) | (1u << sl)) << 8;
    return true;
}
// one primitive test's mailbox bookkeeping (key: its TriAccel index, tag:
// slot << 20 | 0x101 << slot): a miss ors in the low half (the slot written,
// in both masks), a closer hit keeps only the slot (a new best, just boxed);
// ties take the branch
DEV bool mailbox_step(SpecRay &r, uint32_t key, bool isRect, uint32_t prim, bool h, float t, const float4 *hitOut) {
    const uint32_t mb = r.mb, tag = (key & 7u) << 20 | 0x101u << (key & 7u);
    r.mb = h ? (tag & 0x700000u) : ((tag & 0xFFFFu) | mb);
    if (h & (t == r.best)) h = mailbox_tie(r, mb, tag >> 20, isRect ? (0x80000000u | prim) : prim, hitOut);
    return h;
}

template <bool COUNT, bool MB = false>
DEV bool spec_iter(const DevScene &S, SpecRay &r, SpecStack stk, TraceCounts &cnt, float4 *hitOut, const TravLimits &L) {
    const uint2 n = r.cur;
    const bool inner = !(r.bits & SB_TRAVDONE) && !(n.x & 0x80000000u);
    const bool prim = r.lfE < r.lfEnd;
    const bool rootKind = inner && !(n.x & 4u);
    // the first step is planned from the node word alone, so only the pair
    // of the grandchildren on the side taken is fetched (block root: {children,
    // left grandchildren, right grandchildren})
    float tsplit;
    bool goLeft, push;
    spec_plan(r, n, tsplit, goLeft, push);
    // block root: 64-B block n.x >> 3; pair-only node: 16-B pair n.x >> 3
    const uint32_t base = inner ? (n.x >> 3) << ((~n.x >> 1) & 2u) : 0u;
    const uint32_t off = rootKind ? 2u - (uint32_t)goLeft : 0u;
    const uint32_t pi = prim ? r.lfE : 0u;
#if MTSG_LDS_TOP
    // measurement variant: the top four levels (blocks 0-4, mtsg.hip layout)
    // from LDS; a lane's global fetch is skipped when its node is there
    uint4 p0, pc;
    if (base < 20u) p0 = s_top[base]; else p0 = S.blocks[base];
    if (base + off < 20u) pc = s_top[base + off]; else pc = S.blocks[base + off];
#else
    const uint4 p0 = S.blocks[base], pc = S.blocks[base + off];
#endif
#if MTSG_RECT_PEND
    // a rectangle met in the held leaf is tested in the lane's next
    // iteration, its to_object rows read through the primitive slot: no
    // dependent fetch of the rectangle inside an iteration
    const bool rp = (r.bits & SB_RPEND) != 0;
    const float4 *rec = rp ? S.rectM + (size_t)(3u * r.rpend) : S.triL + (size_t)(3u * pi);
#else
    const float4 *rec = S.triL + (size_t)(3u * pi);   // < 2^32: checked at upload
#endif
    const float4 f0 = rec[0], f1 = rec[1], f2 = rec[2];
    asm volatile("" ::"v"(p0.x), "v"(p0.y), "v"(p0.z), "v"(p0.w), "v"(pc.x), "v"(pc.y), "v"(pc.z), "v"(pc.w),
                 "v"(f0.x), "v"(f0.y), "v"(f0.z), "v"(f0.w),
                 "v"(f1.x), "v"(f1.y), "v"(f1.z), "v"(f1.w), "v"(f2.x), "v"(f2.y), "v"(f2.z), "v"(f2.w));
#if MTSG_RECT_PEND
    if (prim && !rp && __float_as_uint(f0.x) == MTSG_TRIACCEL_SHAPE) {
        r.rpend = __float_as_uint(f2.w);
        r.bits |= SB_RPEND;
    } else if (prim) {
        if (COUNT) { cnt.refs++; cnt.tests++; }
        float t, u, v;
        const bool isRect = rp;
        bool h;
        uint32_t key, pid;
        if (rp) {
            h = rect_test_rows(f0, f1, f2, r.o, r.d, r.mint, r.best, t, u, v);
            key = S.n_tri + r.rpend;
            pid = r.rpend;
            r.bits &= ~SB_RPEND;
        } else {
            h = tri_test(f0, f1, f2, r.o, r.d, r.mint, r.best, u, v, t);
            key = __float_as_uint(f2.z);
            pid = __float_as_uint(f2.w);
        }
#else
    if (prim) {
        if (COUNT) { cnt.refs++; cnt.tests++; }
        float t, u, v;
        bool h = tri_test(f0, f1, f2, r.o, r.d, r.mint, r.best, u, v, t);
        const bool isRect = __float_as_uint(f0.x) == MTSG_TRIACCEL_SHAPE;
        if (isRect) h = rect_test(S.rects[__float_as_uint(f2.w)], r.o, r.d, r.mint, r.best, t, u, v);
        const uint32_t key = __float_as_uint(f2.z), pid = __float_as_uint(f2.w);
#endif
#if MTSG_MAILBOX
        // a tie is only flagged here; the ray is then traced again with the
        // mailbox (tie_retrace).  Shadow rays end at their first hit.
        // (a primitive spanning leaves is retested at the same t: not a tie)
        if (MB) h = mailbox_step(r, key, isRect, pid, h, t, hitOut);
        else r.bits |= (h & (t == r.best) & (key != r.bestKey)) ? SB_TIE : 0u;
        if (h) r.bestKey = key;
#endif
        if (h) {
            r.bits |= SB_FOUND;
            if (r.bits & SB_SHADOW) return true;   // any hit occludes
            r.best = t;
            stS(hitOut, make_float4(t, u, v, __uint_as_float(isRect ? (0x80000000u | pid) : pid)));
        }
        ++r.lfE;
    }
    if (inner) {
        if (COUNT) cnt.nodes++;
        const uint2 c = spec_take(r, p0, tsplit, goLeft, push, stk, L.capFlat);
        r.cur = c;
        if (rootKind && !(c.x & 0x80000000u)) {
            if (COUNT) cnt.nodes++;
            float ts2;
            bool gl2, push2;
            spec_plan(r, c, ts2, gl2, push2);
            r.cur = spec_take(r, pc, ts2, gl2, push2, stk, L.capFlat);
        }
    }
    const bool found = (r.bits & SB_FOUND) != 0;
    // the held leaf is finished: Havran's exit, or let the descent take over
    const bool leafDone = (r.lfTmax >= 0.0f) & (r.lfE >= r.lfEnd);
    if (leafDone & found & (r.best < r.lfTmax)) return true;
    r.lfTmax = leafDone ? -1.0f : r.lfTmax;
    const uint2 c = r.cur;
    if ((r.lfTmax < 0.0f) & !(r.bits & SB_TRAVDONE) & (bool)(c.x >> 31)) {
        // the descent reached a leaf: adopt it, then continue from the stack
        const uint32_t st = c.x & 0x7FFFFFFFu;
        const bool nonEmpty = st < c.y;
        if (!nonEmpty & found & (r.best < r.tmax)) return true;
        r.lfE = nonEmpty ? st : r.lfE;
        r.lfEnd = nonEmpty ? c.y : r.lfEnd;
        r.lfTmax = nonEmpty ? r.tmax : r.lfTmax;
        const uint32_t b = r.bits;
#if MTSG_POPSEL
        // pop the stack, or (empty) finish or kd-restart behind this leaf if
        // entries were dropped: both computed, one selected (the stack read
        // of an empty stack is a stale entry, not used)
        const bool hasN = (b & SB_N) != 0;
        const uint32_t top = b & SB_TOP, k = top == 0 ? L.capFlat - 1 : top - 1u;
        const uint2 pn = stk.node(k);
        const float pt = stk.t(k);
        SpecRay rr = r;
        if (COUNT && !hasN && (b & SB_DROPPED)) cnt.restarts++;
#if MTSG_PUSHDOWN
        kd_restart(L, rr, b, r.rroot, c);
#else
        kd_restart(L, rr, b, S.root2, c);
#endif
        r.cur = hasN ? pn : rr.cur;
        r.bits = hasN ? ((b & ~SB_TOP) | k) - SB_N1 : rr.bits;
        r.tmin = hasN ? r.tmax : rr.tmin;
        r.tmax = hasN ? fminf(pt, r.best) : rr.tmax;
#else
        if (b & SB_N) {
            const uint32_t top = b & SB_TOP, k = top == 0 ? L.capFlat - 1 : top - 1u;
            r.cur = stk.node(k);
            const float t = stk.t(k);
            r.bits = ((b & ~SB_TOP) | k) - SB_N1;
            r.tmin = r.tmax;
            r.tmax = fminf(t, r.best);
        } else {
            // empty: done, or a kd-restart behind this leaf if entries were dropped
            if (COUNT && (b & SB_DROPPED)) cnt.restarts++;
#if MTSG_PUSHDOWN
            kd_restart(L, r, b, r.rroot, c);
#else
            kd_restart(L, r, b, S.root2, c);
#endif
        }
#endif
    }
    return (r.bits & SB_TRAVDONE) && r.lfTmax < 0.0f;
}

// Closest ray idx of the work list: origin + mint, direction + maxt.  Bounce
// 0's camera rays (P.camEnc) keep only ray_d = (direction, 1/z): the origin is
// the camera's, and mint / maxt are the same products k_camera formed (near /
// far clip x 1/z), so the ray is bit for bit the one it used to store; a dead
// slot (1/z = -1) keeps a negative maxt
DEV void load_closest_ray(const DevScene &S, const DevPaths &P, uint32_t idx, bool cam, float4 &ro, float4 &rd) {
    rd = ldS(P.ray_d + idx);
    if (cam) {
        const float invZ = rd.w;
        ro = make_float4(S.camO[0], S.camO[1], S.camO[2], S.camNear * invZ);
        rd.w = S.camFar * invZ;
    } else {
        ro = ldS(P.ray_o + idx);
    }
}

// A closest-hit ray whose traversal met an exact tie (SB_TIE: a hit at the
// best distance so far) is traced again from its start with Mitsuba's mailbox
// emulated (mailbox_step): that can only change which of the tied primitives
// its hit record names.  Ties are rare (coplanar faces, shared edges), so the
// traversal loop pays one compare per test for them instead of the mailbox.
DEV void tie_retrace(const DevScene &S, SpecRay &r, SpecStack stk, const float4 ro, const float4 rd,
                     float4 *hitOut, const TravLimits &L) {
    TraceCounts tc{0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (!spec_init(S, xyz(ro), xyz(rd), ro.w, rd.w, false, r)) return;
    while (!spec_iter<false, true>(S, r, stk, tc, hitOut, L)) {}
}

// ---------------------------------------------------------------------------
// Two-level traversal (Instance::rayIntersect, instance.cpp:115-130, over the
// group's ShapeKDTree::rayIntersect, skdtree.h:431-458): the same speculative
// iterations, with a per-lane level.  An instance primitive met in a
// top-level leaf saves the top-level state (node, interval, held leaf range,
// stack counters) to LDS, transforms the ray by the instance's to_local and
// traverses the group tree on the clipped interval [max(mint, near),
// min(best, far)]; when the group traversal ends (or Havran's exit fires
// inside it) the top-level state is restored and the world-space ray is
// reloaded from the work list.  The two levels keep separate LDS stacks
// (top level: OUTER_STACK entries, group: SHORT_STACK), so a group visit
// never evicts top-level entries.  Hits are written through with the
// instance they were found in.
// ---------------------------------------------------------------------------
// the top-level state saved while a lane is inside an instance, two uint4 per
// lane: {cur.x, cur.y, tmin, tmax}, {lfE, lfEnd, lfTmax, bits}.  It lives in
// per-lane global slots (S.instSave, vector k of lane g at k * lanes + g: one
// coalesced 16-B access per vector), not in LDS, which holds only the stacks.
// The world ray is saved too (vectors 2-3: {o, d.x}, {d.y, d.z, -, -}), so
// leaving an instance reloads it from the lane's own coalesced slots instead of the
// ray gathered back from the work list through the path index: 3% faster on
// C3-two-level (r03 variants wsave).  The instance a lane is inside stays in a
// register (k_trace_s / k_finish `inst`).
#ifndef MTSG_SAVE_RAY
#define MTSG_SAVE_RAY 1
#endif
#ifndef MTSG_SAVE_INV
#define MTSG_SAVE_INV 1   // the world reciprocal direction saved too: no divisions on exit (register save:
                          // free at 80 VGPRs, C3 two-level 1102 -> 1119, r05; global slots: 2% slower, r03)
#endif
constexpr int SAVE_VECS = MTSG_SAVE_RAY ? (MTSG_SAVE_INV ? 5 : 4) : 2;
// MTSG_INST_REGSAVE=1 (the default): the saved top-level state and world ray
// stay in the lane's registers (TopSave, 14 VGPRs) instead of the global
// slots: no save / restore traffic and no load latency when a lane leaves an
// instance.  The kernel still fits 6 waves/SIMD (80 VGPRs); measured r04:
// C3 two-level 1070 -> 1164 Msamples/s (0: the round-3 global slots)
#ifndef MTSG_INST_REGSAVE
#define MTSG_INST_REGSAVE 1
#endif
struct TopSave {
#if MTSG_INST_REGSAVE
    uint4 a, b;
    float3 o, d;
#if MTSG_SAVE_INV
    float3 inv;   // variant: the world reciprocal kept (no divisions on exit; 3 more VGPRs)
#endif
#endif
};
// the two levels' stacks in one LDS array: top level in entries
// [0, OUTER_STACK), group level in [OUTER_STACK, OUTER_STACK + INNER_STACK)
__shared__ uint2 s_lvNode[(OUTER_STACK + INNER_STACK) * TRACE_BLOCK];
__shared__ float s_lvT[(OUTER_STACK + INNER_STACK) * TRACE_BLOCK];
enum : uint32_t { SB_INST = 1u << 22, SB_PEND = 1u << 24, SB_XPEND = 1u << 26, SB_MBRUN = 1u << 27 };   // inside an instance; entering one next
                                                                                  // iteration; leaving it (MTSG_EXIT_BATCH)

DEV uint4 &save_vec(const DevScene &S, uint32_t k) {
    return S.instSave[(size_t)k * (gridDim.x * TRACE_BLOCK) + blockIdx.x * TRACE_BLOCK + lane_here()];
}
// the group tree's root words of instance ii (its 8-float4 record, words 6.w / 7.w)
DEV uint2 inst_root(const DevScene &S, uint32_t ii) {
    const float4 *I = S.inst + 8 * (size_t)ii;
    return make_uint2(__float_as_uint(I[6].w), __float_as_uint(I[7].w));
}

// push the far child onto the stack of the lane's level (circular, drops
// the oldest entry when full)
DEV uint2 spec_take_i(const TravLimits &L, SpecRay &r, const uint4 &pr, float tsplit, bool goLeft, bool push) {
    const uint2 c = goLeft ? make_uint2(pr.x, pr.y) : make_uint2(pr.z, pr.w);
    if (push) {
        const uint2 other = goLeft ? make_uint2(pr.z, pr.w) : make_uint2(pr.x, pr.y);
        const uint32_t b = r.bits, top = b & SB_TOP;
        const bool inner = (b & SB_INST) != 0;
        const uint32_t cap = inner ? L.capGrp : L.capTop;
        const uint32_t i = (top + (inner ? (uint32_t)OUTER_STACK : 0u)) * TRACE_BLOCK + lane_here();
        s_lvNode[i] = other;
        s_lvT[i] = r.tmax;
        const bool full = (b & SB_N) == cap * SB_N1;
        r.bits = ((b & ~SB_TOP) | (top == cap - 1 ? 0u : top + 1u)) + (full ? SB_DROPPED - (b & SB_DROPPED) : SB_N1);
        r.tmax = tsplit;
    }
    return c;
}

// back to the top level after a group traversal: restore the saved state,
// keep the hit flag, reload the world-space ray
DEV void inst_exit(const DevScene &S, SpecRay &r, const float4 *wo, const float4 *wd, const TopSave &ts) {
    const uint32_t found = r.bits & (SB_FOUND | SB_ERR | SB_TIE);
#if MTSG_INST_REGSAVE
    const uint4 a = ts.a, b = ts.b;
    r.cur = make_uint2(a.x, a.y);
    r.tmin = __uint_as_float(a.z);
    r.tmax = __uint_as_float(a.w);
    r.lfE = b.x;
    r.lfEnd = b.y;
    r.lfTmax = __uint_as_float(b.z);
    r.bits = b.w | found;
    r.o = ts.o;
    r.d = ts.d;
#if MTSG_SAVE_INV
    r.inv = ts.inv;
#else
    r.inv = mk3(rcp_exact(ts.d.x), rcp_exact(ts.d.y), rcp_exact(ts.d.z));
#endif
#else
    const uint4 a = save_vec(S, 0), b = save_vec(S, 1);
    r.cur = make_uint2(a.x, a.y);
    r.tmin = __uint_as_float(a.z);
    r.tmax = __uint_as_float(a.w);
    r.lfE = b.x;
    r.lfEnd = b.y;
    r.lfTmax = __uint_as_float(b.z);
    r.bits = b.w | found;
#if MTSG_SAVE_RAY
    const uint4 c = save_vec(S, 2), e = save_vec(S, 3);
    const float4 ro = make_float4(__uint_as_float(c.x), __uint_as_float(c.y), __uint_as_float(c.z), 0.f);
    const float4 rd = make_float4(__uint_as_float(c.w), __uint_as_float(e.x), __uint_as_float(e.y), 0.f);
#else
    float4 ro = ldS(wo), rd = ldS(wd);
#endif
    r.o = xyz(ro);
    r.d = xyz(rd);
#if MTSG_SAVE_RAY && MTSG_SAVE_INV
    // the world reciprocal direction as saved: a wave runs this block whenever
    // any of its lanes leaves an instance, so its three IEEE divisions were
    // paid on most iterations
    const uint4 g = save_vec(S, 4);
    r.inv = mk3(__uint_as_float(e.z), __uint_as_float(e.w), __uint_as_float(g.x));
#else
    r.inv = mk3(rcp_exact(rd.x), rcp_exact(rd.y), rcp_exact(rd.z));
#endif
#endif
}

// Instance::rayIntersect (instance.cpp:115-130): the ray in group space
// (Transform::operator()(Ray), transform.h:262-278), clipped to the group
// tree's AABB; when the clipped interval is not empty the top-level state is
// saved and the lane continues in the group tree.  L0-L2: the instance's
// to_local rows, A0 / A1: the group AABB with the root words in .w
DEV bool inst_enter(SpecRay &r, TopSave &ts, const DevScene &S, uint32_t ii, float4 L0, float4 L1, float4 L2, float4 A0,
                    float4 A1) {
    const float3 o = r.o, d = r.d;   // (the library is built with -ffp-contract=off)
    const float3 lo = mk3(L0.x * o.x + L0.y * o.y + L0.z * o.z + L0.w, L1.x * o.x + L1.y * o.y + L1.z * o.z + L1.w,
                          L2.x * o.x + L2.y * o.y + L2.z * o.z + L2.w);
    const float3 ld = mk3(L0.x * d.x + L0.y * d.y + L0.z * d.z, L1.x * d.x + L1.y * d.y + L1.z * d.z,
                          L2.x * d.x + L2.y * d.y + L2.z * d.z);
    const float3 li = mk3(rcp_exact(ld.x), rcp_exact(ld.y), rcp_exact(ld.z));
    float nearT = -INFINITY, farT = INFINITY;
    bool ok = true;
    const float bmn[3] = {A0.x, A0.y, A0.z}, bmx[3] = {A1.x, A1.y, A1.z};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        // (as spec_init: the two cases as selects)
        const float oi = comp(lo, i), di = comp(ld, i), iv = comp(li, i);
        const bool par = di == 0.0f;
        const float t1 = (bmn[i] - oi) * iv, t2 = (bmx[i] - oi) * iv;
        nearT = par ? nearT : fmaxf(fminf(t1, t2), nearT);
        farT = par ? farT : fminf(fmaxf(t1, t2), farT);
        ok &= !par | ((oi >= bmn[i]) & (oi <= bmx[i]));
    }
    const float t0 = fmaxf(r.mint, nearT), t1 = fminf(r.best, farT);
    if (!(ok & (nearT <= farT) & (t1 > t0))) return false;
#if MTSG_INST_REGSAVE
    ts.a = make_uint4(r.cur.x, r.cur.y, __float_as_uint(r.tmin), __float_as_uint(r.tmax));
    ts.b = make_uint4(r.lfE, r.lfEnd, __float_as_uint(r.lfTmax), r.bits & ~SB_FOUND);
    ts.o = o;
    ts.d = d;
#if MTSG_SAVE_INV
    ts.inv = r.inv;
#endif
#else
    save_vec(S, 0) = make_uint4(r.cur.x, r.cur.y, __float_as_uint(r.tmin), __float_as_uint(r.tmax));
    save_vec(S, 1) = make_uint4(r.lfE, r.lfEnd, __float_as_uint(r.lfTmax), r.bits & ~SB_FOUND);
#if MTSG_SAVE_RAY
    save_vec(S, 2) = make_uint4(__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z), __float_as_uint(d.x));
#if MTSG_SAVE_INV
    save_vec(S, 3) = make_uint4(__float_as_uint(d.y), __float_as_uint(d.z), __float_as_uint(r.inv.x), __float_as_uint(r.inv.y));
    save_vec(S, 4) = make_uint4(__float_as_uint(r.inv.z), 0u, 0u, 0u);
#else
    save_vec(S, 3) = make_uint4(__float_as_uint(d.y), __float_as_uint(d.z), 0u, 0u);
#endif
#endif
#endif
    r.o = lo;
    r.d = ld;
    r.inv = li;
    r.tmin = t0;
    r.tmax = t1;
    r.cur = make_uint2(__float_as_uint(A0.w), __float_as_uint(A1.w));
    r.lfE = r.lfEnd = 0;
    r.lfTmax = -1.0f;
    const uint32_t dneg = (ld.x <= 0.0f ? 1u : 0u) | (ld.y <= 0.0f ? 2u : 0u) | (ld.z <= 0.0f ? 4u : 0u);
    r.bits = (r.bits & (SB_FOUND | SB_SHADOW | SB_TIE)) | SB_INST | dneg << SB_DNEG;
    return true;
}

// Prefilter of an instance primitive met in a top-level leaf: the ray's
// interval [mint, best] against the instance's world box from its record
// (f0.yzw min, f1.xyz max; mtsg.hip widens it so that it holds the group box
// with a margin far above float error).  Three quarters of the entries of C3
// two-level left an empty group-space clip (round 5, stats.instance_rejects);
// rejected here, they cost neither the pending iteration nor the entry block.
// Conservative: a ray this test rejects misses the widened box, so the exact
// clip of inst_enter would reject it as well.  An axis the ray runs parallel
// to (inv = +-inf) needs no branch: inside the slab it gives (-inf, inf),
// outside it an empty interval, and exactly on a face (0 * inf = NaN, which
// fminf / fmaxf pass over) a rejection -- of a ray that lies the margin
// outside the group box, which the exact clip rejects too.
#ifndef MTSG_INST_PREFILTER
#define MTSG_INST_PREFILTER 1
#endif
DEV bool inst_box(const SpecRay &r, float4 f0, float4 f1) {
    float t0 = r.mint, t1 = r.best;
    const float bmn[3] = {f0.y, f0.z, f0.w}, bmx[3] = {f1.x, f1.y, f1.z};
    // the slab distances round with the ray's own magnitude (|o| ulps), which
    // the box's margin (its size and position) does not bound for a small
    // instance seen from far away: widen the box by 2^-20 |o|_max (8 ulps of
    // the origin) as well, so the test stays conservative there
    const float e = 0x1p-20f * fmaxf(fmaxf(fabsf(r.o.x), fabsf(r.o.y)), fabsf(r.o.z));
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float oa = comp(r.o, a), ia = comp(r.inv, a);
        const float u = (bmn[a] - e - oa) * ia, v = (bmx[a] + e - oa) * ia;
        t0 = fmaxf(t0, fminf(u, v));
        t1 = fminf(t1, fmaxf(u, v));
    }
    return t0 <= t1;
}

// One iteration of the two-level traversal.  An instance primitive met in a
// top-level leaf is entered in the lane's NEXT iteration (SB_PEND): that
// iteration's fetch slots load the instance record (to_local rows and group
// AABB, 80 B) in place of a node pair and a primitive, so the record is not a
// dependent fetch on the leaf record inside one iteration -- in a 64-lane wave
// some lane enters an instance in almost every iteration, and the wave waited
// for that second round trip each time.  The sequence of top-level state
// transitions is unchanged (the leaf logic that followed an unsuccessful
// entry runs in the entry iteration), so hits are the same bit for bit.
template <bool COUNT>
DEV bool spec_iter_i(const DevScene &S, SpecRay &r, TraceCounts &cnt, const DevPaths &P, uint32_t idx, const TravLimits &L,
                     uint32_t &inst, TopSave &ts) {
    const uint2 n = r.cur;
#if MTSG_EXIT_BATCH
    // batched exit (as the batched entry): a lane whose group traversal ended
    // waits until 1/MTSG_EXIT_BATCH of the busy lanes have, then all of them
    // restore their top-level state together
    {
        const bool xp = (r.bits & SB_XPEND) != 0;
        const uint32_t nX = (uint32_t)__popcll(__ballot(xp)), nAll = (uint32_t)__popcll(__ballot(1));
        if (xp) {
            if (nX * MTSG_EXIT_BATCH >= nAll) {
                const bool sh = (r.bits & SB_SHADOW) != 0;
                inst_exit(S, r, (sh ? P.sh_o : P.ray_o) + idx, (sh ? P.sh_d : P.ray_d) + idx, ts);
            }
            return false;
        }
    }
#endif
    const bool pend = (r.bits & SB_PEND) != 0;
#if MTSG_ENTER_BATCH
    // batched entry: pending lanes wait until at least 1/MTSG_ENTER_BATCH of
    // the wave's busy lanes are pending (always true once no other lane is
    // busy), so the entry block (transform, clip, reciprocals, state save:
    // ~110 VALU that the wave issues whenever any lane enters) runs for
    // several lanes at once; a waiting lane fetches a cached dummy and changes
    // nothing, so every lane takes the same steps as unbatched
    const uint32_t nPend = (uint32_t)__popcll(__ballot(pend)), nBusy = (uint32_t)__popcll(__ballot(1));
    const bool waiting = pend && !(nPend * MTSG_ENTER_BATCH >= nBusy);
#else
    constexpr bool waiting = false;
#endif
    const bool inner = !pend && !(r.bits & SB_TRAVDONE) && !(n.x & 0x80000000u);
    const bool prim = !pend && r.lfE < r.lfEnd;
    const bool rootKind = inner && !(n.x & 4u);
    float tsplit;
    bool goLeft, push;
    spec_plan(r, n, tsplit, goLeft, push);
    const uint32_t base = inner ? (n.x >> 3) << ((~n.x >> 1) & 2u) : 0u;
    const uint32_t off = rootKind ? 2u - (uint32_t)goLeft : 0u;
    const uint32_t pi = prim ? r.lfE : 0u;
    // a pending entry reads the instance record through the same slots
    const float4 *irec = S.inst + 8 * (size_t)inst;
    const uint4 *a0 = pend && !waiting ? reinterpret_cast<const uint4 *>(irec + 6) : S.blocks + base;
    const uint4 *a1 = pend && !waiting ? reinterpret_cast<const uint4 *>(irec + 7) : S.blocks + base + off;
#if MTSG_RECT_PEND_I
    // a top-level rectangle is tested in the lane's next iteration (its index
    // waits in `inst`, unused at the top level: groups hold no rectangles)
    const bool rp = (r.bits & SB_RPEND) != 0;
    const float4 *rec = pend ? irec : (rp ? S.rectM + (size_t)(3u * inst) : S.triL + (size_t)(3u * pi));
#else
    const float4 *rec = pend && !waiting ? irec : S.triL + (size_t)(3u * pi);
#endif
    const uint4 p0 = *a0, pc = *a1;
    const float4 f0 = rec[0], f1 = rec[1], f2 = rec[2];
    asm volatile("" ::"v"(p0.x), "v"(p0.y), "v"(p0.z), "v"(p0.w), "v"(pc.x), "v"(pc.y), "v"(pc.z), "v"(pc.w),
                 "v"(f0.x), "v"(f0.y), "v"(f0.z), "v"(f0.w),
                 "v"(f1.x), "v"(f1.y), "v"(f1.z), "v"(f1.w), "v"(f2.x), "v"(f2.y), "v"(f2.z), "v"(f2.w));
    if (waiting) return false;
    if (pend) {
        r.bits &= ~SB_PEND;
        if (COUNT) cnt.inst++;
        const float4 A0 = make_float4(__uint_as_float(p0.x), __uint_as_float(p0.y), __uint_as_float(p0.z), __uint_as_float(p0.w));
        const float4 A1 = make_float4(__uint_as_float(pc.x), __uint_as_float(pc.y), __uint_as_float(pc.z), __uint_as_float(pc.w));
        if (inst_enter(r, ts, S, inst, f0, f1, f2, A0, A1)) return false;
        // COUNT: entries the group-box clip rejected (stats.instance_rejects)
        if (COUNT) atomicAdd(P.ctr + 58, 1ull);
        // not entered: the leaf logic below, as after the primitive step
    }
    bool enter = false;
    if (prim) {
        const uint32_t k = __float_as_uint(f0.x);
#if MTSG_RECT_PEND_I
        const bool isRect = rp, defer = !rp && k == MTSG_TRIACCEL_SHAPE;
        enter = !rp && k == KINST;
#else
        const bool isRect = k == MTSG_TRIACCEL_SHAPE, defer = false;
        enter = k == KINST;
#endif
        const bool isInst = enter;
#if MTSG_INST_PREFILTER
        if (isInst) {
            enter = !L.prefilter || inst_box(r, f0, f1);
            if (COUNT && !enter) atomicAdd(P.ctr + 59, 1ull);   // stats.instance_prefiltered
        }
#endif
        if (COUNT && !defer) cnt.refs++;
        if (defer) {
            inst = __float_as_uint(f2.w);
            r.bits |= SB_RPEND;
        } else if (!isInst) {
            if (COUNT) cnt.tests++;
            float t, u, v;
#if MTSG_RECT_PEND_I
            bool h;
            uint32_t key, pid;
            if (rp) {
                h = rect_test_rows(f0, f1, f2, r.o, r.d, r.mint, r.best, t, u, v);
                key = S.n_tri + inst;
                pid = inst;
                r.bits &= ~SB_RPEND;
            } else {
                h = tri_test(f0, f1, f2, r.o, r.d, r.mint, r.best, u, v, t);
                key = __float_as_uint(f2.z);
                pid = __float_as_uint(f2.w);
            }
#else
            bool h = tri_test(f0, f1, f2, r.o, r.d, r.mint, r.best, u, v, t);
            if (isRect) h = rect_test(S.rects[__float_as_uint(f2.w)], r.o, r.d, r.mint, r.best, t, u, v);
            const uint32_t key = __float_as_uint(f2.z), pid = __float_as_uint(f2.w);
#endif
#if MTSG_MAILBOX
            // an exact tie is flagged (the ray is traced again by
            // tie_retrace_i); the key tells a primitive of one instance from
            // the same primitive of another, and a retest from a tie: distinct
            // for every (primitive, instance) pair (DevScene::instKeyStride)
            const uint32_t tkey = key + ((r.bits & SB_INST) ? (inst + 1u) * S.instKeyStride : 0u);
            r.bits |= (h & (t == r.best) & (tkey != r.bestKey)) ? SB_TIE : 0u;
            if (h) r.bestKey = tkey;
#endif
            if (h) {
                r.bits |= SB_FOUND;
                if (r.bits & SB_SHADOW) return true;   // any hit occludes
                r.best = t;
                stS(P.hit + idx, make_float4(t, u, v, __uint_as_float(isRect ? (0x80000000u | pid) : pid)));
                P.hitInst[idx] = (r.bits & SB_INST) ? inst : 0xFFFFFFFFu;
            }
        } else if (enter) {
            inst = __float_as_uint(f2.w);
            r.bits |= SB_PEND;
        }
        if (!defer) ++r.lfE;
    }
    if (inner) {
        if (COUNT) cnt.nodes++;
        const uint2 c = spec_take_i(L, r, p0, tsplit, goLeft, push);
        r.cur = c;
        if (rootKind && !(c.x & 0x80000000u)) {
            if (COUNT) cnt.nodes++;
            float ts2;
            bool gl2, push2;
            spec_plan(r, c, ts2, gl2, push2);
            r.cur = spec_take_i(L, r, pc, ts2, gl2, push2);
        }
    }
    if (enter) return false;   // entered (or not) in the next iteration
    const bool found = (r.bits & SB_FOUND) != 0;
    const bool inInst = (r.bits & SB_INST) != 0;
    const bool leafDone = (r.lfTmax >= 0.0f) & (r.lfE >= r.lfEnd);
    // Havran's exit (held leaf finished, or an empty leaf reached, beyond the
    // best hit) and the end of the traversal: the ray is done at the top level,
    // or leaves its instance (one exit point, so inst_exit is inlined once)
    bool leave = leafDone & found & (r.best < r.lfTmax);
    r.lfTmax = leafDone ? -1.0f : r.lfTmax;
    const uint2 c = r.cur;
    if (!leave & (r.lfTmax < 0.0f) & !(r.bits & SB_TRAVDONE) & (bool)(c.x >> 31)) {
        const uint32_t st = c.x & 0x7FFFFFFFu;
        const bool nonEmpty = st < c.y;
        leave = !nonEmpty & found & (r.best < r.tmax);
    }
    if (!leave & (r.lfTmax < 0.0f) & !(r.bits & SB_TRAVDONE) & (bool)(c.x >> 31)) {
        const uint32_t st = c.x & 0x7FFFFFFFu;
        const bool nonEmpty = st < c.y;
        r.lfE = nonEmpty ? st : r.lfE;
        r.lfEnd = nonEmpty ? c.y : r.lfEnd;
        r.lfTmax = nonEmpty ? r.tmax : r.lfTmax;
        const uint32_t b = r.bits;
        const uint32_t cap = inInst ? L.capGrp : L.capTop;
        if (b & SB_N) {
            const uint32_t top = b & SB_TOP, k = top == 0 ? cap - 1 : top - 1u;
            const uint32_t i = (k + (inInst ? (uint32_t)OUTER_STACK : 0u)) * TRACE_BLOCK + lane_here();
            r.cur = s_lvNode[i];
            const float t = s_lvT[i];
            r.bits = ((b & ~SB_TOP) | k) - SB_N1;
            r.tmin = r.tmax;
            r.tmax = fminf(t, r.best);
        } else {
            if (COUNT && (b & SB_DROPPED)) cnt.restarts++;
            kd_restart(L, r, b, inInst ? inst_root(S, inst) : S.root2, c);
        }
    }
    const bool done = leave || ((r.bits & SB_TRAVDONE) && r.lfTmax < 0.0f);
    if (done && inInst) {
#if MTSG_EXIT_BATCH
        r.bits |= SB_XPEND;
#else
        const bool sh = (r.bits & SB_SHADOW) != 0;
        inst_exit(S, r, (sh ? P.sh_o : P.ray_o) + idx, (sh ? P.sh_d : P.ray_d) + idx, ts);
#endif
        return false;
    }
    return done;
}

// ---------------------------------------------------------------------------
// Exact ties in two-level scenes.  The two-level iteration flags a closest
// ray when a different primitive hits at exactly the best distance so far
// (SB_TIE, as the flat one), and the ray is traced again here by a literal
// SAHKDTree3D::rayIntersectHavran (sahkdtree3.h:178-308): entry / exit
// points, a full stack and the 8-entry hashed mailbox, one fresh traversal
// (and mailbox) per level as the reference runs one per ShapeKDTree -- the
// scene's, and the group's inside Instance::rayIntersect (instance.cpp:
// 115-130, skdtree.h:431-458).  Ties are rare (coincident faces, shared
// edges), so this path is written for exactness, not speed: its stack lives
// in scratch.  Mailbox keys are the TriAccel indices of the leaf records
// (the oracle's keys, oracle.cpp havranTree).
// ---------------------------------------------------------------------------
constexpr int HAVRAN_DEPTH = 72;   // the layout refuses trees deeper than 64 (mtsg.hip convert)
struct HavranHit {
    float4 rec;      // t, u, v, primitive (0x80000000 | rectangle)
    uint32_t inst;   // instance of the hit, ~0: top level
    bool err;        // stack overflow (the render fails with MTSG_ERR_TRAVERSAL)
};
// one level; returns whether a primitive of this level (or of an instance
// entered from it) was accepted; maxt shrinks with the accepted hits
template <bool TOP>
DEV bool havran_level(const DevScene &S, float3 o, float3 d, float mint, float maxt, uint2 root, uint32_t inst, HavranHit &H) {
#pragma clang fp contract(off)
    struct Ent { uint2 node; float t; uint32_t prev; float3 p; };
    Ent st[HAVRAN_DEPTH];
    uint32_t mbox[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) mbox[k] = 0xFFFFFFFFu;
    const float3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    auto at = [&](float t) { return mk3(o.x + d.x * t, o.y + d.y * t, o.z + d.z * t); };
    uint32_t en = 0, ex = 1;
    st[0].t = mint;
    st[0].p = at(mint);
    st[1].t = maxt;
    st[1].p = at(maxt);
    st[1].node = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);   // end of the traversal
    bool found = false;
    uint2 cur = root;
    while (!(cur.x == 0xFFFFFFFFu && cur.y == 0xFFFFFFFFu)) {
        while (!(cur.x & 0x80000000u)) {
            const uint32_t axis = cur.x & 3u;
            const float split = __uint_as_float(cur.y);
            const uint4 pr = S.blocks[(cur.x & 4u) ? (cur.x >> 3) : (cur.x >> 3) * 4u];
            const uint2 left = make_uint2(pr.x, pr.y), right = make_uint2(pr.z, pr.w);
            uint2 farChild;
            if (comp(st[en].p, axis) <= split) {
                if (comp(st[ex].p, axis) <= split) { cur = left; continue; }
                if (comp(st[en].p, axis) == split) { cur = right; continue; }
                cur = left;
                farChild = right;
            } else {
                if (split < comp(st[ex].p, axis)) { cur = right; continue; }
                farChild = left;
                cur = right;
            }
            const float dist = (split - comp(o, axis)) * comp(inv, axis);
            const uint32_t tmp = ex++;
            if (ex == en) ++ex;
            if (ex >= (uint32_t)HAVRAN_DEPTH) { H.err = true; return found; }
            st[ex].prev = tmp;
            st[ex].t = dist;
            st[ex].node = farChild;
            float3 p = at(dist);
            if (axis == 0u) p.x = split; else if (axis == 1u) p.y = split; else p.z = split;
            st[ex].p = p;
        }
        for (uint32_t e = cur.x & 0x7FFFFFFFu; e < cur.y; ++e) {
            const float4 *rec = S.triL + 3 * (size_t)e;
            const float4 f0 = rec[0], f1 = rec[1], f2 = rec[2];
            const uint32_t key = __float_as_uint(f2.z);
            if (mbox[key & 7u] == key) continue;
            const uint32_t k = __float_as_uint(f0.x);
            if (TOP && k == KINST) {
                // Instance::rayIntersect: the group's tree on the clipped interval
                const uint32_t ii = __float_as_uint(f2.w);
                const float4 *I = S.inst + 8 * (size_t)ii;
                const float4 L0 = I[0], L1 = I[1], L2 = I[2], A0 = I[6], A1 = I[7];
                const float3 lo = mk3(L0.x * o.x + L0.y * o.y + L0.z * o.z + L0.w, L1.x * o.x + L1.y * o.y + L1.z * o.z + L1.w,
                                      L2.x * o.x + L2.y * o.y + L2.z * o.z + L2.w);
                const float3 ld = mk3(L0.x * d.x + L0.y * d.y + L0.z * d.z, L1.x * d.x + L1.y * d.y + L1.z * d.z,
                                      L2.x * d.x + L2.y * d.y + L2.z * d.z);
                const float3 li = mk3(1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z);
                float nearT = -INFINITY, farT = INFINITY;
                bool ok = true;
                const float bmn[3] = {A0.x, A0.y, A0.z}, bmx[3] = {A1.x, A1.y, A1.z};
                for (int a = 0; a < 3 && ok; ++a) {
                    const float oa = comp(lo, a), da = comp(ld, a);
                    if (da == 0.0f) {
                        if (oa < bmn[a] || oa > bmx[a]) ok = false;
                    } else {
                        float t1 = (bmn[a] - oa) * comp(li, a), t2 = (bmx[a] - oa) * comp(li, a);
                        if (t1 > t2) { const float x = t1; t1 = t2; t2 = x; }
                        nearT = t1 < nearT ? nearT : t1;   // std::max / std::min (aabb.h:308-338)
                        farT = farT < t2 ? farT : t2;
                        if (!(nearT <= farT)) ok = false;
                    }
                }
                if (ok) {
                    if (mint > nearT) nearT = mint;
                    if (maxt < farT) farT = maxt;
                    if (farT > nearT &&
                        havran_level<false>(S, lo, ld, nearT, farT, make_uint2(__float_as_uint(A0.w), __float_as_uint(A1.w)), ii, H)) {
                        maxt = H.rec.x;
                        found = true;
                    }
                    if (H.err) return found;
                }
            } else {
                float t, u, v;
                bool h;
                if (k == MTSG_TRIACCEL_SHAPE) h = rect_test(S.rects[__float_as_uint(f2.w)], o, d, mint, maxt, t, u, v);
                else h = tri_test(f0, f1, f2, o, d, mint, maxt, u, v, t);
                if (h) {
                    maxt = t;
                    found = true;
                    const uint32_t p = __float_as_uint(f2.w);
                    H.rec = make_float4(t, u, v, __uint_as_float(k == MTSG_TRIACCEL_SHAPE ? (0x80000000u | p) : p));
                    H.inst = TOP ? 0xFFFFFFFFu : inst;
                }
            }
            mbox[key & 7u] = key;
        }
        if (st[ex].t > maxt) break;
        en = ex;
        cur = st[ex].node;
        ex = st[en].prev;
    }
    return found;
}

// a closest ray of a two-level scene traced again exactly (ray from its work
// list entry, as spec_init clips it): rewrites its hit record and instance
__attribute__((noinline)) DEV void tie_retrace_i(const DevScene &S, const DevPaths &P, uint32_t idx, bool &err) {
    float4 ro, rd;
    load_closest_ray(S, P, idx, P.camEnc != 0, ro, rd);
    SpecRay r;
    if (!spec_init(S, xyz(ro), xyz(rd), ro.w, rd.w, false, r)) return;
    HavranHit H;
    H.err = false;
    if (havran_level<true>(S, r.o, r.d, r.mint, r.best, S.root2, 0xFFFFFFFFu, H)) {
        stS(P.hit + idx, H.rec);
        P.hitInst[idx] = H.inst;
    }
    err = H.err;
}

// Persistent traversal kernel with lane-level refill (the "while-while +
// dynamic fetch" structure of Aila & Laine 2009, re-tiled for 64-lane waves):
// a wave reserves FETCH work-list entries with ONE atomic into a wave-uniform
// pool (SGPRs), and once MIN_IDLE lanes have finished their rays they take the
// next pool entries.  One launch traces this bounce's closest-hit rays and the
// previous bounce's shadow rays as one work list (both only depend on the
// previous k_shade), so lanes of either kind share waves and the launch has
// one tail instead of two:
//   [0, nC):       closest hit of P.ray_o/ray_d[i]   -> P.hit[i]
//   [nC, nC + nS): any hit of P.sh_o/sh_d[i - nC]    -> unoccluded: L += sh_c
//   cIn: -1 = nIdentity closest rays (bounce 0), 0/1 = count in cnt_q(cIn), -2 = none
//   sIn: 0/1 = count in CNT_S0/CNT_S1, -1 = none

// ---------------------------------------------------------------------------
// Ray order of a bounce (round 6).  The closest rays of bounce b >= 1 sit in
// the order k_shade appended them: tile-major, so consecutive rays start from
// neighbouring surface points of one 16x16 tile, at successive samples -- but
// leave in directions spread over the BSDF lobes.  Rays taken in a random
// order instead cost the C3 traversal 2.2x on the camera rays and +33% on
// bounce 1 (profiles/r06_ray_order.txt: the order's locality is what keeps the
// node and TriAccel fetches in L1/L2).  k_sortwin sorts each window of
// SORT_WINDOW consecutive rays (16 samples of one tile) by an octahedral
// direction bin, so a wave's refills take rays from one tile that also leave
// in one direction cone; the traversal reads entry i from position order[i]
// and writes its hit there, so shading keeps its dense order and the image
// does not change (random numbers are keyed by pixel and sample).  Measured:
// the sorted windows lose (C3 trace +6.7 ms): the production default is the
// append order (MTSG_OPT_RAY_ORDER 0); the sort stays as that option.
// ---------------------------------------------------------------------------
#ifndef MTSG_SORT_WINDOW
#define MTSG_SORT_WINDOW 4096
#endif
#ifndef MTSG_SORT_BINS_LOG
#define MTSG_SORT_BINS_LOG 4   // 16 x 16 octahedral bins (~11 degrees)
#endif
constexpr uint32_t SORT_WINDOW = MTSG_SORT_WINDOW;
constexpr int SORT_BLOCK = 1024;
constexpr int SORT_BINS = 1 << (2 * MTSG_SORT_BINS_LOG);
static_assert(SORT_BINS <= SORT_BLOCK && SORT_WINDOW % SORT_BLOCK == 0, "k_sortwin layout");
// octahedral map of a direction (any length) to one of SORT_BINS cells
DEV uint32_t dir_bin(float3 d) {
    const float s = 1.0f / (fabsf(d.x) + fabsf(d.y) + fabsf(d.z));
    float u = d.x * s, v = d.y * s;
    if (d.z < 0.0f) {
        const float uu = (1.0f - fabsf(v)) * (u < 0.0f ? -1.0f : 1.0f), vv = (1.0f - fabsf(u)) * (v < 0.0f ? -1.0f : 1.0f);
        u = uu;
        v = vv;
    }
    constexpr int n = 1 << MTSG_SORT_BINS_LOG;
    const int iu = min(n - 1, max(0, (int)((u * 0.5f + 0.5f) * (float)n)));
    const int iv = min(n - 1, max(0, (int)((v * 0.5f + 0.5f) * (float)n)));
    return (uint32_t)(iv * n + iu);
}
// one window per workgroup iteration: an LDS counting sort of its rays by
// direction bin (rank within a bin from an LDS atomic: any order of a bin's
// rays is as good), then order[window + slot] = the ray's position
__global__ void __launch_bounds__(SORT_BLOCK) k_sortwin(DevPaths P, int qin) {
    __shared__ uint32_t hist[SORT_BINS];
    __shared__ uint32_t waveSum[SORT_BLOCK / 64];
    constexpr int PER = (int)SORT_WINDOW / SORT_BLOCK;
    const uint32_t n = __atomic_load_n(&P.cnt[cnt_q(qin)], __ATOMIC_RELAXED);
    const uint32_t tid = threadIdx.x;
    for (uint32_t w0 = blockIdx.x * SORT_WINDOW; w0 < n; w0 += gridDim.x * SORT_WINDOW) {
        for (uint32_t k = tid; k < (uint32_t)SORT_BINS; k += SORT_BLOCK) hist[k] = 0u;
        __syncthreads();
        uint32_t key[PER], rank[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t pos = w0 + (uint32_t)j * SORT_BLOCK + tid;
            key[j] = 0u;
            rank[j] = 0u;
            if (pos < n) {
                key[j] = dir_bin(xyz(P.ray_d[pos]));
                rank[j] = atomicAdd(&hist[key[j]], 1u);
            }
        }
        __syncthreads();
        // exclusive prefix sum of the bins: a wave scan per 64 bins, then the
        // waves' totals
        uint32_t v = 0u, incl = 0u;
        if (tid < (uint32_t)SORT_BINS) {
            v = hist[tid];
            incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(incl, o);
                if (__lane_id() >= (uint32_t)o) incl += t;
            }
            if (__lane_id() == 63u) waveSum[tid >> 6] = incl;
        }
        __syncthreads();
        if (tid < (uint32_t)SORT_BINS) {
            uint32_t before = 0u;
            for (uint32_t w = 0; w < (tid >> 6); ++w) before += waveSum[w];
            hist[tid] = before + incl - v;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t pos = w0 + (uint32_t)j * SORT_BLOCK + tid;
            if (pos < n) P.orderBuf[w0 + hist[key[j]] + rank[j]] = pos;
        }
        __syncthreads();
    }
}

// MTSG_SHUFFLE (measurement variant, round 6): the traversal takes its rays in
// a random order -- 1: closest rays, 2: shadow rays too -- to measure what the
// work list's order (tile-major camera rays, append-ordered bounce rays) is
// worth to the traversal: a bijection of [0, n) (cycle-walking over a
// multiply / xor-shift bijection of the enclosing power of two)
#ifndef MTSG_SHUFFLE
#define MTSG_SHUFFLE 0
#endif
DEV uint32_t shuffle_index(uint32_t x, uint32_t n) {
    if (n < 2) return x;
    const uint32_t m = 32u - __clz(n - 1u), mask = m >= 32 ? 0xFFFFFFFFu : (1u << m) - 1u;
    do {
        x = (x * 0x9E3779B1u + 0x7F4A7C15u) & mask;
        x ^= x >> ((m + 1) / 2);
        x = (x * 0x85EBCA6Bu) & mask;
        x ^= x >> ((m + 2) / 3);
    } while (x >= n);
    return x;
}

template <bool COUNT, int MIN_IDLE, bool INST = false, bool KNOBS = false>
__global__ void __launch_bounds__(TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(INST ? (COUNT ? 1 : MTSG_INST_WAVES) : MTSG_SPEC_WAVES)))
k_trace_s(DevScene S, DevPaths P, int cIn, int sIn, uint32_t nIdentity, unsigned long long *wt) {
    const SpecStack stk{};
    const TravLimits L = trav_limits<KNOBS>(S);
    lds_top_init(S);
    const unsigned long long tStart = wt ? wall_clock64() : 0ull;
    const uint32_t nC = cIn == -1 ? nIdentity : (cIn >= 0 ? __atomic_load_n(&P.cnt[cnt_q(cIn)], __ATOMIC_RELAXED) : 0u);
    const uint32_t nS = sIn >= 0 ? __atomic_load_n(&P.cnt[cnt_s(sIn)], __ATOMIC_RELAXED) : 0u;
    Fetch F{&P.cnt[CNT_FETCH], nC + nS, blockIdx.x % XGROUPS, 0, max(1u, gridDim.x / XGROUPS * GUIDE_SPLIT), FETCH};
    TraceCounts cc{0, 0, 0, 0, 0, 0, 0, 0, 0}, cs{0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t poolBase = 0, poolLeft = 0;   // wave-uniform
    bool exhausted = false;
    bool active = false;
    uint32_t idx = 0;                      // index into the ray's own list
    uint32_t inst = 0;                     // INST: the instance the lane is inside
    TopSave ts;                            // (MTSG_INST_REGSAVE: its top-level state)
    uint32_t iters = 0;                    // COUNT: iterations of this ray
    uint32_t n0 = 0, t0c = 0, r0 = 0;      // COUNT: the lane's node / test / restart totals at its start
    unsigned long long tExh = 0;           // wt: when the work list was found empty
    uint32_t drainIters = 0;               // wt: loop iterations after that
    SpecRay r;
    for (;;) {
        unsigned long long idle = __ballot(!active);
        if ((uint32_t)__popcll(idle) < (uint32_t)MIN_IDLE && __any(active)) idle = 0;
        while (idle && !exhausted) {
            if (poolLeft == 0 && !F.next(FETCH, poolBase, poolLeft)) {
                exhausted = true;
                if (WT_DRAIN && wt) tExh = wall_clock64();
                break;
            }
            const uint32_t nIdle = (uint32_t)__popcll(idle);
            const uint32_t take = min(nIdle, poolLeft);
            const uint32_t rank = rank_below(idle);
            if (!active && rank < take) {
                const uint32_t i = poolBase + rank;
                const bool shadow = i >= nC;
                idx = shadow ? i - nC : (P.order ? P.order[i] : i);
#if MTSG_SHUFFLE
                // measurement: the work list in a random order (coherence experiment)
                if (!shadow || MTSG_SHUFFLE == 2) idx = shuffle_index(idx, shadow ? nS : nC);
#endif
                float4 ro, rd;
                if (shadow) {
                    ro = ldS(P.sh_o + idx);
                    rd = ldS(P.sh_d + idx);
                    const float mint = rd.w; rd.w = ro.w; ro.w = mint;   // sh_o.w = maxt, sh_d.w = mint
                } else {
                    load_closest_ray(S, P, idx, !INST && P.camEnc != 0, ro, rd);   // (two-level scenes: never compact)
                }
                if (spec_init(S, xyz(ro), xyz(rd), ro.w, rd.w, shadow, r)) {
                    active = true;
                    if (COUNT) {
                        iters = 0;
                        const TraceCounts &k = shadow ? cs : cc;
                        n0 = k.nodes; t0c = k.tests; r0 = k.restarts;
                    }
                } else if (shadow) {
                    shadow_unoccluded(P, idx);
                } else if (!(rd.w < 0.0f)) {   // maxt < 0: dead slot outside the render rectangle
                    stS(&P.hit[idx], miss_record());
                }
                if (INST && !shadow) P.hitInst[idx] = 0xFFFFFFFFu;
            }
            poolBase += take;
            poolLeft -= take;
            idle = __ballot(!active);
            if (take == nIdle) break;
        }
        if (!__any(active)) {
            if (exhausted) break;
            continue;
        }
        if (COUNT) {
            // wave-level figures are booked with the closest-hit counters
            const uint2 n = r.cur;
            const bool inner = active && !(r.bits & SB_TRAVDONE) && !(n.x & 0x80000000u);
            const bool prim = active && r.lfE < r.lfEnd;
            const bool anyInner = __any(inner), anyPrim = __any(prim);
            const uint32_t nActive = (uint32_t)__popcll(__ballot(active));
            if (__lane_id() == 0) { cc.wsteps += 1; cc.wnodes += anyInner; cc.wtests += anyPrim; cc.wactive += nActive; }
        }
        if (WT_DRAIN && wt && exhausted) ++drainIters;
        bool done = false;
        if (active) {
            if (INST) {
                const bool sh = (r.bits & SB_SHADOW) != 0;
                if (COUNT && sh) done = spec_iter_i<COUNT>(S, r, cs, P, idx, L, inst, ts);
                else done = spec_iter_i<COUNT>(S, r, cc, P, idx, L, inst, ts);
            } else if (TIE_INLINE && (r.bits & SB_MBRUN)) {
                // the retrace of a tie (below): Mitsuba's mailbox emulated (not counted)
                done = spec_iter<false, true>(S, r, stk, cc, P.hit + idx, L);
            } else {
                if (COUNT && (r.bits & SB_SHADOW)) done = spec_iter<COUNT>(S, r, stk, cs, P.hit + idx, L);
                else done = spec_iter<COUNT>(S, r, stk, cc, P.hit + idx, L);
            }
        }
        if (COUNT && active) ++iters;
        if (done && MTSG_MAILBOX && (r.bits & (SB_TIE | SB_SHADOW | SB_MBRUN)) == SB_TIE) {
            if (COUNT) atomicAdd(&P.ctr[51], 1ull);
            if (!INST && TIE_INLINE) {
                // a closest ray that met an exact tie is traced again from its
                // start in this lane with the mailbox (tie_retrace), inside the
                // launch: its drain absorbs the retrace, no k_tie launch follows
                float4 ro, rd;
                load_closest_ray(S, P, idx, P.camEnc != 0, ro, rd);
                spec_init(S, xyz(ro), xyz(rd), ro.w, rd.w, false, r);   // true: it passed before
                r.bits |= SB_MBRUN;
                done = false;
            } else {
                // k_tie_i traces it again with the two-level mailboxes
                P.tie[atomicAdd(&P.cnt[CNT_TIE], 1u)] = idx;
            }
        }
        if (done) {
            active = false;
            if (COUNT) {
                const bool sh = (r.bits & SB_SHADOW) != 0;
                if (!INST) {
                    // kd-restarts of the ray, and those that took the guard's
                    // one-ulp step (restart number >= rstGuard, kd_restart)
                    const uint32_t nr = (r.bits >> SB_RST_SHIFT) & SB_RST_MASK;
                    if (nr) atomicAdd(&P.ctr[56 + sh], (unsigned long long)nr);
                    if (nr > L.rstGuard) {
                        atomicAdd(&P.ctr[52 + sh], 1ull);
                        atomicAdd(&P.ctr[54 + sh], (unsigned long long)(nr - L.rstGuard));
                    }
                }
                atomicMax(&P.ctr[sh ? 15 : 7], (unsigned long long)iters);
                atomicAdd(&P.ctr[(sh ? 32 : 16) + min(15, 31 - __clz(max(iters, 1u)))], 1ull);
                if (iters >= STRAGGLER_ITERS) {
                    const unsigned long long k = atomicAdd(&P.ctr[48], 1ull);
                    if (k < STRAGGLER_MAX) {
                        unsigned long long *o = P.ctr + 64 + 8 * k;
                        o[0] = __float_as_uint(r.o.x); o[1] = __float_as_uint(r.o.y); o[2] = __float_as_uint(r.o.z);
                        o[3] = __float_as_uint(r.d.x); o[4] = __float_as_uint(r.d.y); o[5] = __float_as_uint(r.d.z);
                        const TraceCounts &kk = sh ? cs : cc;
                        o[6] = iters | (sh ? 0x80000000u : 0u);
                        o[7] = min(kk.nodes - n0, 4095u) | min(kk.tests - t0c, 4095u) << 12 | min(kk.restarts - r0, 255u) << 24;
                    }
                }
            }
            if (r.bits & SB_ERR) atomicOr(&P.cnt[CNT_ERR], CNT_ERR_TRAVERSAL);
            // closest: hits were written through, only a miss needs a record
            if (!(r.bits & SB_FOUND)) {
                if (r.bits & SB_SHADOW) shadow_unoccluded(P, idx);
                else stS(&P.hit[idx], miss_record());
            }
        }
    }
    flush_counts<COUNT>(P.ctr, cc);
    flush_counts<COUNT>(P.ctr + 8, cs);
    if (COUNT && INST) {
        unsigned long long vi[2] = {cc.inst, cs.inst};
        for (int k = 0; k < 2; ++k) {
            for (int o2 = 32; o2 > 0; o2 >>= 1) vi[k] += __shfl_down(vi[k], o2);
            if (lane_id() == 0) atomicAdd(P.ctr + 49 + k, vi[k]);
        }
    }
    if (wt && __lane_id() == 0) {
        wt[WT_WORDS * blockIdx.x] = tStart;
        wt[WT_WORDS * blockIdx.x + 1] = wall_clock64();
        wt[WT_WORDS * blockIdx.x + 2] = tExh;
        wt[WT_WORDS * blockIdx.x + 3] = drainIters;
    }
}

// ---------------------------------------------------------------------------
// camera rays (PerspectiveCamera::sampleRayDifferential, perspective.cpp:271-298)
// ---------------------------------------------------------------------------
// pixel of position `pix` (0..255) inside a 16x16 tile: in Z order, so that
// 16 consecutive slots -- one refill of a traversal wave -- are a 4x4 pixel
// block instead of a 16x1 row (measured r06: C3 +0.2%, the slowest 1/8 share
// 22.04 -> 21.70 ms; MTSG_TILE_MORTON=0: row-major)
#ifndef MTSG_TILE_MORTON
#define MTSG_TILE_MORTON 1
#endif
__host__ __device__ inline void tile_pix(uint32_t pix, int &lx, int &ly) {
#if MTSG_TILE_MORTON
    lx = (int)((pix & 1u) | ((pix >> 1) & 2u) | ((pix >> 2) & 4u) | ((pix >> 3) & 8u));
    ly = (int)(((pix >> 1) & 1u) | ((pix >> 2) & 2u) | ((pix >> 3) & 4u) | ((pix >> 4) & 8u));
#else
    lx = (int)(pix % TILE);
    ly = (int)(pix / TILE);
#endif
}
DEV void slot_pixel(const DevBatch &B, uint32_t slot, int &x, int &y, uint32_t &s) {
    const uint32_t pix = slot & (TILE * TILE - 1);
    const uint32_t rest = slot >> 8;
    const uint32_t sl = rest % B.ns;
    const uint32_t tl = rest / B.ns;
    int tx, ty;
    tile_of_key(batch_key(B, B.tile0 + (int)tl), B.tiles_x, tx, ty, B.skew);
    int lx, ly;
    tile_pix(pix, lx, ly);
    x = B.rect_x + tx * TILE + lx;
    y = B.rect_y + ty * TILE + ly;
    s = B.s0 + sl;
}

// the camera-space point on the near plane of pixel (x, y)'s sample at
// (x + a, y + b) (sampleToCamera, perspective.cpp:271-280)
DEV float3 camera_near(const DevCamera &C, int x, int y, float a, float b) {
    const float sx = ((float)x + a) * C.inv_res_x, sy = ((float)y + b) * C.inv_res_y;
    const float *m = C.s2c;
    float px = m[0] * sx + m[1] * sy + m[3], py = m[4] * sx + m[5] * sy + m[7];
    float pz = m[8] * sx + m[9] * sy + m[11], pw = m[12] * sx + m[13] * sy + m[15];
    return pw == 1.0f ? mk3(px, py, pz) : mk3(px, py, pz) / pw;
}
DEV float3 camera_to_world_dir(const DevCamera &C, float3 d) {
    const float *t = C.c2w;
    return mk3(t[0] * d.x + t[1] * d.y + t[2] * d.z, t[4] * d.x + t[5] * d.y + t[6] * d.z, t[8] * d.x + t[9] * d.y + t[10] * d.z);
}
// rx/ryDirection of the ray through nearP (world direction wd), scaled by
// 1/sqrt(spp) (perspective.cpp:282-298, integrator.cpp:148-149, ray.h:163-168)
DEV void camera_differentials(const DevCamera &C, const DevIntegrator &I, float3 nearP, float3 wd, float3 &rxs, float3 &rys) {
    const float3 rxc = normalize(nearP + ld3(C.dx)), ryc = normalize(nearP + ld3(C.dy));
    const float3 rx = camera_to_world_dir(C, rxc), ry = camera_to_world_dir(C, ryc);
    const float scale = 1.0f / sqrtf((float)I.spp);
    rxs = wd + (rx - wd) * scale;
    rys = wd + (ry - wd) * scale;
}
// the scaled differentials of the camera ray of sample s of pixel (x, y), as
// k_camera computes them (its jitter draw, its direction): the shading of a
// bounce-0 environment miss recomputes them instead of reading them back
template <int SMP>
DEV void camera_ray_differentials(const DevCamera &C, const DevIntegrator &I, int x, int y, uint32_t s, float3 &rxs, float3 &rys) {
    float a, b;
    camera_jitter_smp<SMP>(I, x, y, s, a, b);   // (myPath2_OM, the one integrator without the jitter, has no differentials)
    const float3 nearP = camera_near(C, x, y, a, b);
    camera_differentials(C, I, nearP, camera_to_world_dir(C, normalize(nearP)), rxs, rys);
}

// the meta word of camera path `slot` at bounce 0, as k_camera stored it
// through round 6 (the `path` integrator: the jitter always draws): depth 1,
// next dimension 2, the slot, one 2D request; a slot outside the render
// rectangle is dead (0).  Bounce 0 computes it instead of reading 16 B per path.
DEV uint4 camera_meta(const DevBatch &B, uint32_t slot) {
    int x, y;
    uint32_t s;
    slot_pixel(B, slot, x, y, s);
    const bool alive = x < B.rect_x + B.rect_w && y < B.rect_y + B.rect_h;
    return alive ? make_uint4(1u, 2u, slot, 1u) : make_uint4(0u, 0u, slot, 0u);
}

__global__ void __launch_bounds__(BLOCK) k_camera(DevCamera C, DevIntegrator I, DevBatch B, DevPaths P) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    bool alive = false;
    if (slot < B.nslots) {
        int x, y;
        uint32_t s;
        slot_pixel(B, slot, x, y, s);
        alive = x < B.rect_x + B.rect_w && y < B.rect_y + B.rect_h;
        if (alive) {
            float a = 0.5f, b = 0.5f;   // myPath2_OM without jitterSample: the pixel centre, no draw
            const bool jitter = !I.om || I.om_jitter;
            if (jitter) camera_jitter(I, x, y, s, a, b);
            const float3 nearP = camera_near(C, x, y, a, b);
            const float3 d = normalize(nearP);
            const float invZ = 1.0f / d.z;
            const float3 wd = camera_to_world_dir(C, d);
            // flat scenes: the direction and 1/z only (load_closest_ray: C3 / C5
            // k_camera 32 -> 16 B per path); two-level scenes keep the origin for
            // their instance exits and tie retraces
            if (C.compact) {
                stS(&P.ray_d[slot], make_float4(wd.x, wd.y, wd.z, invZ));
            } else {
                stS(&P.ray_o[slot], make_float4(C.c2w[3], C.c2w[7], C.c2w[11], C.near_clip * invZ));
                stS(&P.ray_d[slot], make_float4(wd.x, wd.y, wd.z, C.far_clip * invZ));
            }
            if (C.diffs && !I.om) {   // myPath2_OM uses sensor->sampleRay: no differentials
                float3 rxs, rys;
                camera_differentials(C, I, nearP, wd, rxs, rys);
                // parked in T and aux (throughput 1, no previous vertex) until
                // bounce 0 is shaded
                stS(&P.T[slot], make_float4(rxs.x, rxs.y, rxs.z, 1.f));
                stS(&P.aux[slot], make_float4(rys.x, rys.y, rys.z, 0.f));
            }
            // Lp = (0, 0, 0, 1) is implied at bounce 0, and T = 1 without
            // differentials (load_path): 16-32 B per camera path neither written
            // nor read (r06: Lp with differentials too, C5 -16 B per path twice).
            // The meta word too (camera_meta), except for myPath2_OM, whose
            // shading kernel reads it: depth 1; the jitter used 2 dimensions in
            // one 2D request
            if (I.om) stS(&P.meta[slot], jitter ? make_uint4(1u, 2u, slot, 1u) : make_uint4(1u, 0u, slot, 0u));
        } else {
            // dead slot: bounce 0 runs over all slots and skips it
            stS(&P.ray_d[slot], make_float4(0.f, 0.f, 1.f, -1.0f));
            if (I.om) stS(&P.meta[slot], make_uint4(0u, 0u, slot, 0u));
            stS(&P.L[slot], make_float4(0.f, 0.f, 0.f, 0.f));
        }
    }
}

// ---------------------------------------------------------------------------
// BSDFs (local shading frame)
// ---------------------------------------------------------------------------
struct BsdfSample {
    float3 wo, weight;
    float pdf, eta;
    uint32_t delta;
};

// Material classes compiled into a shading kernel (MATS, a template parameter
// of k_shade).  A kernel's VGPR budget is the maximum over all the BSDF code
// it holds, so a scene whose records are all diffuse / GGX roughconductor /
// dielectric (the per-BSDF dispatch of path.cpp:145-264 over diffuse.cpp:93-150,
// roughconductor.cpp:168-415, dielectric.cpp:148-333) runs a kernel without the
// Beckmann / Phong microfacet code or the classes it does not use
// (mtsg_scene_create picks the smallest compiled set, mats_kernel_set).
enum : int { MAT_DIFFUSE = 1, MAT_RC_GGX = 2, MAT_RC_OTHER = 4, MAT_DIELECTRIC = 8, MATS_ALL = 15 };
// the compiled sets (k_shade<.., MATS> in smp_kernels.hip), smallest first
__host__ __device__ inline int mats_kernel_set(int m) {
    const int sets[3] = {MAT_DIFFUSE, MAT_DIFFUSE | MAT_RC_GGX, MAT_DIFFUSE | MAT_RC_GGX | MAT_DIELECTRIC};
    for (int c : sets)
        if ((m & ~c) == 0) return c;
    return MATS_ALL;
}

// warp.cpp:43-52,81-102
DEV float3 cosine_hemisphere(float sx, float sy) {
    float r1 = 2.0f * sx - 1.0f, r2 = 2.0f * sy - 1.0f;
    float phi, r;
    if (r1 == 0 && r2 == 0) { r = phi = 0; }
    else if (r1 * r1 > r2 * r2) { r = r1; phi = (kPi / 4.0f) * (r2 / r1); }
    else { r = r2; phi = (kPi / 2.0f) - (r1 / r2) * (kPi / 4.0f); }
    float sinPhi, cosPhi;
    mt_sincosf(phi, &sinPhi, &cosPhi);
    float px = r * cosPhi, py = r * sinPhi;
    float z = sqrtf(fmaxf(0.0f, 1.0f - px * px - py * py));
    if (z == 0) z = 1e-10f;
    return mk3(px, py, z);
}

// math.cpp:25-70
DEV float erfinv_m(float x) {
    float w = -mt_fastlog((1.0f - x) * (1.0f + x));
    float p;
    if (w < 5.0f) {
        w = w - 2.5f;
        p = 2.81022636e-08f;
        p = 3.43273939e-07f + p * w;
        p = -3.5233877e-06f + p * w;
        p = -4.39150654e-06f + p * w;
        p = 0.00021858087f + p * w;
        p = -0.00125372503f + p * w;
        p = -0.00417768164f + p * w;
        p = 0.246640727f + p * w;
        p = 1.50140941f + p * w;
    } else {
        w = sqrtf(w) - 3.0f;
        p = -0.000200214257f;
        p = 0.000100950558f + p * w;
        p = 0.00134934322f + p * w;
        p = -0.00367342844f + p * w;
        p = 0.00573950773f + p * w;
        p = -0.0076224613f + p * w;
        p = 0.00943887047f + p * w;
        p = 1.00167406f + p * w;
        p = 2.83297682f + p * w;
    }
    return p * x;
}
DEV float erf_m(float x) {
    const float a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f;
    const float a4 = -1.453152027f, a5 = 1.061405429f, p = 0.3275911f;
    float sign = copysignf(1.0f, x);
    x = fabsf(x);
    float t = 1.0f / (1.0f + p * x);
    float y = 1.0f - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * mt_fastexp(-x * x);
    return sign * y;
}
DEV float hypot2_m(float a, float b) {   // math.cpp:74-86
    float r;
    if (fabsf(a) > fabsf(b)) { r = b / a; r = fabsf(a) * sqrtf(1.0f + r * r); }
    else if (b != 0.0f) { r = a / b; r = fabsf(b) * sqrtf(1.0f + r * r); }
    else r = 0.0f;
    return r;
}

// MicrofacetDistribution, isotropic (microfacet.h:191-697)
struct MF {
    int type;
    float au, av;        // roughness along the shading tangent / bitangent
    bool visible;
    float eu, ev;        // Phong exponents (computePhongExponent, microfacet.h:701-704)
    DEV bool iso() const { return au == av; }
    // microfacet.h:545-552
    DEV float project(float3 v) const {
        const float invSinTheta2 = 1 / (1.0f - v.z * v.z);
        if (iso() || invSinTheta2 <= 0) return au;
        const float cosPhi2 = v.x * v.x * invSinTheta2, sinPhi2 = v.y * v.y * invSinTheta2;
        return sqrtf(cosPhi2 * au * au + sinPhi2 * av * av);
    }
    // microfacet.h:554-565 (RCPOVERFLOW_FLT = 2^-128)
    DEV float phong_exponent(float3 v) const {
        const float sinTheta2 = 1.0f - v.z * v.z;
        if (iso() || sinTheta2 <= 2.93873587705571876e-39f) return eu;
        const float invSinTheta2 = 1 / sinTheta2;
        return eu * (v.x * v.x * invSinTheta2) + ev * (v.y * v.y * invSinTheta2);
    }
    // microfacet.h:191-234
    DEV float D(float3 m) const {
        if (m.z <= 0) return 0.0f;
        float ct2 = m.z * m.z;
        float be = ((m.x * m.x) / (au * au) + (m.y * m.y) / (av * av)) / ct2;
        float result;
        if (type == MTSG_MF_BECKMANN) result = mt_fastexp(-be) / (kPi * au * av * ct2 * ct2);
        else if (type == MTSG_MF_GGX) { float root = (1.0f + be) * ct2; result = 1.0f / (kPi * au * av * root * root); }
        else result = sqrtf((eu + 2) * (ev + 2)) * (0.5f * kInvPi) * mt_powf(m.z, phong_exponent(m));
        if (result * m.z < 1e-20f) result = 0;
        return result;
    }
    // microfacet.h:477-514 (Phong uses the Beckmann approximation)
    DEV float G1(float3 v, float3 m) const {
        if (dot(v, m) * v.z <= 0) return 0.0f;
        float temp = 1 - v.z * v.z;
        float tt = temp <= 0.0f ? 0.0f : fabsf(sqrtf(temp) / v.z);
        if (tt == 0.0f) return 1.0f;
        const float a = project(v);
        if (type != MTSG_MF_GGX) {
            float aa = 1.0f / (a * tt);
            if (aa >= 1.6f) return 1.0f;
            float aSqr = aa * aa;
            return (3.535f * aa + 2.181f * aSqr) / (1.0f + 2.276f * aa + 2.577f * aSqr);
        }
        return 2.0f / (1.0f + hypot2_m(1.0f, a * tt));
    }
    DEV void visible11(float thetaI, float sx, float sy, float &slx, float &sly) const {
        if (type == MTSG_MF_BECKMANN) {
            const float SQRT_PI_INV = 0.56418958354775628695f;
            if (thetaI < 1e-4f) {
                float r = sqrtf(-mt_fastlog(1.0f - sx));
                float sp, cp;
                mt_sincosf(2 * kPi * sy, &sp, &cp);
                slx = r * cp; sly = r * sp;
                return;
            }
            float tanThetaI = mt_tanf(thetaI), cotThetaI = 1 / tanThetaI;
            float aa = -1, c = erf_m(cotThetaI);
            float sample_x = fmaxf(sx, 1e-6f);
            float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
            float b = c - (1 + c) * mt_powf(1 - sample_x, fit);
            float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * mt_expf(-cotThetaI * cotThetaI));
            int it = 0;
            while (++it < 10) {
                if (!(b >= aa && b <= c)) b = 0.5f * (aa + c);
                float invErf = erfinv_m(b);
                float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * mt_expf(-invErf * invErf)) - sample_x;
                float derivative = normalization * (1 - invErf * tanThetaI);
                if (fabsf(value) < 1e-5f) break;
                if (value > 0) c = b; else aa = b;
                b -= value / derivative;
            }
            slx = erfinv_m(b);
            sly = erfinv_m(2.0f * fmaxf(sy, 1e-6f) - 1.0f);
            return;
        }
        if (thetaI < 1e-4f) {
            float r = sqrtf(fmaxf(0.0f, sx / (1 - sx)));
            float sp, cp;
            mt_sincosf(2 * kPi * sy, &sp, &cp);
            slx = r * cp; sly = r * sp;
            return;
        }
        float tanThetaI = mt_tanf(thetaI);
        float aa = 1 / tanThetaI;
        float G1v = 2.0f / (1.0f + sqrtf(fmaxf(0.0f, 1.0f + 1.0f / (aa * aa))));
        float A = 2.0f * sx / G1v - 1.0f;
        if (fabsf(A) == 1) A -= copysignf(1.0f, A) * kEpsilon;
        float tmp = 1.0f / (A * A - 1.0f);
        float B = tanThetaI;
        float D = sqrtf(fmaxf(0.0f, B * B * tmp * tmp - (A * A - B * B) * tmp));
        float s1 = B * tmp - D, s2 = B * tmp + D;
        slx = (A < 0.0f || s2 > 1.0f / tanThetaI) ? s1 : s2;
        float S;
        if (sy > 0.5f) { S = 1.0f; sy = 2.0f * (sy - 0.5f); }
        else { S = -1.0f; sy = 2.0f * (0.5f - sy); }
        float z = (sy * (sy * (sy * (-0.365728915865723f) + 0.790235037209296f) - 0.424965825137544f) + 0.000152998850436920f) /
                  (sy * (sy * (sy * (sy * 0.169507819808272f - 0.397203533833404f) - 0.232500544458471f) + 1.0f) - 0.539825872510702f);
        sly = S * z * sqrtf(1.0f + slx * slx);
    }
    // sampleVisible (microfacet.h:421-459) or sampleAll (:287-397)
    DEV float3 sample(float3 wi_, float sx, float sy, float &pdf) const {
        if (visible) {
            float3 wi = normalize(mk3(au * wi_.x, av * wi_.y, wi_.z));
            float theta = 0, phi = 0;
            if (wi.z < 0.99999f) { theta = mt_acosf(wi.z); phi = mt_atan2f(wi.y, wi.x); }
            float sinPhi, cosPhi;
            mt_sincosf(phi, &sinPhi, &cosPhi);
            float slx, sly;
            visible11(theta, sx, sy, slx, sly);
            float rx = cosPhi * slx - sinPhi * sly, ry = sinPhi * slx + cosPhi * sly;
            rx *= au; ry *= av;
            float normalization = 1.0f / sqrtf(rx * rx + ry * ry + 1.0f);
            float3 m = mk3(-rx * normalization, -ry * normalization, normalization);
            pdf = wi_.z == 0 ? 0.0f : G1(wi_, m) * fabsf(dot(wi_, m)) * D(m) / fabsf(wi_.z);
            return m;
        }
        float sinPhiM, cosPhiM, cosThetaM;
        if (type == MTSG_MF_PHONG) {
            float phiM, exponent;
            if (iso()) {
                phiM = (2.0f * kPi) * sy;
                exponent = eu;
            } else if (sy < 0.25f) {
                phong_quadrant(4 * sy, phiM, exponent);
            } else if (sy < 0.5f) {
                phong_quadrant(4 * (0.5f - sy), phiM, exponent);
                phiM = kPi - phiM;
            } else if (sy < 0.75f) {
                phong_quadrant(4 * (sy - 0.5f), phiM, exponent);
                phiM += kPi;
            } else {
                phong_quadrant(4 * (1 - sy), phiM, exponent);
                phiM = 2 * kPi - phiM;
            }
            mt_sincosf(phiM, &sinPhiM, &cosPhiM);
            cosThetaM = mt_powf(sx, 1.0f / (exponent + 2.0f));
            pdf = sqrtf((eu + 2.0f) * (ev + 2.0f)) * (0.5f * kInvPi) * mt_powf(cosThetaM, exponent + 1.0f);
        } else {
            float alphaSqr;
            if (iso()) {
                mt_sincosf((2.0f * kPi) * sy, &sinPhiM, &cosPhiM);
                alphaSqr = au * au;
            } else {
                const float phiM = mt_atanf(av / au * mt_tanf(kPi + 2 * kPi * sy)) + kPi * floorf(2 * sy + 0.5f);
                mt_sincosf(phiM, &sinPhiM, &cosPhiM);
                const float cosSc = cosPhiM / au, sinSc = sinPhiM / av;
                alphaSqr = 1.0f / (cosSc * cosSc + sinSc * sinSc);
            }
            if (type == MTSG_MF_BECKMANN) {
                float t2 = alphaSqr * -mt_fastlog(1.0f - sx);
                cosThetaM = 1.0f / sqrtf(1.0f + t2);
                pdf = (1.0f - sx) / (kPi * au * av * cosThetaM * cosThetaM * cosThetaM);
            } else {
                float t2 = alphaSqr * sx / (1.0f - sx);
                cosThetaM = 1.0f / sqrtf(1.0f + t2);
                float temp = 1 + t2 / alphaSqr;
                pdf = kInvPi / (au * av * cosThetaM * cosThetaM * cosThetaM * temp * temp);
            }
        }
        if (pdf < 1e-20f) pdf = 0;
        float sinThetaM = sqrtf(fmaxf(0.0f, 1 - cosThetaM * cosThetaM));
        return mk3(sinThetaM * cosPhiM, sinThetaM * sinPhiM, cosThetaM);
    }
    // scaleAlpha (microfacet.h:178-183)
    DEV void scale_alpha(float v) {
        au *= v;
        av *= v;
        if (type == MTSG_MF_PHONG) {
            eu = fmaxf(2.0f / (au * au) - 2.0f, 0.0f);
            ev = fmaxf(2.0f / (av * av) - 2.0f, 0.0f);
        }
    }
    // pdf (microfacet.h:253-262): pdfVisible (:462-466) or pdfAll = D cos
    DEV float pdf(float3 wi, float3 m) const {
        if (visible) return wi.z == 0 ? 0.0f : G1(wi, m) * fabsf(dot(wi, m)) * D(m) / fabsf(wi.z);
        return D(m) * m.z;
    }
    // sampleFirstQuadrant (microfacet.h:707-715)
    DEV void phong_quadrant(float u1, float &phi, float &exponent) const {
        phi = mt_atanf(sqrtf((eu + 2.0f) / (ev + 2.0f)) * mt_tanf(kPi * u1 * 0.5f));
        float sinPhi, cosPhi;
        mt_sincosf(phi, &sinPhi, &cosPhi);
        exponent = eu * cosPhi * cosPhi + ev * sinPhi * sinPhi;
    }
};

// MicrofacetDistribution(props) after the loader's clamping (microfacet.h:96-144):
// Phong never samples visible normals.  MATS without MAT_RC_OTHER: every
// microfacet record of the scene is GGX (the distribution is then a constant
// and the Beckmann / Phong branches compile away)
template <int MATS = MATS_ALL>
DEV MF make_mf(const mtsg_bsdf &b) {
    MF m;
    m.type = (MATS & MAT_RC_OTHER) ? b.distribution : (int)MTSG_MF_GGX;
    m.au = b.alpha_u;
    m.av = b.alpha_v;
    m.visible = b.sample_visible != 0 && m.type != MTSG_MF_PHONG;
    const bool phong = m.type == MTSG_MF_PHONG;
    m.eu = phong ? fmaxf(2.0f / (m.au * m.au) - 2.0f, 0.0f) : 0.0f;
    m.ev = phong ? fmaxf(2.0f / (m.av * m.av) - 2.0f, 0.0f) : 0.0f;
    return m;
}

// util.cpp:739-761
DEV float3 fresnel_conductor(float cosThetaI, float3 eta, float3 k) {
    float c2 = cosThetaI * cosThetaI, s2 = 1 - c2, s4 = s2 * s2;
    float3 temp1 = eta * eta - k * k - mk3(s2, s2, s2);
    float3 a2pb2 = sqrtSafe3(temp1 * temp1 + k * k * eta * eta * 4);
    float3 aa = sqrtSafe3((a2pb2 + temp1) * 0.5f);
    float3 term1 = a2pb2 + mk3(c2, c2, c2), term2 = aa * (2 * cosThetaI);
    float3 Rs2 = (term1 - term2) / (term1 + term2);
    float3 term3 = a2pb2 * c2 + mk3(s4, s4, s4), term4 = term2 * s2;
    float3 Rp2 = Rs2 * (term3 - term4) / (term3 + term4);
    return (Rp2 + Rs2) * 0.5f;
}

// util.cpp:651-681
DEV float fresnel_dielectric(float cosThetaI_, float &cosThetaT_, float eta) {
    if (eta == 1) { cosThetaT_ = -cosThetaI_; return 0.0f; }
    float scale = (cosThetaI_ > 0) ? 1 / eta : eta, c2 = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (c2 <= 0.0f) { cosThetaT_ = 0.0f; return 1.0f; }
    float ci = fabsf(cosThetaI_), ct = sqrtf(c2);
    float Rs = (ci - eta * ct) / (ci + eta * ct), Rp = (eta * ci - ct) / (eta * ci + ct);
    cosThetaT_ = (cosThetaI_ > 0) ? -ct : ct;
    return 0.5f * (Rs * Rs + Rp * Rp);
}

// fresnelDielectricExt without the transmitted cosine (util.cpp:651-681)
DEV float fresnel_dielectric1(float cosThetaI, float eta) {
    float cosThetaT;
    return fresnel_dielectric(cosThetaI, cosThetaT, eta);
}

// plastic.cpp:216-222: the diffuse base renormalised for internal reflection
DEV float3 plastic_diffuse(const mtsg_bsdf &b, float3 diff) {
    if (b.nonlinear) diff = diff / (mk3(1.0f, 1.0f, 1.0f) - diff * b.fdr_int);
    else diff = diff / (1 - b.fdr_int);
    return diff;
}
DEV float plastic_prob_specular(const mtsg_bsdf &b, float Fi) {
    return (Fi * b.spec_sampling_weight) / (Fi * b.spec_sampling_weight + (1 - Fi) * (1 - b.spec_sampling_weight));
}

// evalCubicInterp1D over [0, 1] (spline.cpp:23-60)
DEV float cubic_interp1d(float x, const float *v, int n) {
    if (!(x >= 0.0f && x <= 1.0f)) return 0.0f;
    float t = x * (float)(n - 1);
    const int k = min((int)t, n - 2);
    const float f0 = v[k], f1 = v[k + 1];
    const float d0 = k > 0 ? 0.5f * (v[k + 1] - v[k - 1]) : v[k + 1] - v[k];
    const float d1 = k + 2 < n ? 0.5f * (v[k + 2] - v[k]) : v[k + 1] - v[k];
    t = t - (float)k;
    const float t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
}
// RoughTransmittance::eval with eta and alpha fixed (rtrans.h:169-181, 205-206)
DEV float rough_trans(const mtsg_bsdf &b, float cosTheta) {
    if (!(cosTheta >= 0)) return 0.0f;
    const float r = cubic_interp1d(mt_powf(fabsf(cosTheta), 0.25f), b.rtrans, MTSG_RTRANS_SAMPLES);
    return fminf(1.0f, fmaxf(0.0f, r));
}

// BSDF::eval * cos (ESolidAngle) and pdf for the smooth BSDFs.  EXT: the
// scene has conductor / plastic / twosided records (the shade kernel is
// instantiated without them otherwise: their code costs the common
// diffuse + roughconductor + dielectric kernel its register budget)
// alb: the record's reflectance (`reflectance` / `diffuseReflectance`), the
// constant or its texture's value at the hit (texture_eval)
template <bool EXT, int MATS = MATS_ALL>
DEV float3 bsdf_eval1(const mtsg_bsdf &b, float3 alb, float3 wi, float3 wo, float &pdf) {
    pdf = 0.0f;
    if ((MATS & MAT_DIFFUSE) && b.type == MTSG_BSDF_DIFFUSE) {   // diffuse.cpp:107-126
        if (!b.smooth || wi.z <= 0 || wo.z <= 0) return mk3(0, 0, 0);
        pdf = kInvPi * wo.z;
        return alb * (kInvPi * wo.z);
    }
    if ((MATS & (MAT_RC_GGX | MAT_RC_OTHER)) && b.type == MTSG_BSDF_ROUGHCONDUCTOR) {   // roughconductor.cpp:235-293
        if (wi.z <= 0 || wo.z <= 0) return mk3(0, 0, 0);
        float3 H = normalize(wo + wi);
        const MF mf = make_mf<MATS>(b);
        const float Dv = mf.D(H);
        if (mf.visible) pdf = Dv * mf.G1(wi, H) / (4.0f * wi.z);
        else pdf = Dv * H.z / (4 * fabsf(dot(wo, H)));
        if (Dv == 0) return mk3(0, 0, 0);
        float3 F = fresnel_conductor(dot(wi, H), ld3(b.eta), ld3(b.k)) * ld3(b.spec_refl);
        const float G = mf.G1(wi, H) * mf.G1(wo, H);
        float model = Dv * G / (4.0f * wi.z);
        return F * model;
    }
    if (EXT && b.type == MTSG_BSDF_ROUGHDIELECTRIC) {   // roughdielectric.cpp:265-400
        if (wi.z == 0) return mk3(0, 0, 0);
        const bool reflect = wi.z * wo.z > 0;
        const float eta = wi.z > 0 ? b.ior_eta : b.ior_inv_eta;
        float3 H = reflect ? normalize(wo + wi) : normalize(wi + wo * eta);
        H = H * copysignf(1.0f, H.z);
        float dwh_dwo;
        if (reflect) {
            dwh_dwo = 1.0f / (4.0f * dot(wo, H));
        } else {
            const float sqrtDenom = dot(wi, H) + eta * dot(wo, H);
            dwh_dwo = (eta * eta * dot(wo, H)) / (sqrtDenom * sqrtDenom);
        }
        const MF distr = make_mf(b);
        MF sampleDistr = distr;
        if (!distr.visible) sampleDistr.scale_alpha(1.2f - 0.2f * sqrtf(fabsf(wi.z)));
        float prob = sampleDistr.pdf(wi * copysignf(1.0f, wi.z), H);
        const float F = fresnel_dielectric1(dot(wi, H), b.ior_eta);
        prob *= reflect ? F : (1 - F);
        pdf = fabsf(prob * dwh_dwo);
        const float D = distr.D(H);
        if (D == 0) return mk3(0, 0, 0);
        const float G = distr.G1(wi, H) * distr.G1(wo, H);
        if (reflect) {
            const float value = F * D * G / (4.0f * fabsf(wi.z));
            return ld3(b.spec_refl) * value;
        }
        const float sqrtDenom = dot(wi, H) + eta * dot(wo, H);
        const float value = ((1 - F) * D * G * eta * eta * dot(wi, H) * dot(wo, H)) / (wi.z * sqrtDenom * sqrtDenom);
        const float factor = wi.z > 0 ? b.ior_inv_eta : b.ior_eta;   // ERadiance
        return ld3(b.spec_trans) * fabsf(value * factor * factor);
    }
    if (EXT && b.type == MTSG_BSDF_PLASTIC) {   // plastic.cpp:190-263, the diffuse (ESolidAngle) part
        if (wo.z <= 0 || wi.z <= 0) return mk3(0, 0, 0);
        const float Fi = fresnel_dielectric1(wi.z, b.ior_eta), Fo = fresnel_dielectric1(wo.z, b.ior_eta);
        const float invEta2 = 1 / (b.ior_eta * b.ior_eta);
        pdf = kInvPi * wo.z * (1 - plastic_prob_specular(b, Fi));
        return plastic_diffuse(b, alb) * (kInvPi * wo.z * invEta2 * (1 - Fi) * (1 - Fo));
    }
    if (EXT && b.type == MTSG_BSDF_ROUGHPLASTIC) {   // roughplastic.cpp:302-345 (eval), 347-385 (pdf)
        if (wi.z <= 0 || wo.z <= 0) return mk3(0, 0, 0);
        const MF mf = make_mf(b);
        const float3 H = normalize(wo + wi);
        const float D = mf.D(H);
        const float F = fresnel_dielectric1(dot(wi, H), b.ior_eta);
        const float G = mf.G1(wi, H) * mf.G1(wo, H);
        const float value = F * D * G / (4.0f * wi.z);
        const float T12 = rough_trans(b, wi.z), T21 = rough_trans(b, wo.z);
        const float invEta2 = 1.0f / (b.ior_eta * b.ior_eta);
        float probSpecular = plastic_prob_specular(b, 1 - T12);
        const float dwh_dwo = 1.0f / (4.0f * dot(wo, H));
        pdf = mf.pdf(wi, H) * dwh_dwo * probSpecular + (1 - probSpecular) * (kInvPi * wo.z);
        return ld3(b.spec_refl) * value + plastic_diffuse(b, alb) * (kInvPi * wo.z * T12 * T21 * invEta2);
    }
    return mk3(0, 0, 0);   // dielectric / conductor: delta components only
}

// next1d: the sampler's next1D, drawn only where Mitsuba draws it
// (roughdielectric's reflect/refract choice: roughdielectric.cpp:531-539)
template <bool EXT, int MATS, class Next1D>
DEV bool bsdf_sample1(const mtsg_bsdf &b, float3 alb, float3 wi, float sx, float sy, BsdfSample &r, Next1D &&next1d) {
    r.eta = 1.0f;
    r.delta = 0;
    if ((MATS & MAT_DIFFUSE) && b.type == MTSG_BSDF_DIFFUSE) {   // diffuse.cpp:139-150
        if (wi.z <= 0) return false;
        r.wo = cosine_hemisphere(sx, sy);
        r.pdf = kInvPi * r.wo.z;
        r.weight = alb;
        return !isZero(r.weight);
    }
    if ((MATS & (MAT_RC_GGX | MAT_RC_OTHER)) && b.type == MTSG_BSDF_ROUGHCONDUCTOR) {   // roughconductor.cpp:345-394
        if (wi.z < 0) return false;
        const MF mf = make_mf<MATS>(b);
        float pdf;
        float3 m = mf.sample(wi, sx, sy, pdf);
        if (pdf == 0) return false;
        r.wo = m * (2 * dot(wi, m)) - wi;
        if (r.wo.z <= 0) return false;
        float3 F = fresnel_conductor(dot(wi, m), ld3(b.eta), ld3(b.k)) * ld3(b.spec_refl);
        float weight;
        if (mf.visible) weight = mf.G1(r.wo, m);
        else weight = mf.D(m) * mf.G1(wi, m) * mf.G1(r.wo, m) * dot(wi, m) / (pdf * wi.z);
        r.pdf = pdf / (4.0f * dot(r.wo, m));
        r.weight = F * weight;
        return !isZero(r.weight);
    }
    if ((MATS & MAT_DIELECTRIC) && b.type == MTSG_BSDF_DIELECTRIC) {   // dielectric.cpp:277-333
        float cosThetaT;
        float F = fresnel_dielectric(wi.z, cosThetaT, b.ior_eta);
        r.delta = 1;
        if (sx <= F) {
            r.wo = mk3(-wi.x, -wi.y, wi.z);
            r.pdf = F;
            r.weight = ld3(b.spec_refl);
        } else {
            float scale = -(cosThetaT < 0 ? b.ior_inv_eta : b.ior_eta);
            r.wo = mk3(scale * wi.x, scale * wi.y, cosThetaT);
            r.eta = cosThetaT < 0 ? b.ior_eta : b.ior_inv_eta;
            r.pdf = 1 - F;
            float factor = cosThetaT < 0 ? b.ior_inv_eta : b.ior_eta;
            r.weight = ld3(b.spec_trans) * (factor * factor);
        }
        return !isZero(r.weight);
    }
    if (EXT && b.type == MTSG_BSDF_CONDUCTOR) {   // conductor.cpp:220-236
        if (wi.z <= 0) return false;
        r.delta = 1;
        r.wo = mk3(-wi.x, -wi.y, wi.z);
        r.pdf = 1.0f;
        r.weight = ld3(b.spec_refl) * fresnel_conductor(wi.z, ld3(b.eta), ld3(b.k));
        return !isZero(r.weight);
    }
    if (EXT && b.type == MTSG_BSDF_ROUGHDIELECTRIC) {   // roughdielectric.cpp:508-590
        const MF distr = make_mf(b);
        MF sampleDistr = distr;
        if (!distr.visible) sampleDistr.scale_alpha(1.2f - 0.2f * sqrtf(fabsf(wi.z)));
        float microfacetPDF;
        const float3 m = sampleDistr.sample(wi * copysignf(1.0f, wi.z), sx, sy, microfacetPDF);
        if (microfacetPDF == 0) return false;
        r.pdf = microfacetPDF;
        float cosThetaT;
        const float F = fresnel_dielectric(dot(wi, m), cosThetaT, b.ior_eta);
        bool sampleReflection = true;
        if (next1d() > F) {
            sampleReflection = false;
            r.pdf *= 1 - F;
        } else {
            r.pdf *= F;
        }
        float3 weight;
        float dwh_dwo;
        if (sampleReflection) {
            r.wo = m * (2 * dot(wi, m)) - wi;
            r.eta = 1.0f;
            if (wi.z * r.wo.z <= 0) return false;
            weight = ld3(b.spec_refl);
            dwh_dwo = 1.0f / (4.0f * dot(r.wo, m));
        } else {
            if (cosThetaT == 0) return false;
            const float e = cosThetaT < 0 ? b.ior_inv_eta : b.ior_eta;   // refract (util.cpp:767-772)
            r.wo = m * (dot(wi, m) * e + cosThetaT) - wi * e;
            r.eta = cosThetaT < 0 ? b.ior_eta : b.ior_inv_eta;
            if (wi.z * r.wo.z >= 0) return false;
            const float factor = cosThetaT < 0 ? b.ior_inv_eta : b.ior_eta;
            weight = ld3(b.spec_trans) * (factor * factor);
            const float sqrtDenom = dot(wi, m) + r.eta * dot(r.wo, m);
            dwh_dwo = (r.eta * r.eta * dot(r.wo, m)) / (sqrtDenom * sqrtDenom);
        }
        if (distr.visible) weight = weight * distr.G1(r.wo, m);
        else weight = weight * fabsf(distr.D(m) * (distr.G1(wi, m) * distr.G1(r.wo, m)) * dot(wi, m) / (microfacetPDF * wi.z));
        r.pdf *= fabsf(dwh_dwo);
        r.weight = weight;
        return !isZero(r.weight);
    }
    if (EXT && b.type == MTSG_BSDF_ROUGHPLASTIC) {   // roughplastic.cpp:387-455: component chosen by sample.y
        if (wi.z <= 0) return false;
        const float probSpecular = plastic_prob_specular(b, 1 - rough_trans(b, wi.z));
        if (sy < probSpecular) {
            sy /= probSpecular;
            const MF mf = make_mf(b);
            float mpdf;
            const float3 m = mf.sample(wi, sx, sy, mpdf);
            r.wo = m * (2 * dot(wi, m)) - wi;
            if (r.wo.z <= 0) return false;
        } else {
            sy = (sy - probSpecular) / (1 - probSpecular);
            r.wo = cosine_hemisphere(sx, sy);
        }
        float pdf;
        const float3 val = bsdf_eval1<EXT, MATS>(b, alb, wi, r.wo, pdf);
        if (pdf == 0) return false;
        r.pdf = pdf;
        r.weight = val / pdf;
        return !isZero(r.weight);
    }
    if (EXT && b.type == MTSG_BSDF_PLASTIC) {   // plastic.cpp:344-375 (both components)
        if (wi.z <= 0) return false;
        const float Fi = fresnel_dielectric1(wi.z, b.ior_eta);
        const float probSpecular = plastic_prob_specular(b, Fi);
        if (sx < probSpecular) {
            r.delta = 1;
            r.wo = mk3(-wi.x, -wi.y, wi.z);
            r.pdf = probSpecular;
            r.weight = ld3(b.spec_refl) * Fi / probSpecular;
        } else {
            r.wo = cosine_hemisphere((sx - probSpecular) / (1 - probSpecular), sy);
            const float Fo = fresnel_dielectric1(r.wo.z, b.ior_eta);
            const float invEta2 = 1 / (b.ior_eta * b.ior_eta);
            r.pdf = (1 - probSpecular) * (kInvPi * r.wo.z);
            r.weight = plastic_diffuse(b, alb) * (invEta2 * (1 - Fi) * (1 - Fo) / (1 - probSpecular));
        }
        return !isZero(r.weight);
    }
    return false;
}

// twosided.cpp:103-170: a twosided front record hands back-side queries to
// bsdfs[back] with the z components negated
// alb belongs to the record that answers (the back record for back-side
// queries of a twosided front record)
template <bool EXT, int MATS = MATS_ALL>
DEV float3 bsdf_eval(const mtsg_bsdf *all, const mtsg_bsdf &b, float3 alb, float3 wi, float3 wo, float &pdf) {
    if (EXT && b.twosided && !(wi.z > 0)) {
        wi.z = -wi.z;
        wo.z = -wo.z;
        return bsdf_eval1<EXT, MATS>(all[b.back], alb, wi, wo, pdf);
    }
    return bsdf_eval1<EXT, MATS>(b, alb, wi, wo, pdf);
}
template <bool EXT, int MATS = MATS_ALL, class Next1D>
DEV bool bsdf_sample(const mtsg_bsdf *all, const mtsg_bsdf &b, float3 alb, float3 wi, float sx, float sy, BsdfSample &r,
                     Next1D &&next1d) {
    if (EXT && b.twosided && wi.z < 0) {
        wi.z = -wi.z;
        if (!bsdf_sample1<EXT, MATS>(all[b.back], alb, wi, sx, sy, r, next1d)) return false;
        r.wo.z = -r.wo.z;
        return true;
    }
    return bsdf_sample1<EXT, MATS>(b, alb, wi, sx, sy, r, next1d);
}

DEV float mis(float pdfA, float pdfB) {   // path.cpp:296-300
    pdfA *= pdfA;
    pdfB *= pdfB;
    return pdfA / (pdfA + pdfB);
}

// DiscreteDistribution::sampleReuse (pmf.h:128-188): lower_bound over cdf[0..n]
DEV uint32_t pmf_sample_reuse(const float *cdf, uint32_t n, float &x, float &pdf) {
    uint32_t lo = 0, len = n + 1;
    while (len > 0) {   // std::lower_bound
        uint32_t half = len >> 1;
        if (cdf[lo + half] < x) { lo += half + 1; len -= half + 1; }
        else len = half;
    }
    int idx = (int)lo - 1;
    uint32_t index = (uint32_t)min((int)n - 1, max(0, idx));
    while ((cdf[index + 1] - cdf[index]) == 0 && index < n) ++index;
    float c0 = cdf[index], c1 = cdf[index + 1];
    pdf = c1 - c0;
    x = (x - c0) / (c1 - c0);
    return index;
}

// ---------------------------------------------------------------------------
// shading
// ---------------------------------------------------------------------------
struct Its {
    float3 p, geoN;
    Frame3 sh;
    int shape, bsdf, emitter;
};

// ShapeKDTree::fillIntersectionRecord<true> (skdtree.h:343-428) + computeShadingFrame (util.cpp:603-608).
// inst != ~0: the hit was found inside that instance; the group tree fills
// the record from the group-space ray (BarycentricPos = false, so p = ray(t))
// and Instance::fillIntersectionRecord (instance.cpp:146-160) maps it back
// with toWorld, normals by the inverse transpose (transform.h:203-211)
DEV void fill_its(const DevScene &S, float3 ro, float3 rd, float4 h, uint32_t inst, Its &its) {
#pragma clang fp contract(off)
    const uint32_t p = __float_as_uint(h.w);   // triangle, or 0x80000000 | rectangle
    float3 dpdu, n;
    if (!(p & 0x80000000u)) {
        const float4 *rec = S.shrec + 6 * (size_t)p;
        const float4 r0 = rec[0], r1 = rec[1], r2 = rec[2], r3 = rec[3], r4 = rec[4], r5 = rec[5];
        const float3 p0 = mk3(r0.x, r0.y, r0.z), p1 = mk3(r0.w, r1.x, r1.y), p2 = mk3(r1.z, r1.w, r2.x);
        const float3 n0 = mk3(r2.y, r2.z, r2.w), n1 = mk3(r3.x, r3.y, r3.z), n2 = mk3(r3.w, r4.x, r4.y);
        dpdu = mk3(r4.z, r4.w, r5.x);
        its.shape = (int)__float_as_uint(r5.y);
        const uint32_t bw = __float_as_uint(r5.z);
        its.bsdf = (int)(bw & 0x7FFFFFFFu);
        its.emitter = (int)__float_as_uint(r5.w);
        const float bx = 1 - h.y - h.z, by = h.y, bz = h.z;
        float3 fn = cross(p1 - p0, p2 - p0);
        if (!isZero(fn)) fn = fn / length(fn);
        if (!(bw & 0x80000000u)) {
            n = normalize(n0 * bx + n1 * by + n2 * bz);
            if (dot(fn, n) < 0) fn = -fn;
        } else {
            n = fn;
        }
        if (inst == 0xFFFFFFFFu) {
            its.p = p0 * bx + p1 * by + p2 * bz;
            its.geoN = fn;
        } else {
            const float4 *I = S.inst + 8 * (size_t)inst;
            const float4 L0 = I[0], L1 = I[1], L2 = I[2], W0 = I[3], W1 = I[4], W2 = I[5];
            const float3 lo = mk3(L0.x * ro.x + L0.y * ro.y + L0.z * ro.z + L0.w, L1.x * ro.x + L1.y * ro.y + L1.z * ro.z + L1.w,
                                  L2.x * ro.x + L2.y * ro.y + L2.z * ro.z + L2.w);
            const float3 ld = mk3(L0.x * rd.x + L0.y * rd.y + L0.z * rd.z, L1.x * rd.x + L1.y * rd.y + L1.z * rd.z,
                                  L2.x * rd.x + L2.y * rd.y + L2.z * rd.z);
            const float3 pl = lo + ld * h.x;
            auto normalT = [&](float3 v) {
                return mk3(L0.x * v.x + L1.x * v.y + L2.x * v.z, L0.y * v.x + L1.y * v.y + L2.y * v.z,
                           L0.z * v.x + L1.z * v.y + L2.z * v.z);
            };
            n = normalize(normalT(n));
            its.geoN = normalize(normalT(fn));
            dpdu = mk3(W0.x * dpdu.x + W0.y * dpdu.y + W0.z * dpdu.z, W1.x * dpdu.x + W1.y * dpdu.y + W1.z * dpdu.z,
                       W2.x * dpdu.x + W2.y * dpdu.y + W2.z * dpdu.z);
            its.p = mk3(W0.x * pl.x + W0.y * pl.y + W0.z * pl.z + W0.w, W1.x * pl.x + W1.y * pl.y + W1.z * pl.z + W1.w,
                        W2.x * pl.x + W2.y * pl.y + W2.z * pl.z + W2.w);
        }
    } else {
        const float4 a = S.rectSh[2 * (size_t)(p & 0x7FFFFFFFu)], b = S.rectSh[2 * (size_t)(p & 0x7FFFFFFFu) + 1];
        its.shape = (int)__float_as_uint(a.w);
        const uint32_t be = __float_as_uint(b.w);
        its.bsdf = (int)(be & 0xFFFFu);
        its.emitter = (int)(be >> 16) - 1;
        its.geoN = xyz(a);
        n = its.geoN;
        dpdu = xyz(b);
        its.p = ro + rd * h.x;
    }
    its.sh.n = n;
    its.sh.s = normalize(dpdu - n * dot(n, dpdu));
    its.sh.t = cross(n, its.sh.s);
}

// `bitmap` texture value of a hit (Texture2D::eval(its, filter),
// texture.cpp:112-121, over BitmapTexture::eval, bitmap.cpp:431-499, times
// the ScaleTexture of ensureEnergyConservation).  The hit's uv and dpdv come
// from the triangle's texture record (skdtree.h:369-405; rectangles:
// rectangle.cpp:155-164), dpdu from its shading record; instances map both
// tangents with toWorld (instance.cpp:146-160).  diffs: the camera ray's
// scaled differentials rxD / ryD exist (bounce 0), so the lookup is filtered
// with the UV partials of Intersection::computePartials (intersection.cpp:5-80)
DEV float3 texture_eval(const DevScene &S, int tex, float4 h, uint32_t inst, const Its &its, float3 ro, bool diffs, float3 rxD,
                        float3 ryD) {
#pragma clang fp contract(off)
    const mtsg_texture &T = S.textures[tex];
    const DevMip M{&T.mip, S.tex_texels};
    const uint32_t p = __float_as_uint(h.w);
    float2 uv;
    float3 dpdu, dpdv;
    if (!(p & 0x80000000u)) {
        const float4 *t = S.ttex + 3 * (size_t)p;
        const float4 t0 = t[0], t1 = t[1], t2 = t[2];
        const float bx = 1 - h.y - h.z, by = h.y, bz = h.z;
        uv = make_float2(t0.x * bx + t0.z * by + t1.x * bz, t0.y * bx + t0.w * by + t1.y * bz);
        dpdv = mk3(t1.z, t1.w, t2.x);
        const float4 *rec = S.shrec + 6 * (size_t)p;
        const float4 r4 = rec[4], r5 = rec[5];
        dpdu = mk3(r4.z, r4.w, r5.x);
        if (inst != 0xFFFFFFFFu) {
            const float4 *I = S.inst + 8 * (size_t)inst;
            const float4 W0 = I[3], W1 = I[4], W2 = I[5];
            dpdu = mk3(W0.x * dpdu.x + W0.y * dpdu.y + W0.z * dpdu.z, W1.x * dpdu.x + W1.y * dpdu.y + W1.z * dpdu.z,
                       W2.x * dpdu.x + W2.y * dpdu.y + W2.z * dpdu.z);
            dpdv = mk3(W0.x * dpdv.x + W0.y * dpdv.y + W0.z * dpdv.z, W1.x * dpdv.x + W1.y * dpdv.y + W1.z * dpdv.z,
                       W2.x * dpdv.x + W2.y * dpdv.y + W2.z * dpdv.z);
        }
    } else {
        const mtsg_rect &r = S.rects[p & 0x7FFFFFFFu];
        uv = make_float2(0.5f * (h.y + 1), 0.5f * (h.z + 1));
        dpdu = ld3(r.dpdu);
        dpdv = ld3(r.dpdv);
    }
    const float2 uvs = make_float2(uv.x * T.uv_scale[0] + T.uv_offset[0], uv.y * T.uv_scale[1] + T.uv_offset[1]);
    float3 value;
    if (diffs && T.mip.filter >= MTSG_MIP_TRILINEAR) {
        float dudx = 0, dvdx = 0, dudy = 0, dvdy = 0;
        const float3 n = its.geoN;
        if (!(isZero(dpdu) && isZero(dpdv))) {
            const float pp = dot(n, its.p), po = dot(n, ro), prx = dot(n, rxD), pry = dot(n, ryD);
            if (!(prx == 0 || pry == 0)) {
                const float tx = (pp - po) / prx, ty = (pp - po) / pry;
                const float ax = fabsf(n.x), ay = fabsf(n.y), az = fabsf(n.z);
                int a0, a1;
                if (ax > ay && ax > az) { a0 = 1; a1 = 2; }
                else if (ay > az) { a0 = 0; a1 = 2; }
                else { a0 = 0; a1 = 1; }
                auto c = [](float3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); };
                const float A00 = c(dpdu, a0), A01 = c(dpdv, a0), A10 = c(dpdu, a1), A11 = c(dpdv, a1);
                const float3 px = ro + rxD * tx, py = ro + ryD * ty;
                const float Bx0 = c(px, a0) - c(its.p, a0), Bx1 = c(px, a1) - c(its.p, a1);
                const float By0 = c(py, a0) - c(its.p, a0), By1 = c(py, a1) - c(its.p, a1);
                // solveLinearSystem2x2 (util.cpp:527-539); on failure dudx = 1,
                // dvdx = 0, dudy = 1 (the reference leaves dvdy unset: 0 here)
                const float det = A00 * A11 - A01 * A10;
                if (fabsf(det) <= 0x1p-128f) {
                    dudx = 1; dvdx = 0; dudy = 1; dvdy = 0;
                } else {
                    const float inv = 1.0f / det;
                    dudx = (A11 * Bx0 - A01 * Bx1) * inv;
                    dvdx = (A00 * Bx1 - A10 * Bx0) * inv;
                    dudy = (A11 * By0 - A01 * By1) * inv;
                    dvdy = (A00 * By1 - A10 * By0) * inv;
                }
            }
        }
        value = mip_filtered(M, uvs.x, uvs.y, dudx * T.uv_scale[0], dvdx * T.uv_scale[1], dudy * T.uv_scale[0], dvdy * T.uv_scale[1]);
    } else {
        value = T.mip.filter == MTSG_MIP_NEAREST ? mip_box(M, 0, uvs.x, uvs.y) : mip_bilinear(M, 0, uvs.x, uvs.y);
    }
    return value * T.scale;
}

// Shape::sampleDirect over TriMesh / Rectangle samplePosition (shape.cpp:102-115,
// trimesh.cpp:412-423, triangle.cpp:24-60, rectangle.cpp:200-207)
DEV void emitter_sample_position(const DevScene &S, const mtsg_emitter &em, uint32_t ei, float sx, float sy, float3 &p,
                                 float3 &n) {
    const float4 *er = S.emitRect + 4 * (size_t)ei;
    const float4 r0 = er[0], r1 = er[1], r2 = er[2], r3 = er[3];
    if (__float_as_uint(r3.w) == (uint32_t)MTSG_SHAPE_MESH) {
        const mtsg_shape &sh = S.shapes[em.shape];
        float pdfDummy;
        uint32_t index = pmf_sample_reuse(S.emitter_tri_cdf + em.cdf_offset, sh.tri_count, sy, pdfDummy);
        const uint4 ti = S.tidx[sh.tri_begin + index];
        const float3 p0 = xyz(S.vpos[ti.x]), p1 = xyz(S.vpos[ti.y]), p2 = xyz(S.vpos[ti.z]);
        float a = sqrtf(fmaxf(0.0f, 1.0f - sx));
        float bx = 1 - a, by = a * sy;
        float3 sideA = p1 - p0, sideB = p2 - p0;
        p = p0 + (sideA * bx) + (sideB * by);
        if (!sh.face_normals)
            n = normalize(xyz(S.vnrm[ti.x]) * (1.0f - bx - by) + xyz(S.vnrm[ti.y]) * bx + xyz(S.vnrm[ti.z]) * by);
        else
            n = normalize(cross(sideA, sideB));
    } else {
        const float x = sx * 2 - 1, y = sy * 2 - 1;
        p = mk3(r0.x * x + r0.y * y + r0.w, r1.x * x + r1.y * y + r1.w, r2.x * x + r2.y * y + r2.w);
        n = xyz(r3);
    }
}

// Block-aggregated queue append: one LDS atomic per wave, one global atomic
// per workgroup and queue (a contended global word costs ~11 ns per atomic).
struct BlockAppend {
    uint32_t cnt[2];
    uint32_t base[2];
    uint32_t bin[8];   // block_append2_oct: survivors per direction octant, then their offsets
};

#ifndef MTSG_SORT_OCT
#define MTSG_SORT_OCT 0   // variant: a workgroup's survivors grouped by direction octant
#endif
// block_append2 with the survivors (p1) of the workgroup grouped by key (the
// octant of the continuation direction): a trace wave takes consecutive work
// list entries, so its lanes then start from nearby origins (paths of one
// workgroup) in one octant.  The order of the paths does not change the
// image (the random numbers are keyed by pixel and sample).
DEV void block_append2_oct(BlockAppend &ba, uint32_t *gcnt0, uint32_t *gcnt1, bool p0, bool p1, uint32_t key,
                           uint32_t &i0, uint32_t &i1) {
    if (threadIdx.x < 8) ba.bin[threadIdx.x] = 0;
    if (threadIdx.x == 0) ba.cnt[0] = 0;
    __syncthreads();
    const unsigned long long below = (1ull << lane_id()) - 1ull;
    const unsigned long long m0 = __ballot(p0);
    uint32_t w0 = 0;
    if (lane_id() == 0 && m0) w0 = atomicAdd(&ba.cnt[0], (uint32_t)__popcll(m0));
    w0 = __shfl(w0, 0);
    uint32_t rank = 0, wk = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
        const unsigned long long mk = __ballot(p1 && key == k);
        uint32_t w = 0;
        if (lane_id() == 0 && mk) w = atomicAdd(&ba.bin[k], (uint32_t)__popcll(mk));
        w = __shfl(w, 0);
        if (key == k) { rank = (uint32_t)__popcll(mk & below); wk = w; }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ba.base[0] = ba.cnt[0] ? atomicAdd(gcnt0, ba.cnt[0]) : 0u;
        uint32_t run = 0;
        for (int k = 0; k < 8; ++k) { const uint32_t c = ba.bin[k]; ba.bin[k] = run; run += c; }
        ba.base[1] = run ? atomicAdd(gcnt1, run) : 0u;
    }
    __syncthreads();
    i0 = ba.base[0] + w0 + (uint32_t)__popcll(m0 & below);
    i1 = ba.base[1] + ba.bin[key & 7u] + wk + rank;
}

DEV void block_append2(BlockAppend &ba, uint32_t *gcnt0, uint32_t *gcnt1, bool p0, bool p1, uint32_t &i0, uint32_t &i1) {
    if (threadIdx.x == 0) { ba.cnt[0] = 0; ba.cnt[1] = 0; }
    __syncthreads();
    const unsigned long long m0 = __ballot(p0), m1 = __ballot(p1);
    const unsigned long long below = (1ull << lane_id()) - 1ull;
    uint32_t w0 = 0, w1 = 0;
    if (lane_id() == 0) {
        if (m0) w0 = atomicAdd(&ba.cnt[0], (uint32_t)__popcll(m0));
        if (m1) w1 = atomicAdd(&ba.cnt[1], (uint32_t)__popcll(m1));
    }
    w0 = __shfl(w0, 0);
    w1 = __shfl(w1, 0);
    __syncthreads();
    if (threadIdx.x == 0) {
        ba.base[0] = ba.cnt[0] ? atomicAdd(gcnt0, ba.cnt[0]) : 0u;
        ba.base[1] = ba.cnt[1] ? atomicAdd(gcnt1, ba.cnt[1]) : 0u;
    }
    __syncthreads();
    i0 = ba.base[0] + w0 + (uint32_t)__popcll(m0 & below);
    i1 = ba.base[1] + w1 + (uint32_t)__popcll(m1 & below);
}

// outgoing records of one workgroup: 7 rows of 16 B per lane, 28 KB, so with
// the staged tables a 256-thread workgroup stays under 32 KB and 5 fit a CU
// (5 waves/SIMD; 9 rows, 36 KB, held k_shade at 4).  The continuation origin
// and the shadow origin are the same point (its.p), and the constant .w words
// of the outgoing rays (mint = Epsilon, maxt = inf; shadow mint = Epsilon)
// carry the path's meta words instead (depth | flags, dimension, 2D
// requests; the slot is the caller's): the write-out restores the constants.
struct ShadeStage {
    float4 p[SHADE_BLOCK];     // its.p, shadow maxt
    float4 d[SHADE_BLOCK];     // continuation direction, meta.x
    float4 T[SHADE_BLOCK], aux[SHADE_BLOCK], L[SHADE_BLOCK];
    float4 shd[SHADE_BLOCK];   // shadow direction, meta.y
    float4 shc[SHADE_BLOCK];   // NEE contribution, meta.w
};

// One bounce of one path (the body of MIPathTracer::Li's loop, path.cpp:119-294,
// entered after scene->rayIntersect): reads the path at position i of the
// current arrays and its hit, and hands the outgoing records to `out`
// (Out::shadow: NEE shadow ray + contribution; Out::next: continuation ray;
// Out::state: throughput, radiance, meta of a continuing path).  A path that
// ends writes its sample's final radiance.  first: bounce 0 (camera rays).
// the small per-scene tables a path reads after its shading record: the BSDF
// records, the emitters and their discrete CDF.  k_shade stages them in LDS
// when they are small (MTSG_SHADE_LDS), so those reads are not another L2
// round trip in each path's chain of dependent loads; elsewhere they point
// at the scene's global arrays.
struct ShadeTables {
    const mtsg_bsdf *bsdfs;
    const mtsg_emitter *emitters;
    const float *emitter_cdf;
};
DEV ShadeTables global_tables(const DevScene &S) { return ShadeTables{S.bsdfs, S.emitters, S.emitter_cdf}; }

// the path's records at position i that do not depend on its meta word:
// loaded together with it, so the hit -> shading record chain starts one
// memory round trip earlier (k_shade issues them before it knows whether a
// bounce-0 slot is live)
struct PathLoads {
    float4 h, ro4, rd4, L4, T4;
};
DEV PathLoads load_path(const DevScene &S, const DevPaths &P, uint32_t i, bool first) {
    PathLoads pl;
    pl.h = ldS(&P.hit[i]);
    load_closest_ray(S, P, i, first && S.camCompact, pl.ro4, pl.rd4);
    // a camera path starts with L = 0, alpha 1, T = 1, eta = 1: k_camera writes
    // no L, and no T unless it holds the ray differentials (cam_diffs)
    const bool fresh = first && !S.cam_diffs;
    pl.L4 = first ? make_float4(0.f, 0.f, 0.f, 1.f) : ldS(&P.Lp[i]);
    pl.T4 = fresh ? make_float4(1.f, 1.f, 1.f, 1.f) : ldS(&P.T[i]);
    return pl;
}
DEV PathLoads load_path_rest(const DevScene &S, const DevPaths &P, uint32_t i, bool first) {
    PathLoads pl;
    load_closest_ray(S, P, i, first && S.camCompact, pl.ro4, pl.rd4);
    const bool fresh = first && !S.cam_diffs;
    pl.L4 = first ? make_float4(0.f, 0.f, 0.f, 1.f) : ldS(&P.Lp[i]);
    pl.T4 = fresh ? make_float4(1.f, 1.f, 1.f, 1.f) : ldS(&P.T[i]);
    return pl;
}
// MTSG_SHADE_PRELOAD: what k_shade loads together with the meta word (1:
// every record of load_path, 2: the hit only, 0: nothing -- round 3)
#ifndef MTSG_SHADE_PRELOAD
#define MTSG_SHADE_PRELOAD 0   // measured r04: 1 (all) C3 -0.5%, C5 -3.5% (spills at the 128-VGPR cap); 2 (hit) C3 -0.4%
#endif

template <bool ENV, int SMP, bool EXT, class Out, int MATS = MATS_ALL>
DEV void shade_path(const DevScene &S, const DevIntegrator &I, const DevBatch &B, const DevPaths &P, bool first, uint32_t i,
                    const uint4 meta, const PathLoads &pl, int hasAlpha, Out &out, bool &cont, bool &shadow,
                    const ShadeTables &tb) {
    const uint32_t slot = meta.z;
    const float4 h = pl.h;
    const float3 ro = xyz(pl.ro4), rd = xyz(pl.rd4);
    float4 L4 = pl.L4;
    float4 T4 = pl.T4;
    PathSampler smp;
    {
        int x, y;
        uint32_t sIdx;
        slot_pixel(B, slot, x, y, sIdx);
        smp = path_sampler(I, x, y, sIdx, meta.y, meta.w);
    }
    float3 L = xyz(L4), T = xyz(T4);
    float eta = T4.w;
    uint32_t depth = meta.x & 0xFFFFu;
    uint32_t flags = meta.x & 0xFFFF0000u;
    const bool valid = __float_as_uint(h.w) != 0xFFFFFFFFu;
    bool done = false;
    Its its;
    const uint32_t inst = (valid && S.inst) ? P.hitInst[i] : 0xFFFFFFFFu;
    if (valid) fill_its(S, ro, rd, h, inst, its);
    float3 rxd = mk3(0, 0, 0), ryd = mk3(0, 0, 0);   // camera differentials (textured EXT scenes)
    if (first) {
        // RadianceQueryRecord::rayIntersect (records.inl:117-143)
        if (hasAlpha) L4.w = valid ? 1.0f : 0.0f;
        if (!valid) {
            // Scene::evalEnvironment of the differential camera ray (path.cpp:136-143)
            if (ENV && !I.hide_emitters) {
                float3 rxd, ryd;
                if (S.cam_diffs) {
                    rxd = T;
                    ryd = xyz(ldS(&P.aux[i]));
                } else {   // (cam_env_diffs) recomputed from the camera, bit for bit as k_camera's
                    int x, y;
                    uint32_t sIdx;
                    slot_pixel(B, slot, x, y, sIdx);
                    camera_ray_differentials<SMP>(*S.camDev, I, x, y, sIdx, rxd, ryd);
                }
                L += env_eval(S.env, rd, true, rxd, ryd);   // throughput 1
            }
            done = true;
        }
        if (S.cam_diffs) {   // T / aux held the camera's scaled differentials
            if (EXT && S.textures) { rxd = T; ryd = xyz(ldS(&P.aux[i])); }
            T = mk3(1.f, 1.f, 1.f);
        }
    } else {
        // tail of the previous iteration after scene->rayIntersect (path.cpp:226-286)
        if (!valid) {
            // environment hit by the BSDF sample (path.cpp:236-246, 257-265)
            if (ENV && !(I.hide_emitters && !(flags & F_SCATTERED))) {
                // evalEnvironment and pdfDirect look the same local
                // direction up (envmap.cpp:386-387, 606-607): its atan2f /
                // acosf are evaluated once for both
                const float3 v = env_rot(S.env.E->to_local, rd);
                float ux, uy;
                env_uv(v, ux, uy);
                const float3 value = env_eval_uv(S.env, v, ux, uy, false, rd, rd);
                float nearT, farT;
                if (env_sphere(S.env, ro, rd, nearT, farT) && !(nearT > 0) && !(farT < 0)) {
                    float lumPdf = 0.0f;
                    if (!(flags & F_DELTA))   // Scene::pdfEmitterDirect -> EnvironmentMap::pdfDirect
                        lumPdf = env_internal_pdf_uv(S.env, v, ux, uy) * tb.emitters[S.env.E->emitter].pdf_discrete;
                    L += T * value * mis(ldS(&P.aux[i]).w, lumPdf);
                }
            }
            done = true;
        } else {
            const int em = its.emitter;
            if (em >= 0) {
                const mtsg_emitter &E = tb.emitters[em];
                const float3 value = dot(its.sh.n, -rd) > 0 ? ld3(E.radiance) : mk3(0, 0, 0);
                float lumPdf = 0.0f;
                if (!(flags & F_DELTA)) {
                    // Scene::pdfEmitterDirect with dRec.setQuery(ray, its)
                    const float4 ax = ldS(&P.aux[i]);
                    const float3 refN = xyz(ax);
                    if (dot(rd, refN) >= 0 && dot(rd, its.sh.n) < 0)
                        lumPdf = E.inv_area * (h.x * h.x) / fabsf(dot(rd, its.sh.n));
                    lumPdf *= E.pdf_discrete;
                }
                L += T * value * mis(ldS(&P.aux[i]).w, lumPdf);
            }
            if (depth++ >= (uint32_t)I.rr_depth) {
                float q = fminf(maxc(T) * eta * eta, 0.95f);
                if (next1D<SMP>(I, smp) >= q) done = true;
                else T = T / q;
            }
        }
    }
    if (!done && !((int)depth <= I.max_depth || I.max_depth < 0)) done = true;
    if (!done) {
        const mtsg_bsdf &bsdf = tb.bsdfs[its.bsdf];
        const float3 wi = its.sh.toLocal(-rd);
        float3 alb;
        if (EXT) {
            const mtsg_bsdf &eff = (bsdf.twosided && !(wi.z > 0)) ? tb.bsdfs[bsdf.back] : bsdf;
            alb = eff.texture ? texture_eval(S, eff.texture - 1, h, inst, its, ro, first && S.cam_diffs, rxd, ryd)
                              : ld3(eff.reflectance);
        } else {
            alb = ld3(bsdf.reflectance);
        }
        if (first && its.emitter >= 0 && !I.hide_emitters) {
            if (dot(its.sh.n, -rd) > 0) L += T * ld3(tb.emitters[its.emitter].radiance);
        }
        if (((int)depth >= I.max_depth && I.max_depth > 0) ||
            (I.strict_normals && dot(rd, its.geoN) * wi.z >= 0)) {
            done = true;
        } else {
            const float3 refN = bsdf.ref_n_zero ? mk3(0, 0, 0) : its.sh.n;
            // ---- direct illumination (path.cpp:172-200)
            if (bsdf.smooth) {
                float sx, sy;
                next2D<SMP>(I, smp, sx, sy);
                float emPdf;
                const uint32_t ei = pmf_sample_reuse(tb.emitter_cdf, S.n_emitters, sx, emPdf);
                const mtsg_emitter &E = tb.emitters[ei];
                float3 dd, value;
                float dist, pdf;
                bool accepted;
                if (ENV && E.type == MTSG_EMITTER_ENVMAP) {
                    accepted = env_sample_direct(S.env, its.p, sx, sy, dd, dist, value, pdf);
                } else {
                    float3 ep, en;
                    emitter_sample_position(S, E, ei, sx, sy, ep, en);
                    dd = ep - its.p;
                    const float distSquared = dot(dd, dd);
                    dist = sqrtf(distSquared);
                    dd = dd / dist;
                    const float dp = fabsf(dot(dd, en));
                    pdf = E.inv_area * (dp != 0 ? (distSquared / dp) : 0.0f);
                    accepted = dot(dd, refN) >= 0 && dot(dd, en) < 0 && pdf != 0;
                    if (accepted) value = ld3(E.radiance) / pdf;
                }
                if (accepted) {
                    pdf *= emPdf;
                    value = value / emPdf;
                    const float3 wo = its.sh.toLocal(dd);
                    float bpdf;
                    const float3 bval = bsdf_eval<EXT, MATS>(S.bsdfs, bsdf, alb, wi, wo, bpdf);
                    if (!isZero(bval) && (!I.strict_normals || dot(its.geoN, dd) * wo.z > 0)) {
                        const float weight = mis(pdf, bpdf);
                        const float3 c = T * value * bval * weight;
                        if (!isZero(c)) {
                            shadow = true;
                            out.shadow(make_float4(its.p.x, its.p.y, its.p.z, dist * (1 - kShadowEpsilon)),
                                       make_float4(dd.x, dd.y, dd.z, kEpsilon), make_float4(c.x, c.y, c.z, 0.f));
                        }
                    }
                }
            }
            // ---- BSDF sampling (path.cpp:206-221)
            float sx, sy;
            next2D<SMP>(I, smp, sx, sy);
            BsdfSample bs;
            if (!bsdf_sample<EXT, MATS>(S.bsdfs, bsdf, alb, wi, sx, sy, bs, [&]() { return next1D<SMP>(I, smp); })) {
                done = true;
            } else {
                flags |= F_SCATTERED;
                const float3 wo = its.sh.toWorld(bs.wo);
                if (I.strict_normals && dot(its.geoN, wo) * bs.wo.z <= 0) {
                    done = true;
                } else {
                    T = T * bs.weight;
                    eta *= bs.eta;
                    flags = bs.delta ? (flags | F_DELTA) : (flags & ~F_DELTA);
                    out.next(make_float4(its.p.x, its.p.y, its.p.z, kEpsilon), make_float4(wo.x, wo.y, wo.z, INFINITY),
                             make_float4(refN.x, refN.y, refN.z, bs.pdf));
                    cont = true;
                }
            }
        }
    }
    if ((SMP == MTSG_SAMPLER_HALTON || SMP == MTSG_SAMPLER_HAMMERSLEY || SMP == MTSG_SAMPLER_SOBOL) && smp.dimError)
        atomicOr(&P.cnt[CNT_ERR], CNT_ERR_QMC_DIM);   // the render fails as Mitsuba's Log(EError) would
    const float4 finalL = make_float4(L.x, L.y, L.z, L4.w);
    if (cont) {
        out.state(make_float4(T.x, T.y, T.z, eta), finalL, make_uint4(depth | flags, smp.dim, slot, smp.n2));
    } else {
        stS(&P.L[slot], finalL);   // path ended: its sample's final radiance
    }
}

// ---------------------------------------------------------------------------
// myPath2_OM: the fork's path tracer with occupancy-map visibility
// (src/integrators/testOM/myPath2_OM.cpp:317-485, myOM.h)
// ---------------------------------------------------------------------------
// OccupancyMap::nearestOMindex over direct2uv (myOM.h:603-615,
// testOM/helpers.h:6-44).  Like the reference, it flips d in place when
// d.z < 0 (the caller's direction stays flipped).  The mixed float / double
// arithmetic follows the reference's expressions (M_PI is a double).
DEV int om_index(float3 &d) {
#pragma clang fp contract(off)
    if (d.z < 0) d = -d;
    const double PI = 3.14159265358979323846;
    const float r = sqrtf(1 - d.z);
    float phi = mt_atan2f(d.y, d.x);
    float u = 0, v = 0;
    if (r != 0) {
        float a, b;
        if ((double)phi < -PI / 4) phi = (float)((double)phi + 2 * PI);
        if ((double)phi < PI / 4) {
            a = r;
            b = (float)((double)(phi * a) / (PI / 4));
        } else if ((double)phi < PI * 3 / 4) {
            b = r;
            a = (float)(-((double)phi - PI / 2) * (double)b / (PI / 4));
        } else if ((double)phi < PI * 5 / 4) {
            a = -r;
            b = (float)(((double)phi - PI) * (double)a / (PI / 4));
        } else {
            b = -r;
            a = (float)(-((double)phi - PI * 3 / 2) * (double)b / (PI / 4));
        }
        u = (a + 1) / 2;
        v = (b + 1) / 2;
    }
    if ((double)u > 0.999999) u = (float)0.999999;
    if ((double)v > 0.999999) v = (float)0.999999;
    return (int)floorf(u * MTSG_OM_SQRT) * MTSG_OM_SQRT + (int)floorf(v * MTSG_OM_SQRT);
}

// OccupancyMap::Visible(o1, o2) of rotated map `id` (myOM.h:383-503, the
// 32-bit column path): o1 rotated into the map's frame, o2 placed `length`
// along m_dir from it, and the z cells strictly between theirs tested in
// the (x, y) column.  The reference accepts x == 256 / y == 256 and reads
// past the column array there; this build answers "visible".
DEV bool om_visible(const DevScene &S, int id, float3 o1, float3 o2) {
#pragma clang fp contract(off)
    const mtsg_om &O = *S.om;
    const float3 dir = mk3(O.dir[id][0], O.dir[id][1], O.dir[id][2]);
    const float3 o21 = o2 - o1;
    float len = sqrtf(o21.x * o21.x + o21.y * o21.y + o21.z * o21.z);
    if (dot(dir, o21) < 0) len = -len;
    const float *m = O.rotate[id];
    const float3 c = mk3(O.center[0], O.center[1], O.center[2]);
    const float3 q = o1 - c;   // Point - Vector
    const float3 a1 = mk3(m[0] * q.x + m[1] * q.y + m[2] * q.z + 0.0f, m[3] * q.x + m[4] * q.y + m[5] * q.z + 0.0f,
                          m[6] * q.x + m[7] * q.y + m[8] * q.z + 0.0f) + c;
    const float3 a2 = a1 + dir * len;
    const float rc = O.grid_size_recp;
    const int x = (int)floorf((a1.x - O.aabb_min[0]) * rc + kEpsilon), y = (int)floorf((a1.y - O.aabb_min[1]) * rc + kEpsilon);
    if (x < 0 || x >= MTSG_OM_SIZE || y < 0 || y >= MTSG_OM_SIZE) return true;
    int z1 = (int)floorf((a1.z - O.aabb_min[2]) * rc + kEpsilon), z2 = (int)floorf((a2.z - O.aabb_min[2]) * rc + kEpsilon);
    if (z1 > z2) { const int t = z1; z1 = z2; z2 = t; }
    if (z2 - z1 < 2) return true;
    z1 = min(max(z1 + 1, 0), MTSG_OM_SIZE - 1);
    z2 = min(max(z2 - 1, 0), MTSG_OM_SIZE - 1);
    const uint32_t *col = S.om_bits + (((size_t)id * MTSG_OM_SIZE + x) * MTSG_OM_SIZE + y) * (MTSG_OM_SIZE / 32);
    const int p1 = z1 >> 5, p2 = z2 >> 5, r1 = z1 & 31, r2 = (31 - z2) & 31;
    if (p1 == p2) return ((col[p1] >> r1) << (r1 + r2)) == 0u;
    if ((col[p1] >> r1) != 0u) return false;
    for (int k = p1 + 1; k < p2; ++k)
        if (col[k] != 0u) return false;
    return (col[p2] << r2) == 0u;
}

// nearestOMindex + Visible for the parity tests (mtsg_om_query)
__global__ void k_om_query(DevScene S, const float *dirs, const float *o1, const float *o2, uint32_t n, int32_t *ids, int32_t *vis) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float3 d = mk3(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
    const int id = om_index(d);
    ids[i] = id;
    vis[i] = om_visible(S, id, mk3(o1[3 * i], o1[3 * i + 1], o1[3 * i + 2]), mk3(o2[3 * i], o2[3 * i + 1], o2[3 * i + 2])) ? 1 : 0;
}

// myPath2OMIntegrator::mis / misWeight (myPath2_OM.cpp:276-314)
DEV float om_mis(const DevIntegrator &I, float p1, float p2) {
    if (I.om_mis == MTSG_OM_MIS_UNIFORM) return 0.5f;
    if (I.om_mis == MTSG_OM_MIS_BALANCE) return p1 / (p1 + p2);
    return (p1 * p1) / ((p1 * p1) + (p2 * p2));
}
DEV float om_weight_nee(const DevIntegrator &I, float pdfBSDF, float pdfDirect) {
    if (I.om_strategy == MTSG_OM_STRATEGY_BSDF) return 0.0f;
    if (I.om_strategy == MTSG_OM_STRATEGY_NEE) return 1.0f;
    return om_mis(I, pdfDirect, pdfBSDF);
}
DEV float om_weight_bsdf(const DevIntegrator &I, float pdfBSDF, float pdfDirect) {
    if (I.om_strategy == MTSG_OM_STRATEGY_BSDF) return 1.0f;
    if (I.om_strategy == MTSG_OM_STRATEGY_NEE) return 0.0f;
    return om_mis(I, pdfBSDF, pdfDirect);
}

// One iteration of myPath2OMIntegrator::Li (myPath2_OM.cpp:386-485) for the
// path at position i; the independent sampler only (see build.cpp).
// Bounce 0: a camera ray that hits an emitter returns its radiance (:396-397).
// Later bounces first finish the previous iteration: a BSDF ray that found
// an emitter adds its MIS-weighted emission and ends the path (:462-472),
// otherwise Russian roulette (:475-479) and ++depth.  Then next-event
// estimation against occupancy-map visibility and the BSDF sample.
template <bool EXT, class Out>
DEV void shade_path_om(const DevScene &S, const DevIntegrator &I, const DevBatch &B, const DevPaths &P, bool first, uint32_t i,
                       const uint4 meta, Out &out, bool &cont) {
    constexpr int SMP = MTSG_SAMPLER_INDEPENDENT;
    const uint32_t slot = meta.z;
    const float4 h = ldS(&P.hit[i]);
    float4 ro4, rd4;
    load_closest_ray(S, P, i, first && S.camCompact, ro4, rd4);
    const float3 ro = xyz(ro4), rd = xyz(rd4);
    const float4 L4 = first ? make_float4(0.f, 0.f, 0.f, 1.f) : ldS(&P.Lp[i]);   // camera paths: see shade_path
    const float4 T4 = first ? make_float4(1.f, 1.f, 1.f, 1.f) : ldS(&P.T[i]);
    PathSampler smp;
    {
        int x, y;
        uint32_t sIdx;
        slot_pixel(B, slot, x, y, sIdx);
        smp = path_sampler(I, x, y, sIdx, meta.y, meta.w);
    }
    float3 L = xyz(L4), T = xyz(T4);
    float eta = T4.w;
    uint32_t depth = meta.x & 0xFFFFu;
    uint32_t flags = meta.x & 0xFFFF0000u;
    const bool valid = __float_as_uint(h.w) != 0xFFFFFFFFu;
    bool done = false;
    Its its;
    const uint32_t inst = (valid && S.inst) ? P.hitInst[i] : 0xFFFFFFFFu;
    if (valid) fill_its(S, ro, rd, h, inst, its);
    if (first) {
        if (valid && its.emitter >= 0) {   // its.Le(-ray.d) (area.cpp:104-109)
            if (dot(its.sh.n, -rd) > 0) L = ld3(S.emitters[its.emitter].radiance);
            done = true;
        }
    } else {
        if (valid && its.emitter >= 0) {
            const mtsg_emitter &E = S.emitters[its.emitter];
            const float3 value = dot(its.sh.n, -rd) > 0 ? ld3(E.radiance) : mk3(0, 0, 0);
            float lumPdf = 0.0f;
            const float4 ax = ldS(&P.aux[i]);
            if (!(flags & F_DELTA)) {   // Scene::pdfEmitterDirect after dRec.setQuery(ray, its)
                if (dot(rd, xyz(ax)) >= 0 && dot(rd, its.sh.n) < 0) lumPdf = E.inv_area * (h.x * h.x) / fabsf(dot(rd, its.sh.n));
                lumPdf *= E.pdf_discrete;
            }
            L += T * value * om_weight_bsdf(I, ax.w, lumPdf);
            done = true;   // return Li
        } else {
            const float q = fminf(maxc(T) * eta * eta, 0.95f);
            if (next1D<SMP>(I, smp) >= q) done = true;
            else T = T / q;
            ++depth;
        }
    }
    if (!done && ((int)depth > I.max_depth || !valid)) done = true;
    if (!done) {
        const mtsg_bsdf &bsdf = S.bsdfs[its.bsdf];
        const float3 wi = its.sh.toLocal(-rd);
        float3 alb;
        if (EXT) {   // rays from sensor->sampleRay carry no differentials: unfiltered lookups
            const mtsg_bsdf &eff = (bsdf.twosided && !(wi.z > 0)) ? S.bsdfs[bsdf.back] : bsdf;
            alb = eff.texture ? texture_eval(S, eff.texture - 1, h, inst, its, ro, false, ro, ro) : ld3(eff.reflectance);
        } else {
            alb = ld3(bsdf.reflectance);
        }
        const float3 refN = bsdf.ref_n_zero ? mk3(0, 0, 0) : its.sh.n;
        if (bsdf.smooth) {
            // scene->sampleEmitterDirect(dRec, next2D, testVisibility = false)
            float sx, sy;
            next2D<SMP>(I, smp, sx, sy);
            float emPdf;
            const uint32_t ei = pmf_sample_reuse(S.emitter_cdf, S.n_emitters, sx, emPdf);
            const mtsg_emitter &E = S.emitters[ei];
            float3 dd, value, ep = mk3(0, 0, 0);
            float dist, pdf;
            bool accepted, onSurface = true;
            if (S.has_env && E.type == MTSG_EMITTER_ENVMAP) {
                accepted = env_sample_direct(S.env, its.p, sx, sy, dd, dist, value, pdf);
                if (accepted) ep = its.p + dd * dist;   // ray(farT)
                onSurface = false;
            } else {
                float3 en;
                emitter_sample_position(S, E, ei, sx, sy, ep, en);
                dd = ep - its.p;
                const float distSquared = dot(dd, dd);
                dist = sqrtf(distSquared);
                dd = dd / dist;
                const float dp = fabsf(dot(dd, en));
                pdf = E.inv_area * (dp != 0 ? (distSquared / dp) : 0.0f);
                accepted = dot(dd, refN) >= 0 && dot(dd, en) < 0 && pdf != 0;
                if (accepted) value = ld3(E.radiance) / pdf;
            }
            if (accepted) {
                pdf *= emPdf;
                value = value / emPdf;
            } else {
                value = mk3(0, 0, 0);
            }
            // roma[nearestOMindex(dRec.d)].Visible(its.p + its.shFrame.n * 0.5, dRec.p)
            // (the reference evaluates it twice, for its timing, with the same answer)
            const int id = om_index(dd);
            const bool vis = om_visible(S, id, its.p + its.sh.n * 0.5f, ep);
            if (vis && !isZero(value)) {
                const float3 wo = its.sh.toLocal(dd);   // the possibly flipped dRec.d, as in the reference
                float bpdf;
                const float3 bval = bsdf_eval<EXT>(S.bsdfs, bsdf, alb, wi, wo, bpdf);
                if (!isZero(bval)) {
                    const float bsdfPdf = onSurface ? bpdf : 0.0f;   // isOnSurface && ESolidAngle
                    L += T * value * bval * om_weight_nee(I, bsdfPdf, pdf);
                }
            }
        }
        float sx, sy;
        next2D<SMP>(I, smp, sx, sy);
        BsdfSample bs;
        if (!bsdf_sample<EXT>(S.bsdfs, bsdf, alb, wi, sx, sy, bs, [&]() { return next1D<SMP>(I, smp); })) {
            done = true;
        } else {
            const float3 wo = its.sh.toWorld(bs.wo);
            T = T * bs.weight;
            eta *= bs.eta;
            flags = bs.delta ? (flags | F_DELTA) : (flags & ~F_DELTA);
            out.next(make_float4(its.p.x, its.p.y, its.p.z, kEpsilon), make_float4(wo.x, wo.y, wo.z, INFINITY),
                     make_float4(refN.x, refN.y, refN.z, bs.pdf));
            cont = true;
        }
    }
    const float4 finalL = make_float4(L.x, L.y, L.z, L4.w);
    if (cont) out.state(make_float4(T.x, T.y, T.z, eta), finalL, make_uint4(depth | flags, smp.dim, slot, smp.n2));
    else stS(&P.L[slot], finalL);
}

// k_shade's outgoing records: lane-private LDS rows until the block append
// (ShadeStage: the .w words of d / shd / shc hold meta.x / .y / .w; o.w and
// d.w are the constants kEpsilon / inf, shd.w kEpsilon, restored by stage_write)
struct StageOut {
    ShadeStage &st;
    DEV void shadow(float4 o, float4 d, float4 c) {
        const int t = threadIdx.x;
        st.p[t] = o;
        st.shd[t].x = d.x; st.shd[t].y = d.y; st.shd[t].z = d.z;
        st.shc[t].x = c.x; st.shc[t].y = c.y; st.shc[t].z = c.z;
    }
    DEV void next(float4 o, float4 d, float4 aux) {
        const int t = threadIdx.x;
        st.p[t].x = o.x; st.p[t].y = o.y; st.p[t].z = o.z;
        st.d[t].x = d.x; st.d[t].y = d.y; st.d[t].z = d.z;
        st.aux[t] = aux;
    }
    DEV void state(float4 T, float4 L, uint4 meta) {
        const int t = threadIdx.x;
        st.T[t] = T;
        st.L[t] = L;
        st.d[t].w = __uint_as_float(meta.x);
        st.shd[t].w = __uint_as_float(meta.y);
        st.shc[t].w = __uint_as_float(meta.w);
    }
};
// a survivor's records into the next bounce's arrays at position ic, and a
// shadow ray into the shadow arrays at position is (sh_c.w: the target)
DEV void stage_write_next(const ShadeStage &st, const DevPaths &P, int tid, uint32_t ic, uint32_t slot) {
    const float4 p = st.p[tid], d = st.d[tid];
    stS(&P.n_ray_o[ic], make_float4(p.x, p.y, p.z, kEpsilon));
    stS(&P.n_ray_d[ic], make_float4(d.x, d.y, d.z, INFINITY));
    stS(&P.n_T[ic], st.T[tid]);
    stS(&P.n_aux[ic], st.aux[tid]);
    stS(&P.n_Lp[ic], st.L[tid]);
    stS(&P.n_meta[ic], make_uint4(__float_as_uint(d.w), __float_as_uint(st.shd[tid].w), slot, __float_as_uint(st.shc[tid].w)));
}
DEV void stage_write_shadow(const ShadeStage &st, const DevPaths &P, int tid, uint32_t is, uint32_t target) {
    const float4 d = st.shd[tid], c = st.shc[tid];
    stS(&P.sh_o[is], st.p[tid]);
    stS(&P.sh_d[is], make_float4(d.x, d.y, d.z, kEpsilon));
    stS(&P.sh_c[is], make_float4(c.x, c.y, c.z, __uint_as_float(target)));
}

// myPath2_OM's shading launch: one iteration of its Li per path (no shadow
// rays: visibility comes from the occupancy maps inside the kernel)
template <bool EXT>
__global__ void __launch_bounds__(SHADE_BLOCK) k_shade_om(DevScene S, DevIntegrator I, DevBatch B, DevPaths P, int bounce, int qin,
                                                        uint32_t nIdentity) {
    __shared__ BlockAppend ba;
    __shared__ ShadeStage stage;
    uint32_t count = nIdentity;
    if (qin >= 0) count = __atomic_load_n(&P.cnt[cnt_q(qin)], __ATOMIC_RELAXED);
    const uint32_t nIter = (count + gridDim.x * blockDim.x - 1) / (gridDim.x * blockDim.x);
    const int qout = qin < 0 ? 1 : (qin ^ 1);
    for (uint32_t it = 0; it < nIter; ++it) {
        const uint32_t i = (it * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
        bool alive = i < count;
        bool cont = false;
        uint4 meta = make_uint4(0u, 0u, 0u, 0u);
        if (alive) {
            meta = ldS(&P.meta[i]);
            if (meta.x == 0u) alive = false;   // dead slot (bounce 0)
        }
        if (alive) {
            StageOut out{stage};
            shade_path_om<EXT>(S, I, B, P, bounce == 0, i, meta, out, cont);
        }
        const int tid = threadIdx.x;
        uint32_t is, ic;
        block_append2(ba, &P.cnt[cnt_s(bounce & 1)], &P.cnt[cnt_q(qout)], false, cont, is, ic);
        if (cont) stage_write_next(stage, P, tid, ic, meta.z);
    }
}

// qin < 0: bounce 0 over the identity queue of nIdentity slots
#ifndef MTSG_SHADE_LDS
#define MTSG_SHADE_LDS 1   // BSDF / emitter tables staged in LDS when they fit (k_shade): +1.4% on C3
#endif
constexpr int SHADE_LDS_BSDFS = 4, SHADE_LDS_EMITTERS = 16;
#ifndef MTSG_SHADE_LDS_PAD
#define MTSG_SHADE_LDS_PAD 0
#endif
#ifndef MTSG_SHADE_WAVES
#define MTSG_SHADE_WAVES 4   // 127 VGPRs: 4 waves/SIMD (3 at 144; 5+ spill heavily)
#endif
// the material-specialised kernels (MATS != MATS_ALL) fit 96 VGPRs: with the
// 28-KB stage (ShadeStage) 5 workgroups share a CU, 5 waves/SIMD
#ifndef MTSG_SHADE_WAVES_MATS
#define MTSG_SHADE_WAVES_MATS 5
#endif
#ifndef MTSG_SHADE_WAVES_MATS_ENV
#define MTSG_SHADE_WAVES_MATS_ENV 5
#endif
#define SHADE_WAVES_OF(ENV, MATS) ((MATS) == MATS_ALL ? MTSG_SHADE_WAVES : (ENV) ? MTSG_SHADE_WAVES_MATS_ENV : MTSG_SHADE_WAVES_MATS)
#if MTSG_SHADE_WAVES > 0
#define SHADE_ATTR(ENV, MATS) __launch_bounds__(SHADE_BLOCK) __attribute__((amdgpu_waves_per_eu(SHADE_WAVES_OF(ENV, MATS))))
#else
#define SHADE_ATTR(ENV, MATS) __launch_bounds__(SHADE_BLOCK)
#endif
// Event order inside a workgroup (round 6): a wave runs the union of the code
// paths its lanes take, so a wave that mixes an environment miss, a
// dielectric hit and a smooth hit with next-event estimation pays all three.
// Before shading, each workgroup classifies its 256 paths -- dead slot, miss,
// or the BSDF class of the hit (dielectric / diffuse / roughconductor /
// other: path.cpp:145-264 dispatches on these) -- and hands them to its
// threads sorted by class, so most waves shade one kind of event: the
// per-material queues of SURVEY §7 step 6, kept inside the workgroup so the
// path state stays dense (the gathers stay within the workgroup's 256
// positions).  Which thread shades a path changes nothing in its arithmetic.
#ifndef MTSG_SHADE_SORT
#define MTSG_SHADE_SORT 1
#endif
// measured r06 (profiles/r06_shade_sort.txt): C5 shade 424 -> 410 ms; where
// the events barely diverge the classification only costs (C2, diffuse only:
// +3.0 ms; C3, no environment: +1.2 ms shade, -1.2 ms trace), so the sort is
// compiled into the kernels of scenes with an environment emitter (misses and
// environment sampling are their expensive events) and several classes
template <bool ENV, int MATS>
constexpr bool shade_sorted() { return MTSG_SHADE_SORT && ENV && (MATS & (MATS - 1)) != 0; }
constexpr int SHADE_CLASSES = 6;
DEV uint32_t shade_class(const DevScene &S, const DevBatch &B, const DevPaths &P, uint32_t i, bool first, const ShadeTables &tb) {
    if (first && camera_meta(B, i).x == 0u) return 0u;   // dead slot (bounce 0)
    const uint32_t p = __float_as_uint(P.hit[i].w);
    if (p == 0xFFFFFFFFu) return 1u;
    const uint32_t bsdf = !(p & 0x80000000u) ? __float_as_uint(S.shrec[6 * (size_t)p + 5].z) & 0x7FFFFFFFu
                                             : __float_as_uint(S.rectSh[2 * (size_t)(p & 0x7FFFFFFFu) + 1].w) & 0xFFFFu;
    const int t = tb.bsdfs[bsdf].type;
    return t == MTSG_BSDF_DIELECTRIC ? 2u : t == MTSG_BSDF_DIFFUSE ? 3u : t == MTSG_BSDF_ROUGHCONDUCTOR ? 4u : 5u;
}
// the workgroup's counting sort by class: returns the offset (within the
// workgroup's 256 positions) of the path this thread shades
DEV uint32_t shade_sort(uint32_t cls, uint32_t *cnt, uint16_t *perm) {
    const uint32_t tid = threadIdx.x;
    if (tid < (uint32_t)SHADE_CLASSES) cnt[tid] = 0u;
    __syncthreads();
    const unsigned long long below = (1ull << lane_id()) - 1ull;
    uint32_t rank = 0u;
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)SHADE_CLASSES; ++k) {
        const unsigned long long m = __ballot(cls == k);
        uint32_t w = 0u;
        if (m && lane_id() == 0) w = atomicAdd(&cnt[k], (uint32_t)__popcll(m));
        w = __shfl(w, 0);
        if (cls == k) rank = w + (uint32_t)__popcll(m & below);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t run = 0u;
        for (int k = 0; k < SHADE_CLASSES; ++k) { const uint32_t c = cnt[k]; cnt[k] = run; run += c; }
    }
    __syncthreads();
    perm[cnt[cls] + rank] = (uint16_t)tid;
    __syncthreads();
    return perm[tid];
}

// ENV: the scene has an environment emitter (the variant without it keeps
// the environment code, and its registers, out of the common case)
// SMP: the render's sampler (MTSG_SAMPLER_*)
// MATS: the material classes compiled in (MAT_*; the scene's set or a superset)
// FIRST: 1 = bounce 0 only (camera rays: differentials, the EWA environment
// lookup of a primary miss, hideEmitters' camera case), 0 = later bounces only
// (that code compiled out: C5's kernel then holds 96 VGPRs without spilling),
// 2 = either (run-time)
template <bool ENV, int SMP, bool EXT, int MATS = MATS_ALL, int FIRST = 2>
__global__ void SHADE_ATTR(ENV, MATS) k_shade(DevScene S, DevIntegrator I, DevBatch B, DevPaths P, int bounce, int qin,
                                                 uint32_t nIdentity, int hasAlpha) {
    __shared__ BlockAppend ba;
    __shared__ ShadeStage stage;
    constexpr bool SORT = shade_sorted<ENV, MATS>();
    __shared__ uint32_t s_classCnt[SHADE_CLASSES];
    __shared__ uint16_t s_perm[SORT ? SHADE_BLOCK : 1];
#if MTSG_SHADE_LDS_PAD
    // measurement: unused LDS that caps the workgroups per CU
    __shared__ uint32_t s_shadePad[MTSG_SHADE_LDS_PAD / 4];
    if (threadIdx.x == 0) ((volatile uint32_t *)s_shadePad)[(S.n_tri & 0xFFFFu) % (MTSG_SHADE_LDS_PAD / 4)] = 0u;
#endif
#if MTSG_SHADE_LDS
    __shared__ mtsg_bsdf s_bsdfs[SHADE_LDS_BSDFS];
    __shared__ mtsg_emitter s_emitters[SHADE_LDS_EMITTERS];
    __shared__ float s_ecdf[SHADE_LDS_EMITTERS + 1];
    ShadeTables tb = global_tables(S);
    const uint32_t nb = S.n_bsdfs, ne = S.n_emitters;
    if (nb <= (uint32_t)SHADE_LDS_BSDFS && ne <= (uint32_t)SHADE_LDS_EMITTERS) {
        for (uint32_t w = threadIdx.x; w < nb * (uint32_t)(sizeof(mtsg_bsdf) / 4); w += blockDim.x)
            ((uint32_t *)s_bsdfs)[w] = ((const uint32_t *)S.bsdfs)[w];
        for (uint32_t w = threadIdx.x; w < ne * (uint32_t)(sizeof(mtsg_emitter) / 4); w += blockDim.x)
            ((uint32_t *)s_emitters)[w] = ((const uint32_t *)S.emitters)[w];
        for (uint32_t w = threadIdx.x; w <= ne; w += blockDim.x) s_ecdf[w] = S.emitter_cdf[w];
        __syncthreads();
        tb = ShadeTables{s_bsdfs, s_emitters, s_ecdf};
    }
#else
    const ShadeTables tb = global_tables(S);
#endif
    uint32_t count = nIdentity;
    if (qin >= 0) count = __atomic_load_n(&P.cnt[cnt_q(qin)], __ATOMIC_RELAXED);
    const uint32_t nIter = (count + gridDim.x * blockDim.x - 1) / (gridDim.x * blockDim.x);
    const int qout = qin < 0 ? 1 : (qin ^ 1);
    const bool first = FIRST == 2 ? bounce == 0 : FIRST == 1;
    for (uint32_t it = 0; it < nIter; ++it) {
        const uint32_t i0 = (it * gridDim.x + blockIdx.x) * blockDim.x;
        uint32_t i = i0 + threadIdx.x;
        if constexpr (SORT)
            i = i0 + shade_sort(i < count ? shade_class(S, B, P, i, first, tb) : 0u, s_classCnt, s_perm);
        bool alive = i < count;
        bool cont = false, shadow = false;
        uint4 meta = make_uint4(0u, 0u, 0u, 0u);
        PathLoads pl;
        if (alive) {
            meta = first ? camera_meta(B, i) : ldS(&P.meta[i]);
#if MTSG_SHADE_PRELOAD == 1
            pl = load_path(S, P, i, first);
#elif MTSG_SHADE_PRELOAD == 2
            pl.h = ldS(&P.hit[i]);
#endif
            if (meta.x == 0u) alive = false;   // dead slot (bounce 0)
        }
        if (alive) {
#if MTSG_SHADE_PRELOAD == 0
            pl = load_path(S, P, i, first);
#elif MTSG_SHADE_PRELOAD == 2
            {
                const float4 h = pl.h;
                pl = load_path_rest(S, P, i, first);
                pl.h = h;
            }
#endif
            StageOut out{stage};
            shade_path<ENV, SMP, EXT, StageOut, MATS>(S, I, B, P, first, i, meta, pl, hasAlpha, out, cont, shadow, tb);
        }
        const uint32_t slot = meta.z;
        // The output positions come from the workgroup-aggregated append; the
        // outgoing records wait for it in LDS (lane-private rows) rather than
        // in registers live across its barriers.
        const int tid = threadIdx.x;
        uint32_t is, ic;
#if MTSG_SORT_OCT
        const float4 nd = stage.d[tid];
        const uint32_t key = (nd.x < 0.f ? 1u : 0u) | (nd.y < 0.f ? 2u : 0u) | (nd.z < 0.f ? 4u : 0u);
        block_append2_oct(ba, &P.cnt[cnt_s(bounce & 1)], &P.cnt[cnt_q(qout)], shadow, cont, cont ? key : 0u, is, ic);
#else
        block_append2(ba, &P.cnt[cnt_s(bounce & 1)], &P.cnt[cnt_q(qout)], shadow, cont, is, ic);
#endif
        // survivor: compacted into the next bounce's arrays
        if (cont) stage_write_next(stage, P, tid, ic, slot);
        if (shadow) stage_write_shadow(stage, P, tid, is, cont ? ic : (0x80000000u | slot));
    }
}

// ---------------------------------------------------------------------------
// Tail kernel: the batch's remaining paths carried through ALL their
// remaining bounces in one persistent launch.  Once few paths are left, every
// per-bounce traversal launch is mostly tail (its slowest rays' dependent
// fetch chains, 0.1-0.4 ms whatever the launch size), so a launch per bounce
// costs a tail per bounce; here a lane owns one path from its current bounce
// to its end (shade -> NEE shadow ray -> continuation ray -> shade ...) and
// the tails of different bounces overlap.  The arithmetic and its order are
// those of the per-bounce kernels (shade_path, spec_iter, shadow_unoccluded
// in the same sequence per path), so the image is bit-identical wherever the
// switch happens.  Path state is updated in place at the path's position
// (only its lane touches it), the shadow ray of a path uses the shadow
// arrays at that same position.
// ---------------------------------------------------------------------------
struct FinishOut {
    const DevPaths &P;
    uint32_t i;
    float4 c;   // NEE contribution; sh_c is written once the path's fate is known
    DEV void shadow(float4 o, float4 d, float4 cc) { stS(&P.sh_o[i], o); stS(&P.sh_d[i], d); c = cc; }
    DEV void next(float4 o, float4 d, float4 aux) { stS(&P.ray_o[i], o); stS(&P.ray_d[i], d); stS(&P.aux[i], aux); }
    DEV void state(float4 T, float4 L, uint4 meta) { stS(&P.T[i], T); stS(&P.Lp[i], L); stS(&P.meta[i], meta); }
};
enum : uint32_t { FS_IDLE = 0, FS_SHADE = 1, FS_TRACE = 2 };
constexpr uint32_t FINISH_FETCH = 64;   // paths per wave draw (small pools: the launch is all tail)
#ifndef MTSG_FINISH_WAVES
#define MTSG_FINISH_WAVES 3   // waves/SIMD asked of the compiler (r04: 3 at 168 VGPRs, 64 B of spills; C5 finish 52 -> 47 ms)
#endif
// the material-specialised tail kernels (MATS != MATS_ALL, round 6) fit 128
// VGPRs: 4 waves/SIMD (the generic one holds 168 at 3)
#ifndef MTSG_FINISH_WAVES_MATS
#define MTSG_FINISH_WAVES_MATS 4
#endif
#ifndef MTSG_FINISH_MATS
#define MTSG_FINISH_MATS 1   // 0: the tail always runs the all-materials kernel (A/B)
#endif
// whether launch_finish_inst runs a material-specialised k_finish (independent
// sampler, flat scene, built-in BSDFs, a specialised material set)
inline bool finish_uses_mats(int smp, bool ext, bool inst, int mats) {
    return MTSG_FINISH_MATS && smp == MTSG_SAMPLER_INDEPENDENT && !ext && !inst && mats_kernel_set(mats) != MATS_ALL;
}
#if MTSG_FINISH_WAVES > 0
#define FINISH_ATTR(MATS) __launch_bounds__(TRACE_BLOCK) \
    __attribute__((amdgpu_waves_per_eu((MATS) == MATS_ALL ? MTSG_FINISH_WAVES : MTSG_FINISH_WAVES_MATS)))
#else
#define FINISH_ATTR(MATS) __launch_bounds__(TRACE_BLOCK)
#endif

// qin: work list of the paths at their current bounce (their hits are ready:
// the bounce's trace launch ran).  shadeMin: a wave shades once that many of
// its busy lanes wait for shading (or none is tracing).
// INST: the two-level traversal (and its exact tie retrace) is compiled only
// into the instantiations for instanced scenes, so the flat kernel carries
// neither its registers nor the retrace's scratch stack
template <bool ENV, int SMP, bool EXT, bool INST, int MATS = MATS_ALL>
__global__ void FINISH_ATTR(MATS) k_finish(DevScene S, DevIntegrator I, DevBatch B, DevPaths P, int qin, int hasAlpha, uint32_t shadeMin) {
    const SpecStack stk{};
    lds_top_init(S);
    const uint32_t n = __atomic_load_n(&P.cnt[cnt_q(qin)], __ATOMIC_RELAXED);
    Fetch F{&P.cnt[CNT_FETCH], n, blockIdx.x % XGROUPS, 0, max(1u, gridDim.x / XGROUPS * GUIDE_SPLIT), FINISH_FETCH};
    TraceCounts tc{0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t poolBase = 0, poolLeft = 0;   // wave-uniform
    bool exhausted = false;
    uint32_t state = FS_IDLE;
    bool pendingCont = false;   // tracing the NEE shadow ray of a path that continues
    uint32_t idx = 0;
    uint32_t inst = 0;          // two-level: the instance the lane is inside
    TopSave ts;                 // (MTSG_INST_REGSAVE: its top-level state)
    SpecRay r;
    // the continuation ray of path idx (written by shade_path); a ray that
    // misses the scene bounds gets its miss record and is shaded next
    auto startClosest = [&]() {
        const float4 ro = ldS(&P.ray_o[idx]), rd = ldS(&P.ray_d[idx]);
        if (INST) P.hitInst[idx] = 0xFFFFFFFFu;   // two-level: no instance until a hit in one
        if (spec_init(S, xyz(ro), xyz(rd), ro.w, rd.w, false, r)) {
            state = FS_TRACE;
        } else {
            stS(&P.hit[idx], miss_record());
            state = FS_SHADE;
        }
    };
    for (;;) {
        unsigned long long idle = __ballot(state == FS_IDLE);
        while (idle && !exhausted) {
            if (poolLeft == 0 && !F.next(FINISH_FETCH, poolBase, poolLeft)) {
                exhausted = true;
                break;
            }
            const uint32_t nIdle = (uint32_t)__popcll(idle);
            const uint32_t take = min(nIdle, poolLeft);
            const uint32_t rank = rank_below(idle);
            if (state == FS_IDLE && rank < take) {
                idx = poolBase + rank;
                state = FS_SHADE;
            }
            poolBase += take;
            poolLeft -= take;
            idle = __ballot(state == FS_IDLE);
            if (take == nIdle) break;
        }
        const unsigned long long shading = __ballot(state == FS_SHADE), tracing = __ballot(state == FS_TRACE);
        if (!(shading | tracing)) {
            if (exhausted) break;
            continue;
        }
        if (shading && (!tracing || (uint32_t)__popcll(shading) >= min(shadeMin, (uint32_t)__popcll(shading | tracing)))) {
            if (state == FS_SHADE) {
                const uint4 meta = ldS(&P.meta[idx]);
                FinishOut out{P, idx, make_float4(0.f, 0.f, 0.f, 0.f)};
                bool cont = false, shadow = false;
                shade_path<ENV, SMP, EXT, FinishOut, MATS>(S, I, B, P, false, idx, meta, load_path(S, P, idx, false), hasAlpha, out, cont, shadow,
                                          global_tables(S));
                state = FS_IDLE;
                if (shadow) {
                    out.c.w = __uint_as_float(cont ? idx : (0x80000000u | meta.z));
                    stS(&P.sh_c[idx], out.c);
                    float4 ro = ldS(&P.sh_o[idx]), rd = ldS(&P.sh_d[idx]);
                    if (spec_init(S, xyz(ro), xyz(rd), rd.w, ro.w, true, r)) {   // sh_o.w = maxt, sh_d.w = mint
                        state = FS_TRACE;
                        pendingCont = cont;
                    } else {
                        shadow_unoccluded(P, idx);
                        if (cont) startClosest();
                    }
                } else if (cont) {
                    startClosest();
                }
            }
        }
        bool done = false;
        if (state == FS_TRACE) {
            // two-level scenes: the per-lane level switch of k_trace_s<.., true>
            // (its save slots are sized for this grid too)
            if (INST) done = spec_iter_i<false>(S, r, tc, P, idx, trav_limits<false>(S), inst, ts);
            else done = spec_iter<false>(S, r, stk, tc, P.hit + idx, trav_limits<false>(S));
        }
        if (done) {
            if (MTSG_MAILBOX && (r.bits & (SB_TIE | SB_SHADOW)) == SB_TIE) {
                if (!INST) {
                    tie_retrace(S, r, stk, ldS(P.ray_o + idx), ldS(P.ray_d + idx), P.hit + idx, trav_limits<false>(S));
                } else {
                    bool herr = false;
                    tie_retrace_i(S, P, idx, herr);
                    if (herr) r.bits |= SB_ERR;
                }
            }
            if (r.bits & SB_ERR) atomicOr(&P.cnt[CNT_ERR], CNT_ERR_TRAVERSAL);
            if (r.bits & SB_SHADOW) {
                if (!(r.bits & SB_FOUND)) shadow_unoccluded(P, idx);
                state = FS_IDLE;
                if (pendingCont) startClosest();
            } else {
                if (!(r.bits & SB_FOUND)) stS(&P.hit[idx], miss_record());
                state = FS_SHADE;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// film splat: one workgroup per 16x16 tile, LDS accumulation of the
// discretized reconstruction filter (imageblock.h:124-204), then one float
// atomic per texel into the tile+border block in HBM.
// ---------------------------------------------------------------------------
constexpr int MAX_BORDER = 4;
constexpr int LT = TILE + 2 * MAX_BORDER;   // LDS tile edge
#ifndef MTSG_SPLAT_CHUNK
#define MTSG_SPLAT_CHUNK 64   // r04: 16 -> 64 samples per workgroup, a quarter of the film atomics: C3 splat 2.86 -> 2.34 ms
#endif
constexpr int SPLAT_CHUNK = MTSG_SPLAT_CHUNK;   // samples per pixel per workgroup
#ifndef MTSG_SPLAT_LDS_FILTER
#define MTSG_SPLAT_LDS_FILTER 1   // 0: the filter table read from the kernel arguments (round-5 splat)
#endif

// One workgroup = one 16x16 tile x one chunk of SPLAT_CHUNK samples per pixel.
// Each thread owns one pixel: all its samples fall in [x, x+1) x [y, y+1), so
// their filter footprints lie in the K x K window centred on the pixel
// (K = 2 * border + 1).  The thread accumulates that window in registers
// (weights of texels outside a sample's [ceil, floor] range are exactly 0,
// as evalDiscretized returns m_values[31] = 0 there), then the workgroup
// reduces the windows into an LDS tile in K*K conflict-free phases (each
// phase shifts every window by the same offset, so no two threads touch the
// same texel: no atomics, fixed order) and flushes the tile with one float
// atomic per texel and channel into the HBM ImageBlock.
// winSz > 0: film holds one winSz x winSz window (the tile and its border) per tile of
// the call, window v = virtual tile v (mtsg_render_device_tiles)
template <int K, int CH>
__global__ void __launch_bounds__(BLOCK) k_splat(DevCamera C, DevIntegrator I, DevBatch B, DevPaths P, float *film, int blockW, int blockH,
                                                 int winSz) {
    __shared__ float acc[CH][LT * LT];
    constexpr int R = K / 2;
    for (int k = threadIdx.x; k < CH * LT * LT; k += BLOCK) (&acc[0][0])[k] = 0.0f;
#if MTSG_SPLAT_LDS_FILTER
    // the discretized filter's 32 values in LDS: the 2K per-sample lookups
    // are lane-indexed, so from the kernel arguments each was a vector load
    __shared__ float flt[32];
    if (threadIdx.x < 32) flt[threadIdx.x] = C.filter_values[threadIdx.x];
    __syncthreads();
#else
    const float *flt = C.filter_values;
#endif
    const int tl = blockIdx.x;
    int tx, ty;
    tile_of_key(batch_key(B, B.tile0 + tl), B.tiles_x, tx, ty, B.skew);
    const int x0 = B.rect_x + tx * TILE, y0 = B.rect_y + ty * TILE;   // tile origin (film coords)
    const int bord = C.border;
    const int pix = threadIdx.x;
    int lx, ly;
    tile_pix((uint32_t)pix, lx, ly);
    const int x = x0 + lx, y = y0 + ly;
    const bool inside = x < B.rect_x + B.rect_w && y < B.rect_y + B.rect_h;
    // block (tile rect + border) bounds relative to the window origin (x - R, y - R)
    const int bx0 = (B.rect_x - bord) - (x - R), by0 = (B.rect_y - bord) - (y - R);
    // Mitsuba computes a sample's filter offsets relative to the origin of the
    // 32x32 render block that holds its pixel (ImageBlock::put,
    // imageblock.h:158-160; blocks of BlockedImageProcess, imageproc.cpp:28-78,
    // scene.cpp:27), and `pos - 0.5 - origin` can round when it crosses a power
    // of two: the same origin is used here so the weights are bit-identical
    const int mbx = B.rect_x + ((x - B.rect_x) & ~31) - bord, mby = B.rect_y + ((y - B.rect_y) & ~31) - bord;
    const int wxo = (x - R) - mbx, wyo = (y - R) - mby;   // window origin in that block
    float win[K][K][CH];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
            for (int h = 0; h < CH; ++h) win[r][c][h] = 0.0f;
    const uint32_t sBeg = blockIdx.y * SPLAT_CHUNK, sEnd = min(B.ns, sBeg + SPLAT_CHUNK);
    if (inside) {
        for (uint32_t sl = sBeg; sl < sEnd; ++sl) {
            const uint32_t slot = ((uint32_t)tl * B.ns + sl) * (TILE * TILE) + pix;
            const float4 L = ldS(&P.L[slot]);
            float ja, jb;
            camera_jitter(I, x, y, B.s0 + sl, ja, jb);
            // invalid samples are rejected (imageblock.h:147-151)
            if (!(isfinite(L.x) && isfinite(L.y) && isfinite(L.z) && L.x >= 0 && L.y >= 0 && L.z >= 0)) continue;
            // sample position relative to the Mitsuba block origin
            // (imageblock.h:158-160)
            const float px = ((float)x + ja) - 0.5f - (float)mbx;
            const float py = ((float)y + jb) - 0.5f - (float)mby;
            float wx[K], wy[K];
#pragma unroll
            for (int c = 0; c < K; ++c) {
                const bool okx = c >= bx0 && c < bx0 + blockW;
                const bool oky = c >= by0 && c < by0 + blockH;
                wx[c] = okx ? flt[min((int)fabsf(((float)(wxo + c) - px) * C.filter_scale), 31)] : 0.0f;
                wy[c] = oky ? flt[min((int)fabsf(((float)(wyo + c) - py) * C.filter_scale), 31)] : 0.0f;
            }
            const float v[5] = {L.x, L.y, L.z, L.w, 1.0f};
            {
                // the K*K*CH window update is the kernel's VALU bound: one FMA
                // per term instead of a multiply and an add (the film sums
                // differ from the oracle's by rounding only; the weights and
                // their lookup above stay uncontracted, so no sample moves)
#pragma clang fp contract(fast)
#pragma unroll
                for (int r = 0; r < K; ++r)
#pragma unroll
                    for (int c = 0; c < K; ++c) {
                        const float w = wx[c] * wy[r];
#pragma unroll
                        for (int h = 0; h < CH; ++h) win[r][c][h] += w * v[CH == 5 ? h : (h == 3 ? 4 : h)];
                    }
            }
        }
    }
    __syncthreads();
    // K*K shifted phases: texel (ly + r + MAX_BORDER - R, lx + c + MAX_BORDER - R)
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
        for (int c = 0; c < K; ++c) {
            const int o = (ly + r + MAX_BORDER - R) * LT + (lx + c + MAX_BORDER - R);
#pragma unroll
            for (int h = 0; h < CH; ++h) acc[h][o] += win[r][c][h];
            __syncthreads();
        }
    // flush into the HBM block (blockW x blockH x 5, origin = rect - border):
    // one float per lane, so the lanes of a wave add to consecutive floats of
    // a texel row (4-5 64-B atomic requests per wave instruction, where one
    // texel per lane with its 5 channels strided 20 B apart touched ~20)
    for (int j = threadIdx.x; j < LT * LT * 5; j += BLOCK) {
        const int k = j / 5, h = j - 5 * k;
        const int ty2 = k / LT, tx2 = k % LT;
        const int fx = x0 - MAX_BORDER + tx2 - (B.rect_x - bord), fy = y0 - MAX_BORDER + ty2 - (B.rect_y - bord);
        if (fx < 0 || fy < 0 || fx >= blockW || fy >= blockH) continue;
        const float w = acc[CH - 1][k];
        if (w == 0.0f) continue;
        // window texel (the filter's support ends at the border: outside it w == 0)
        const int wx = tx2 - (MAX_BORDER - bord), wy = ty2 - (MAX_BORDER - bord);
        if (winSz && (wx < 0 || wy < 0 || wx >= winSz || wy >= winSz)) continue;
        float *dst = winSz ? film + (((size_t)(B.tile0 + tl) * winSz + wy) * winSz + wx) * 5 : film + ((size_t)fy * blockW + fx) * 5;
        // no alpha channel (CH == 4): alpha == 1 per sample, so its sum is the weight
        const float v = h < 3 ? acc[h][k] : (h == 3 && CH == 5 ? acc[CH == 5 ? 3 : 0][k] : w);
        unsafeAtomicAdd(dst + h, v);
    }
}

// zero the counters bounce b appends to (next-bounce paths qout, shadow rays
// S(sOut); sOut < 0: none) and the work-fetch counters of its trace launch
__global__ void k_reset(uint32_t *cnt, int qout, int sOut) {
    if (threadIdx.x == 0) {
        if (qout >= 0) cnt[qout ? CNT_Q1 : CNT_Q0] = 0;
        if (sOut >= 0) cnt[sOut ? CNT_S1 : CNT_S0] = 0;
    }
    if (threadIdx.x < XGROUPS) cnt[CNT_FETCH + 32 * threadIdx.x] = 0;
    if (threadIdx.x == 32) cnt[CNT_TIE] = 0;
}

// the closest rays of the trace launch before it that met an exact tie,
// traced again with the mailbox (tie_retrace); its grid strides over them
template <bool KNOBS>
__global__ void __launch_bounds__(TRACE_BLOCK) k_tie(DevScene S, DevPaths P) {
    const uint32_t n = __atomic_load_n(&P.cnt[CNT_TIE], __ATOMIC_RELAXED);
    // (most launches flag no tie: a workgroup with no entry leaves before it
    // stages the tree's top in LDS; the exit is uniform over the workgroup)
    if (blockIdx.x * TRACE_BLOCK >= n) return;
    const SpecStack stk{};
    lds_top_init(S);
    const TravLimits L = trav_limits<KNOBS>(S);
    SpecRay r;
    for (uint32_t i = blockIdx.x * TRACE_BLOCK + threadIdx.x; i < n; i += gridDim.x * TRACE_BLOCK) {
        const uint32_t idx = P.tie[i];
        float4 ro, rd;
        load_closest_ray(S, P, idx, P.camEnc != 0, ro, rd);
        tie_retrace(S, r, stk, ro, rd, P.hit + idx, L);
        if (r.bits & SB_ERR) atomicOr(&P.cnt[CNT_ERR], CNT_ERR_TRAVERSAL);
    }
}

// the same for two-level scenes: the exact two-level Havran (tie_retrace_i)
__global__ void __launch_bounds__(TRACE_BLOCK) k_tie_i(DevScene S, DevPaths P) {
    const uint32_t n = __atomic_load_n(&P.cnt[CNT_TIE], __ATOMIC_RELAXED);
    if (blockIdx.x * TRACE_BLOCK >= n) return;
    for (uint32_t i = blockIdx.x * TRACE_BLOCK + threadIdx.x; i < n; i += gridDim.x * TRACE_BLOCK) {
        bool err = false;
        tie_retrace_i(S, P, P.tie[i], err);
        if (err) atomicOr(&P.cnt[CNT_ERR], CNT_ERR_TRAVERSAL);
    }
}

}  // namespace
