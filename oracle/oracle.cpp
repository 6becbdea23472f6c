// oracle.cpp -- TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// Scalar CPU restatement of the reference's `path` hot path, written to follow
// the reference's own control flow line by line (AoS records, virtual-free
// switch dispatch, Havran kd-tree traversal), so that the HIP wavefront
// implementation can be checked against it.  Every function cites the
// reference file:line it restates (paths relative to the reference root).
#include "oracle.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;
int g_debug = 0;   // oracle_debug_pixel_sample(): print the path to stderr
std::vector<float> *g_rayLog = nullptr;   // closest-hit rays of the debugged path
#define DBG(...) do { if (g_debug) fprintf(stderr, __VA_ARGS__); } while (0)

// ---------------------------------------------------------------------------
// math (include/mitsuba/core/vector.h, frame.h)
// ---------------------------------------------------------------------------
struct Vec {
    float x, y, z;
    Vec() : x(0), y(0), z(0) {}
    Vec(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit Vec(float a) : x(a), y(a), z(a) {}
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
inline Vec operator+(Vec a, Vec b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline Vec operator-(Vec a, Vec b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline Vec operator-(Vec a) { return {-a.x, -a.y, -a.z}; }
inline Vec operator*(Vec a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline Vec operator*(float s, Vec a) { return {a.x * s, a.y * s, a.z * s}; }
inline Vec operator/(Vec a, float s) { float r = 1.0f / s; return {a.x * r, a.y * r, a.z * r}; }
inline float dot(Vec a, Vec b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float absDot(Vec a, Vec b) { return std::abs(dot(a, b)); }
inline Vec cross(Vec a, Vec b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float length(Vec a) { return std::sqrt(dot(a, a)); }
inline Vec normalize(Vec a) { return a / length(a); }

// RGB Spectrum (SPECTRUM_SAMPLES = 3)
struct Spec {
    float s[3];
    Spec() { s[0] = s[1] = s[2] = 0; }
    explicit Spec(float v) { s[0] = s[1] = s[2] = v; }
    Spec(float a, float b, float c) { s[0] = a; s[1] = b; s[2] = c; }
    static Spec of(const float *p) { return Spec(p[0], p[1], p[2]); }
    bool isZero() const { return s[0] == 0 && s[1] == 0 && s[2] == 0; }
    float max() const { return std::max(s[0], std::max(s[1], s[2])); }
    float luminance() const { return s[0] * 0.212671f + s[1] * 0.715160f + s[2] * 0.072169f; }   // spectrum.h (RGB)
};
inline Spec operator*(Spec a, Spec b) { return {a.s[0] * b.s[0], a.s[1] * b.s[1], a.s[2] * b.s[2]}; }
inline Spec operator*(Spec a, float f) { return {a.s[0] * f, a.s[1] * f, a.s[2] * f}; }
inline Spec operator/(Spec a, float f) { float r = 1.0f / f; return {a.s[0] * r, a.s[1] * r, a.s[2] * r}; }
inline Spec operator+(Spec a, Spec b) { return {a.s[0] + b.s[0], a.s[1] + b.s[1], a.s[2] + b.s[2]}; }
inline Spec operator-(Spec a, Spec b) { return {a.s[0] - b.s[0], a.s[1] - b.s[1], a.s[2] - b.s[2]}; }
inline Spec operator/(Spec a, Spec b) { return {a.s[0] / b.s[0], a.s[1] / b.s[1], a.s[2] / b.s[2]}; }
inline Spec &operator+=(Spec &a, Spec b) { a = a + b; return a; }
inline Spec &operator*=(Spec &a, Spec b) { a = a * b; return a; }
inline Spec sqrtSafe(Spec a) { return {std::sqrt(std::max(0.f, a.s[0])), std::sqrt(std::max(0.f, a.s[1])), std::sqrt(std::max(0.f, a.s[2]))}; }

// util.cpp:590-600
void coordinateSystem(const Vec &a, Vec &b, Vec &c) {
    if (std::abs(a.x) > std::abs(a.y)) {
        float invLen = 1.0f / std::sqrt(a.x * a.x + a.z * a.z);
        c = Vec(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / std::sqrt(a.y * a.y + a.z * a.z);
        c = Vec(0.0f, a.z * invLen, -a.y * invLen);
    }
    b = cross(c, a);
}

struct Frame {
    Vec s, t, n;
    Frame() {}
    explicit Frame(const Vec &nn) : n(nn) { coordinateSystem(nn, s, t); }   // frame.h:55-57
    Vec toLocal(const Vec &v) const { return Vec(dot(v, s), dot(v, t), dot(v, n)); }
    Vec toWorld(const Vec &v) const { return s * v.x + t * v.y + n * v.z; }
};
inline float cosTheta(const Vec &v) { return v.z; }
inline float cosTheta2(const Vec &v) { return v.z * v.z; }
inline float sinTheta2(const Vec &v) { return 1.0f - v.z * v.z; }
inline float tanTheta(const Vec &v) {   // frame.h:122-127
    float temp = 1 - v.z * v.z;
    if (temp <= 0.0f) return 0.0f;
    return std::sqrt(temp) / v.z;
}

// util.cpp:603-608
void computeShadingFrame(const Vec &n, const Vec &dpdu, Frame &frame) {
    frame.n = n;
    frame.s = normalize(dpdu - frame.n * dot(frame.n, dpdu));
    frame.t = cross(frame.n, frame.s);
}

// math.h:184-199 (Linux x86_64 variant)
inline float fastexp(float v) { return (float)::exp((double)v); }
inline float fastlog(float v) { return (float)::log((double)v); }
inline float signum(float v) { return copysignf(1.0f, v); }
inline float safe_sqrt(float v) { return std::sqrt(std::max(0.0f, v)); }

// math.cpp:25-70
float erfinv(float x) {
    float w = -fastlog((1.0f - x) * (1.0f + x));
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
        w = std::sqrt(w) - 3.0f;
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
float erf(float x) {
    const float a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f;
    const float a4 = -1.453152027f, a5 = 1.061405429f, p = 0.3275911f;
    float sign = signum(x);
    x = std::abs(x);
    float t = 1.0f / (1.0f + p * x);
    float y = 1.0f - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * fastexp(-x * x);
    return sign * y;
}
// math.cpp:74-86
float hypot2(float a, float b) {
    float r;
    if (std::abs(a) > std::abs(b)) { r = b / a; r = std::abs(a) * std::sqrt(1.0f + r * r); }
    else if (b != 0.0f) { r = a / b; r = std::abs(b) * std::sqrt(1.0f + r * r); }
    else r = 0.0f;
    return r;
}

const float kEpsilon = 1e-4f;        // constants.h:28
const float kShadowEpsilon = 1e-3f;  // constants.h:29
const float kDeltaEpsilon = 1e-3f;   // constants.h:31
const float kInvPi = 0.31830988618379067154f;
const float kInvTwoPi = 0.15915494309189533577f;   // constants.h:65

// ---------------------------------------------------------------------------
// SFMT-19937 (src/libcore/random.cpp:66-81 parameters, :130-640)
// ---------------------------------------------------------------------------
const int MEXP = 19937, N128 = MEXP / 128 + 1, N32 = N128 * 4, N64 = N128 * 2;
const int POS1 = 122, SL1 = 18, SL2 = 1, SR1 = 11, SR2 = 1;
const uint32_t MSK[4] = {0xdfffffefU, 0xddfecb7fU, 0xbffaffffU, 0xbffffff6U};
const uint32_t PARITY[4] = {0x00000001U, 0x00000000U, 0x00000000U, 0x13c9e684U};

struct Sfmt {
    union {
        uint32_t u32[N32];
        uint64_t u64[N64];
    };
    int idx = -1;

    static void rshift128(uint32_t out[4], const uint32_t in[4], int shift) {
        uint64_t th = ((uint64_t)in[3] << 32) | in[2], tl = ((uint64_t)in[1] << 32) | in[0];
        uint64_t oh = th >> (shift * 8), ol = tl >> (shift * 8);
        ol |= th << (64 - shift * 8);
        out[0] = (uint32_t)ol; out[1] = (uint32_t)(ol >> 32); out[2] = (uint32_t)oh; out[3] = (uint32_t)(oh >> 32);
    }
    static void lshift128(uint32_t out[4], const uint32_t in[4], int shift) {
        uint64_t th = ((uint64_t)in[3] << 32) | in[2], tl = ((uint64_t)in[1] << 32) | in[0];
        uint64_t oh = th << (shift * 8), ol = tl << (shift * 8);
        oh |= tl >> (64 - shift * 8);
        out[0] = (uint32_t)ol; out[1] = (uint32_t)(ol >> 32); out[2] = (uint32_t)oh; out[3] = (uint32_t)(oh >> 32);
    }
    static void doRecursion(uint32_t r[4], const uint32_t a[4], const uint32_t b[4], const uint32_t c[4], const uint32_t d[4]) {
        uint32_t x[4], y[4];
        lshift128(x, a, SL2);
        rshift128(y, c, SR2);
        for (int k = 0; k < 4; ++k) r[k] = a[k] ^ x[k] ^ ((b[k] >> SR1) & MSK[k]) ^ y[k] ^ (d[k] << SL1);
    }
    void genRandAll() {   // random.cpp:353-392 (scalar branch)
        uint32_t *r1 = &u32[4 * (N128 - 2)], *r2 = &u32[4 * (N128 - 1)];
        int i;
        for (i = 0; i < N128 - POS1; ++i) {
            uint32_t out[4];
            doRecursion(out, &u32[4 * i], &u32[4 * (i + POS1)], r1, r2);
            memcpy(&u32[4 * i], out, 16);
            r1 = r2;
            r2 = &u32[4 * i];
        }
        for (; i < N128; ++i) {
            uint32_t out[4];
            doRecursion(out, &u32[4 * i], &u32[4 * (i + POS1 - N128)], r1, r2);
            memcpy(&u32[4 * i], out, 16);
            r1 = r2;
            r2 = &u32[4 * i];
        }
    }
    void periodCertification() {   // random.cpp:322-351
        int inner = 0;
        for (int i = 0; i < 4; ++i) inner ^= u32[i] & PARITY[i];
        for (int i = 16; i > 0; i >>= 1) inner ^= inner >> i;
        inner &= 1;
        if (inner == 1) return;
        for (int i = 0; i < 4; ++i) {
            uint32_t work = 1;
            for (int j = 0; j < 32; ++j) {
                if ((work & PARITY[i]) != 0) { u32[i] ^= work; return; }
                work = work << 1;
            }
        }
    }
    void initGenRand(uint64_t seed) {   // random.cpp:397-406
        u64[0] = seed;
        for (int i = 1; i < N64; ++i) u64[i] = 6364136223846793005ULL * (u64[i - 1] ^ (u64[i - 1] >> 62)) + (uint64_t)i;
        idx = N32;
        periodCertification();
    }
    static uint32_t func1(uint32_t x) { return (x ^ (x >> 27)) * (uint32_t)1664525UL; }
    static uint32_t func2(uint32_t x) { return (x ^ (x >> 27)) * (uint32_t)1566083941UL; }
    void initByArray(const uint32_t *key, int keyLength) {   // random.cpp:408-470
        int i, j, count;
        uint32_t r;
        const int size = N32, lag = 11, mid = (size - lag) / 2;
        memset(u32, 0x8b, sizeof(u32));
        count = keyLength + 1 > N32 ? keyLength + 1 : N32;
        r = func1(u32[0] ^ u32[mid] ^ u32[N32 - 1]);
        u32[mid] += r;
        r += keyLength;
        u32[mid + lag] += r;
        u32[0] = r;
        count--;
        for (i = 1, j = 0; (j < count) && (j < keyLength); j++) {
            r = func1(u32[i] ^ u32[(i + mid) % N32] ^ u32[(i + N32 - 1) % N32]);
            u32[(i + mid) % N32] += r;
            r += key[j] + i;
            u32[(i + mid + lag) % N32] += r;
            u32[i] = r;
            i = (i + 1) % N32;
        }
        for (; j < count; j++) {
            r = func1(u32[i] ^ u32[(i + mid) % N32] ^ u32[(i + N32 - 1) % N32]);
            u32[(i + mid) % N32] += r;
            r += i;
            u32[(i + mid + lag) % N32] += r;
            u32[i] = r;
            i = (i + 1) % N32;
        }
        for (j = 0; j < N32; j++) {
            r = func2(u32[i] + u32[(i + mid) % N32] + u32[(i + N32 - 1) % N32]);
            u32[(i + mid) % N32] ^= r;
            r -= i;
            u32[(i + mid + lag) % N32] ^= r;
            u32[i] = r;
            i = (i + 1) % N32;
        }
        idx = N32;
        periodCertification();
    }
    void seedFrom(Sfmt &parent) {   // random.cpp:528-546 Random::seed(Random*)
        uint64_t buf[N64];
        for (int i = 0; i < N64; ++i) buf[i] = parent.nextULong();
        initByArray(reinterpret_cast<const uint32_t *>(buf), N64 * 2);
    }
    uint64_t nextULong() {   // gen_rand64
        if (idx >= N32) { genRandAll(); idx = 0; }
        uint64_t r = u64[idx / 2];
        idx += 2;
        return r;
    }
    float nextFloat() {   // random.cpp:629-639
        union { uint32_t u; float f; } x;
        x.u = (uint32_t)(((nextULong() & 0xFFFFFFFFULL) >> 9) | 0x3f800000UL);
        return x.f - 1.0f;
    }
};

// ---------------------------------------------------------------------------
// counter-mode RNG (shared spec with the GPU; DESIGN.md "RNG")
// ---------------------------------------------------------------------------
inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ULL;
    x ^= x >> 27; x *= 0x94D049BB133111EBULL;
    x ^= x >> 31;
    return x;
}
inline uint64_t counterKey(uint32_t seed, uint64_t sampleId) {
    return mix64(sampleId * 0x9E3779B97F4A7C15ULL + (uint64_t)seed);
}
inline float counterFloat(uint64_t key, uint32_t dim) {
    uint32_t u = (uint32_t)(mix64(key + (uint64_t)(dim + 1) * 0xD1B54A32D192ED03ULL) >> 32);
    union { uint32_t u; float f; } x;
    x.u = (u >> 9) | 0x3f800000U;
    return x.f - 1.0f;
}

// ---------------------------------------------------------------------------
// Quasi-Monte Carlo samplers (src/samplers/halton.cpp, hammersley.cpp,
// ldsampler.cpp; src/libcore/qmc.cpp).  Tables come from the scene
// description (host/qmc.cpp); the arithmetic below restates qmc.cpp.
// ---------------------------------------------------------------------------
constexpr float kOneMinusEps = 0x1.fffffep-1f;   // ONE_MINUS_EPS_FLT (constants.h:56)

// RINV / SCRAMBLED_RINV (qmc.cpp:141-167) with a run-time base
float radicalInverseFast(uint32_t base, uint64_t index, const uint16_t *perm) {
#pragma clang fp contract(off)
    const float radical = 1.0f / (float)base;
    uint64_t value = 0;
    float factor = 1.0f;
    while (index) {
        const uint64_t next = index / base;
        const uint64_t digit = index - next * base;
        value = value * base + (perm ? perm[digit] : digit);
        factor *= radical;
        index = next;
    }
    float inverse;
    if (perm) inverse = factor * ((float)value + radical * (float)perm[0] / (1 - radical));
    else inverse = (float)value * factor;
    return std::min(inverse, kOneMinusEps);
}

// halton.cpp:195-209 / hammersley.cpp:165-179
uint64_t inverseScrambledRadicalInverse(uint32_t base, uint64_t inverse, uint64_t digits, const uint16_t *invPerm) {
    uint64_t index = 0;
    while (digits) {
        uint64_t digit = inverse % base;
        if (invPerm) digit = invPerm[digit];
        inverse /= base;
        index = index * base + digit;
        --digits;
    }
    return index;
}

// halton.cpp:211-234
void extendedGCD(int64_t a, int64_t b, int64_t &x, int64_t &y) {
    if (b == 0) { x = 1; y = 0; return; }
    int64_t d = a / b, x_, y_;
    extendedGCD(b, a % b, x_, y_);
    x = y_;
    y = x_ - d * y_;
}
uint64_t multiplicativeInverse(int64_t a, int64_t n) {
    int64_t x, y;
    extendedGCD(a, n, x, y);
    int64_t m = x % n;
    return (uint64_t)(m < 0 ? m + n : m);
}

// qmc.h:43-58, 82-87
float radicalInverse2Single(uint32_t n, uint32_t scramble) {
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ffu) << 8) | ((n & 0xff00ff00u) >> 8);
    n = ((n & 0x0f0f0f0fu) << 4) | ((n & 0xf0f0f0f0u) >> 4);
    n = ((n & 0x33333333u) << 2) | ((n & 0xccccccccu) >> 2);
    n = ((n & 0x55555555u) << 1) | ((n & 0xaaaaaaaau) >> 1);
    n = (n >> (32 - 24)) ^ (scramble & ~(0xFFFFFFFFu << 24));
    return (float)n / (float)(1u << 24);
}
float sobol2Single(uint32_t n, uint32_t scramble) {
    for (uint32_t v = 1u << 31; n != 0; n >>= 1, v ^= v >> 1)
        if (n & 1) scramble ^= v;
    return (float)scramble / (float)(1ull << 32);
}

// ldsampler in counter mode: the per-pixel random shuffle of each dimension's
// sample set (ldsampler.cpp:156,178 m_random->shuffle) as a keyed bijection
// of [0, 2^bits) (xor, odd multiply, xorshift rounds)
uint32_t ldShuffle(uint32_t s, uint32_t bits, uint64_t h) {
    if (bits == 0) return 0;
    const uint32_t mask = bits >= 32 ? 0xFFFFFFFFu : (1u << bits) - 1u;
    uint32_t x = s & mask;
    for (uint32_t r = 0; r < 3; ++r) {
        const uint64_t k = mix64(h + (uint64_t)(r + 1) * 0x9E3779B97F4A7C15ULL);
        x ^= (uint32_t)k & mask;
        x = (x * ((uint32_t)(k >> 32) | 1u)) & mask;
        x ^= x >> ((bits + 1) / 2);
    }
    return x;
}
constexpr uint32_t kLdSalt = 0x6C64736Du;   // "ldsm": pixel keys of the ldsampler
constexpr const char *kSobolDimError = "Lookup dimension exceeds the direction number table size! "
                                       "You may have to reduce the 'maxDepth' parameter of your integrator.";
constexpr const char *kDimError = "Lookup dimension exceeds the prime number table size! "
                                  "You may have to reduce the 'maxDepth' parameter of your integrator.";

// Per-render sampler constants (setFilmResolution with blocked = true, as
// Integrator::configureSampler does for a SamplingIntegrator, integrator.cpp:39-43)
struct Qmc {
    int type = MTSG_SAMPLER_INDEPENDENT;
    const uint32_t *primes = nullptr, *off = nullptr;
    const uint16_t *perm = nullptr;
    uint16_t inv[2][3] = {{0, 0, 0}, {0, 0, 0}};   // inverse permutations of bases 2 and 3
    // halton.cpp:240-271
    uint64_t stride = 1, multInv[2] = {0, 0};
    int primePow[2] = {1, 1}, primeExp[2] = {0, 0};
    // hammersley.cpp:181-200
    int res[2] = {1, 1};
    uint32_t logH = 0;
    float factor = 1.0f;
    int ldDim = 4;
    uint32_t ldBits = 0;
    // sobol.cpp:147-158 (bucketed): resolution = roundToPowerOfTwo(max crop side)
    const uint32_t *sobolM = nullptr;
    const uint64_t *vdc = nullptr, *vdcInv = nullptr;
    uint32_t logRes = 0;
    float sobolRes = 1.0f;
    uint64_t sobolScramble = 0;

    // sobolseq.h:43-58 sampleSingle
    float sobolSample(uint64_t index, uint32_t dim) const {
        uint32_t result = (uint32_t)sobolScramble;
        for (uint32_t i = dim * MTSG_SOBOL_COLUMNS; index; index >>= 1, ++i)
            if (index & 1) result ^= sobolM[i];
        return std::min(result * (1.0f / 4294967296.0f), kOneMinusEps);
    }
    // sobolseq.h:99-131 look_up (single precision)
    uint64_t sobolLookUp(uint32_t m, uint32_t frame, uint32_t px, uint32_t py) const {
        const uint32_t m2 = m << 1;
        uint64_t index = (uint64_t)frame << m2;
        uint64_t delta = 0;
        for (uint32_t c = 0; frame; frame >>= 1, ++c)
            if (frame & 1) delta ^= vdc[(size_t)(m - 1) * MTSG_SOBOL_COLUMNS + c];
        const uint64_t scramble = (sobolScramble & 0xFFFFFFFFull) >> (32 - m);
        uint64_t b = ((((uint64_t)px ^ scramble) << m) | ((uint64_t)py ^ scramble)) ^ delta;
        for (uint32_t c = 0; b; b >>= 1, ++c)
            if (b & 1) index ^= vdcInv[(size_t)(m - 1) * MTSG_SOBOL_COLUMNS + c];
        return index;
    }

    const uint16_t *permOf(uint32_t dim) const { return perm ? perm + off[dim] : nullptr; }

    Qmc(const mtsg_scene_desc &d, uint32_t spp) {
        type = d.sampler.type;
        ldDim = d.sampler.dimension;
        while ((1u << ldBits) < spp) ++ldBits;
        if (type == MTSG_SAMPLER_SOBOL) {
            sobolM = d.sobol_matrices;
            vdc = d.sobol_vdc;
            vdcInv = d.sobol_vdc_inv;
            sobolScramble = d.sobol_scramble;
            uint32_t r = 1;
            const uint32_t mx = (uint32_t)std::max(d.camera.crop_w, d.camera.crop_h);
            while (r < mx) r <<= 1;   // math::roundToPowerOfTwo
            sobolRes = (float)r;
            logRes = 0;
            while ((1u << (logRes + 1)) <= r) ++logRes;   // math::log2i
            if (logRes > d.sobol_vdc_inv_rows) throw std::runtime_error("sobol: film too large for the tables");
            return;
        }
        if (type != MTSG_SAMPLER_HALTON && type != MTSG_SAMPLER_HAMMERSLEY) return;
        primes = d.qmc_primes;
        off = d.qmc_perm_offset;
        perm = d.qmc_perm;
        if (perm)
            for (int b = 0; b < 2; ++b)
                for (uint32_t j = 0; j < primes[b]; ++j) inv[b][perm[off[b] + j]] = (uint16_t)j;
        const int cw = d.camera.crop_w, ch = d.camera.crop_h;
        const int crop[2] = {cw, ch};
        if (type == MTSG_SAMPLER_HALTON) {
            stride = 1;
            for (int i = 0; i < 2; ++i) {
                int prime = (int)primes[i], value = 1, e = 0;
                while (value < std::min(crop[i], 128)) { value *= prime; ++e; }
                primePow[i] = value;
                primeExp[i] = e;
                stride *= (uint64_t)value;
            }
            multInv[0] = multiplicativeInverse(primePow[1], primePow[0]);
            multInv[1] = multiplicativeInverse(primePow[0], primePow[1]);
        } else {
            for (int i = 0; i < 2; ++i) {
                uint32_t r = 1;
                while (r < (uint32_t)crop[i]) r <<= 1;   // math::roundToPowerOfTwo
                res[i] = (int)std::min<uint32_t>(128, r);
            }
            logH = 0;
            while ((1 << (logH + 1)) <= res[1]) ++logH;   // math::log2i
            factor = 1.0f / (float)((size_t)spp * (size_t)res[0] * (size_t)res[1]);
            stride = (uint64_t)res[1];
        }
    }

    // generate(pos): offset of the pixel's subsequence (halton.cpp:277-293,
    // hammersley.cpp:206-218)
    uint64_t pixelOffset(int x, int y, uint32_t spp) const {
        const int pp[2] = {x % 128, y % 128};
        if (type == MTSG_SAMPLER_HALTON) {
            if (stride <= 1) return 0;
            uint64_t o = 0;
            for (int i = 0; i < 2; ++i) {
                uint64_t v = inverseScrambledRadicalInverse(primes[i], (uint64_t)pp[i], (uint64_t)primeExp[i],
                                                            perm ? inv[i] : nullptr);
                o += v * (stride / (uint64_t)primePow[i]) * multInv[i];
            }
            return o % stride;
        }
        if (type == MTSG_SAMPLER_HAMMERSLEY)
            return (uint64_t)pp[0] * (uint64_t)res[1] * spp +
                   inverseScrambledRadicalInverse(2, (uint64_t)pp[1], logH, perm ? inv[0] : nullptr);
        return 0;
    }
};

struct Sampler {
    int mode;
    Sfmt *sfmt = nullptr;
    uint64_t key = 0;
    uint32_t dim = 0;             // dimensions consumed (next1D: 1, next2D: 2)
    uint32_t n2 = 0;              // next2D calls (ldsampler keeps 1D and 2D apart)
    const Qmc *q = nullptr;
    int px = 0, py = 0;
    uint32_t s = 0;
    uint64_t offset = 0, ldKey = 0;
    uint64_t sobolIndex = 0;      // m_sobolSampleIndex (sobol.cpp:204-216)

    // start sample s of pixel (x, y) (Sampler::generate + setSampleIndex)
    void begin(const Qmc *qmc, uint32_t seed, int film_w, uint32_t spp, int x, int y, uint32_t si) {
        q = qmc;
        px = x; py = y; s = si;
        dim = 0; n2 = 0;
        key = counterKey(seed, ((uint64_t)y * film_w + x) * spp + si);
        offset = q ? q->pixelOffset(x, y, spp) : 0;
        if (q && q->type == MTSG_SAMPLER_LDSAMPLER) ldKey = counterKey(seed ^ kLdSalt, (uint64_t)y * film_w + x);
        if (q && q->type == MTSG_SAMPLER_SOBOL)
            sobolIndex = (q->logRes > 1 && x >= 0) ? q->sobolLookUp(q->logRes, si, (uint32_t)x, (uint32_t)y) : (uint64_t)si;
    }
    int kind() const { return q ? q->type : MTSG_SAMPLER_INDEPENDENT; }
    float indep() { return mode == ORACLE_RNG_SFMT ? sfmt->nextFloat() : counterFloat(key, dim); }
    // nextFloat of halton.cpp:343-350 / hammersley.cpp:228-236
    float qmcFloat(uint64_t idx) {
        const uint32_t d = dim++;
        if (q->type == MTSG_SAMPLER_HAMMERSLEY) {
            if (d == 0) return (float)idx * q->factor;
            return radicalInverseFast(q->primes[d - 1], idx, q->permOf(d - 1));
        }
        return radicalInverseFast(q->primes[d], idx, q->permOf(d));
    }
    float next1D() {
        switch (kind()) {
            case MTSG_SAMPLER_HALTON:
            case MTSG_SAMPLER_HAMMERSLEY:
                if (dim >= MTSG_QMC_PRIMES) throw std::runtime_error(kDimError);
                return qmcFloat(offset + q->stride * s);
            case MTSG_SAMPLER_SOBOL:   // sobol.cpp:218-228 (no sample arrays: nothing to skip)
                if (dim >= MTSG_SOBOL_DIMS) throw std::runtime_error(kSobolDimError);
                return q->sobolSample(sobolIndex, dim++);
            case MTSG_SAMPLER_LDSAMPLER: {   // ldsampler.cpp:202-208
                const uint32_t n1 = dim - 2 * n2;
                if ((int)n1 < q->ldDim) {
                    const uint64_t h = mix64(ldKey + (uint64_t)(2 * n1 + 1) * 0xD1B54A32D192ED03ULL);
                    ++dim;
                    return radicalInverse2Single(ldShuffle(s, q->ldBits, h), (uint32_t)(h >> 32));
                }
                const float v = counterFloat(key, dim);
                ++dim;
                return v;
            }
            default: {
                const float v = indep();
                ++dim;
                return v;
            }
        }
    }
    void next2D(float &a, float &b) {
        switch (kind()) {
            case MTSG_SAMPLER_HALTON:
            case MTSG_SAMPLER_HAMMERSLEY: {   // halton.cpp:365-386, hammersley.cpp:258-283
                if (dim + 1 >= MTSG_QMC_PRIMES) throw std::runtime_error(kDimError);
                const uint64_t idx = offset + q->stride * s;
                if (dim == 0) {
                    const bool h = q->type == MTSG_SAMPLER_HALTON;
                    const float v1 = qmcFloat(idx), v2 = qmcFloat(idx);
                    a = v1 * (float)(h ? q->primePow[0] : q->res[0]) - (float)(px % 128);
                    b = v2 * (float)(h ? q->primePow[1] : q->res[1]) - (float)(py % 128);
                } else {
                    a = qmcFloat(idx);
                    b = qmcFloat(idx);
                }
                break;
            }
            case MTSG_SAMPLER_SOBOL: {   // sobol.cpp:230-250
                if (dim + 1 >= MTSG_SOBOL_DIMS) throw std::runtime_error(kSobolDimError);
                if (dim == 0 && sobolIndex != (uint64_t)s) {
                    a = q->sobolSample(sobolIndex, dim++) * q->sobolRes - (float)px;
                    b = q->sobolSample(sobolIndex, dim++) * q->sobolRes - (float)py;
                } else {
                    a = q->sobolSample(sobolIndex, dim++);
                    b = q->sobolSample(sobolIndex, dim++);
                }
                ++n2;
                break;
            }
            case MTSG_SAMPLER_LDSAMPLER: {   // ldsampler.cpp:210-216
                if ((int)n2 < q->ldDim) {
                    const uint64_t h = mix64(ldKey + (uint64_t)(2 * n2 + 2) * 0xD1B54A32D192ED03ULL);
                    const uint64_t sc = mix64(h ^ 0x5851F42D4C957F2DULL);
                    const uint32_t i = ldShuffle(s, q->ldBits, h);
                    a = radicalInverse2Single(i, (uint32_t)sc);
                    b = sobol2Single(i, (uint32_t)(sc >> 32));
                    dim += 2;
                } else {
                    a = counterFloat(key, dim++);
                    b = counterFloat(key, dim++);
                }
                ++n2;
                break;
            }
            default:   // independent.cpp:99-103
                a = next1D();
                b = next1D();
                ++n2;
        }
        if (kind() == MTSG_SAMPLER_HALTON || kind() == MTSG_SAMPLER_HAMMERSLEY) ++n2;
    }
};

// ---------------------------------------------------------------------------
// Ray (include/mitsuba/core/ray.h:45-143)
// ---------------------------------------------------------------------------
struct Ray {
    Vec o, d, dRcp;
    float mint, maxt;
    void setDirection(const Vec &dd) { d = dd; dRcp = Vec(1.0f / d.x, 1.0f / d.y, 1.0f / d.z); }
    Vec operator()(float t) const { return o + d * t; }
};

struct Counters {
    uint64_t nodes = 0, refs = 0, tests = 0, closest = 0, shadow = 0, inst = 0;
};

// ---------------------------------------------------------------------------
// TMIPMap lookups (include/mitsuba/render/mipmap.h:498-840) over a pyramid
// built by the host library (mtsg_mipmap + half-rounded RGB texels): the
// environment map and the bitmap textures
// ---------------------------------------------------------------------------
struct MipMap {
    const mtsg_mipmap &M;
    const float *texels;
    static int modulo(int a, int b) { int r = a % b; return r < 0 ? r + b : r; }   // math::modulo
    static float log2f_m(float v) {   // math.cpp:103-106
        const float invLn2 = 1.0f / std::log(2.0f);
        return (float)std::log((double)v) * invLn2;
    }
    // one boundary condition of evalTexel (mipmap.h:503-562); false: the
    // constant `c` (EZero / EOne) replaces the texel
    static bool wrap(int mode, int &x, int n, float &c) {
        if (x >= 0 && x < n) return true;
        switch (mode) {
            case MTSG_WRAP_REPEAT: x = modulo(x, n); return true;
            case MTSG_WRAP_CLAMP: x = std::min(std::max(x, 0), n - 1); return true;
            case MTSG_WRAP_MIRROR:
                x = modulo(x, 2 * n);
                if (x >= n) x = 2 * n - x - 1;
                return true;
            case MTSG_WRAP_ZERO: c = 0.0f; return false;
            default: c = 1.0f; return false;
        }
    }
    Spec texel(int level, int x, int y) const {
        const int w = M.level_w[level], h = M.level_h[level];
        float c;
        if (!wrap(M.wrap_u, x, w, c)) return Spec(c);
        if (!wrap(M.wrap_v, y, h, c)) return Spec(c);
        return Spec::of(texels + M.level_offset[level] + 3 * ((size_t)y * w + x));
    }
    Spec box(int level, float u, float v) const {   // mipmap.h:566-569
        return texel(level, (int)std::floor(u * M.level_w[level]), (int)std::floor(v * M.level_h[level]));
    }
    Spec bilinear(int level, float ux, float uy) const {   // mipmap.h:575-596
        if (!std::isfinite(ux) || !std::isfinite(uy)) return Spec(0.0f);
        if (level >= M.levels) return box(M.levels - 1, ux, uy);
        const float u = ux * M.level_w[level] - 0.5f, v = uy * M.level_h[level] - 0.5f;
        const int xPos = (int)std::floor(u), yPos = (int)std::floor(v);
        const float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
        return texel(level, xPos, yPos) * dx2 * dy2 + texel(level, xPos, yPos + 1) * dx2 * dy1 +
               texel(level, xPos + 1, yPos) * dx1 * dy2 + texel(level, xPos + 1, yPos + 1) * dx1 * dy1;
    }
    Spec ewa(int level, float ux, float uy, float A, float B, float C) const {   // mipmap.h:775-840
        if (!std::isfinite(A + B + C + ux + uy)) return Spec(0.0f);
        if (level >= M.levels) return box(M.levels - 1, ux, uy);
        const float u = ux * M.level_w[level] - 0.5f, v = uy * M.level_h[level] - 0.5f;
        const float rx = M.size_ratio_x[level], ry = M.size_ratio_y[level];
        A /= rx * rx;
        B /= rx * ry;
        C /= ry * ry;
        const float invDet = 1.0f / (-B * B + 4.0f * A * C), deltaU = 2.0f * std::sqrt(C * invDet),
                    deltaV = 2.0f * std::sqrt(A * invDet);
        const int u0 = (int)std::ceil(u - deltaU), u1 = (int)std::floor(u + deltaU);
        const int v0 = (int)std::ceil(v - deltaV), v1 = (int)std::floor(v + deltaV);
        const float As = A * MTSG_MIPMAP_LUT_SIZE, Bs = B * MTSG_MIPMAP_LUT_SIZE, Cs = C * MTSG_MIPMAP_LUT_SIZE;
        Spec result(0.0f);
        float denominator = 0.0f;
        const float ddq = 2 * As, uu0 = (float)u0 - u;
        for (int vt = v0; vt <= v1; ++vt) {
            const float vv = (float)vt - v;
            float q = As * uu0 * uu0 + (Bs * uu0 + Cs * vv) * vv;
            float dq = As * (2 * uu0 + 1) + Bs * vv;
            for (int ut = u0; ut <= u1; ++ut) {
                if (q < (float)MTSG_MIPMAP_LUT_SIZE) {
                    const uint32_t qi = (uint32_t)q;
                    if (qi < MTSG_MIPMAP_LUT_SIZE) {
                        const float weight = M.weight_lut[(int)q];
                        result += texel(level, ut, vt) * weight;
                        denominator += weight;
                    }
                }
                q += dq;
                dq += ddq;
            }
        }
        if (denominator == 0) return bilinear(level, ux, uy);
        return result / denominator;
    }
    // TMIPMap::eval(uv, d0, d1) (mipmap.h:633-722)
    Spec filtered(float ux, float uy, float d0x, float d0y, float d1x, float d1y) const {
        if (M.filter == MTSG_MIP_NEAREST) return box(0, ux, uy);
        if (M.filter == MTSG_MIP_BILINEAR) return bilinear(0, ux, uy);
        const float du0 = d0x * M.level_w[0], dv0 = d0y * M.level_h[0], du1 = d1x * M.level_w[0], dv1 = d1y * M.level_h[0];
        float A = dv0 * dv0 + dv1 * dv1, B = -2.0f * (du0 * dv0 + du1 * dv1), C = du0 * du0 + du1 * du1,
              F = A * C - B * B * 0.25f;
        const float root = hypot2(A - C, B), Aprime = 0.5f * (A + C - root), Cprime = 0.5f * (A + C + root);
        float majorRadius = Aprime != 0 ? std::sqrt(F / Aprime) : 0, minorRadius = Cprime != 0 ? std::sqrt(F / Cprime) : 0;
        if (M.filter == MTSG_MIP_TRILINEAR || !(minorRadius > 0) || !(majorRadius > 0) || F < 0) {
            const float level = log2f_m(std::max(majorRadius, kEpsilon));
            const int ilevel = (int)std::floor(level);
            if (ilevel < 0) return bilinear(0, ux, uy);
            const float a = level - ilevel;
            return bilinear(ilevel, ux, uy) * (1.0f - a) + bilinear(ilevel + 1, ux, uy) * a;
        }
        if (minorRadius * M.max_anisotropy < majorRadius) {
            minorRadius = majorRadius / M.max_anisotropy;
            const float theta = 0.5f * std::atan(B / (A - C));
            const float sinTheta = std::sin(theta), cosTheta = std::cos(theta);
            const float a2 = majorRadius * majorRadius, b2 = minorRadius * minorRadius, sinTheta2 = sinTheta * sinTheta,
                        cosTheta2 = cosTheta * cosTheta, sin2Theta = 2 * sinTheta * cosTheta;
            A = a2 * cosTheta2 + b2 * sinTheta2;
            B = (a2 - b2) * sin2Theta;
            C = a2 * sinTheta2 + b2 * cosTheta2;
            F = a2 * b2;
        }
        const float scale = 1.0f / F;
        A *= scale; B *= scale; C *= scale;
        const float level = std::max(0.0f, log2f_m(minorRadius));
        const int ilevel = (int)level;
        const float a = level - ilevel;
        if (majorRadius < 1 || !(A > 0 && C > 0)) return bilinear(ilevel, ux, uy);
        return ewa(ilevel, ux, uy, A, B, C) * (1.0f - a) + ewa(ilevel + 1, ux, uy, A, B, C) * a;
    }
    // BitmapTexture::eval(uv) (bitmap.cpp:431-454): no partials
    Spec unfiltered(float ux, float uy) const {
        return M.filter == MTSG_MIP_NEAREST ? box(0, ux, uy) : bilinear(0, ux, uy);
    }
};

// ---------------------------------------------------------------------------
// Scene view over the flat descriptor
// ---------------------------------------------------------------------------
struct Its {
    float t = std::numeric_limits<float>::infinity();
    Vec p;
    Frame geoFrame, shFrame;
    Vec dpdu, dpdv, wi;
    float u = 0, v = 0;              // its.uv
    int shape = -1;
    bool valid() const { return t != std::numeric_limits<float>::infinity(); }
    Vec toLocal(const Vec &v) const { return shFrame.toLocal(v); }
    Vec toWorld(const Vec &v) const { return shFrame.toWorld(v); }
};

// IntersectionCache (skdtree.h:236-241); for a hit inside an instance the
// group tree's cache, and the instance (Instance::rayIntersect passes its
// temp space down to the group's ShapeKDTree, instance.cpp:115-122)
struct Cache { uint32_t shapeIndex, primIndex; float u, v, rx, ry; uint32_t inst = 0xFFFFFFFFu; };

struct SceneView {
    const mtsg_scene_desc &d;
    explicit SceneView(const mtsg_scene_desc &dd) : d(dd) {}

    Vec vtx(uint32_t i) const { return Vec(d.vtx_pos[3 * i], d.vtx_pos[3 * i + 1], d.vtx_pos[3 * i + 2]); }
    Vec nrm(uint32_t i) const { return Vec(d.vtx_nrm[3 * i], d.vtx_nrm[3 * i + 1], d.vtx_nrm[3 * i + 2]); }

    // AABB::rayIntersect (aabb.h:308-338)
    bool aabbIntersect(const Ray &ray, float &nearT, float &farT) const {
        return aabbIntersect(ray, d.aabb_min, d.aabb_max, nearT, farT);
    }
    static bool aabbIntersect(const Ray &ray, const float *bmin, const float *bmax, float &nearT, float &farT) {
        nearT = -std::numeric_limits<float>::infinity();
        farT = std::numeric_limits<float>::infinity();
        for (int i = 0; i < 3; i++) {
            const float origin = ray.o[i], minVal = bmin[i], maxVal = bmax[i];
            if (ray.d[i] == 0) {
                if (origin < minVal || origin > maxVal) return false;
            } else {
                float t1 = (minVal - origin) * ray.dRcp[i];
                float t2 = (maxVal - origin) * ray.dRcp[i];
                if (t1 > t2) std::swap(t1, t2);
                nearT = std::max(t1, nearT);
                farT = std::min(t2, farT);
                if (!(nearT <= farT)) return false;
            }
        }
        return true;
    }

    // TriAccel::rayIntersect (triaccel.h:96-158)
    static bool triIntersect(const mtsg_triaccel &ta, const Ray &ray, float mint, float maxt, float &u, float &v, float &t) {
        float o_u, o_v, o_k, d_u, d_v, d_k;
        switch (ta.k) {
            case 0: o_u = ray.o.y; o_v = ray.o.z; o_k = ray.o.x; d_u = ray.d.y; d_v = ray.d.z; d_k = ray.d.x; break;
            case 1: o_u = ray.o.z; o_v = ray.o.x; o_k = ray.o.y; d_u = ray.d.z; d_v = ray.d.x; d_k = ray.d.y; break;
            case 2: o_u = ray.o.x; o_v = ray.o.y; o_k = ray.o.z; d_u = ray.d.x; d_v = ray.d.y; d_k = ray.d.z; break;
            default: return false;
        }
        t = (ta.n_d - o_u * ta.n_u - o_v * ta.n_v - o_k) / (d_u * ta.n_u + d_v * ta.n_v + d_k);
        if (t < mint || t > maxt) return false;
        const float hu = o_u + t * d_u - ta.a_u;
        const float hv = o_v + t * d_v - ta.a_v;
        u = hv * ta.b_nu + hu * ta.b_nv;
        v = hu * ta.c_nu + hv * ta.c_nv;
        return u >= 0 && v >= 0 && u + v <= 1.0f;
    }

    // Rectangle::rayIntersect (rectangle.cpp:115-139): object-space plane test
    bool rectIntersect(const mtsg_rect &r, const Ray &wr, float mint, float maxt, float &t, float &lx, float &ly) const {
        const float *m = r.to_object;
        Vec o(m[0] * wr.o.x + m[1] * wr.o.y + m[2] * wr.o.z + m[3],
              m[4] * wr.o.x + m[5] * wr.o.y + m[6] * wr.o.z + m[7],
              m[8] * wr.o.x + m[9] * wr.o.y + m[10] * wr.o.z + m[11]);
        Vec dd(m[0] * wr.d.x + m[1] * wr.d.y + m[2] * wr.d.z,
               m[4] * wr.d.x + m[5] * wr.d.y + m[6] * wr.d.z,
               m[8] * wr.d.x + m[9] * wr.d.y + m[10] * wr.d.z);
        float hit = -o.z / dd.z;
        if (!(hit >= mint && hit <= maxt)) return false;
        Vec local = o + dd * hit;
        if (std::abs(local.x) <= 1 && std::abs(local.y) <= 1) {
            t = hit; lx = local.x; ly = local.y;
            return true;
        }
        return false;
    }

    // ShapeKDTree::intersect (skdtree.h:248-337)
    bool primIntersect(const Ray &ray, uint32_t idx, float mint, float maxt, float &t, Cache *cache,
                       Counters *ctr = nullptr) const {
        const mtsg_triaccel &ta = d.triaccel[idx];
        if (ta.k != MTSG_TRIACCEL_SHAPE) {
            float u, v, tt;
            if (triIntersect(ta, ray, mint, maxt, u, v, tt)) {
                t = tt;
                if (cache) { cache->shapeIndex = ta.shape_index; cache->primIndex = ta.prim_index; cache->u = u; cache->v = v; }
                return true;
            }
            return false;
        }
        if (d.shapes[ta.shape_index].type == MTSG_SHAPE_INSTANCE)
            return instanceIntersect<false>(ray, ta.prim_index, mint, maxt, t, cache, ctr);
        float tt, lx, ly;
        if (rectIntersect(d.rects[ta.prim_index], ray, mint, maxt, tt, lx, ly)) {
            t = tt;
            if (cache) { cache->shapeIndex = ta.shape_index; cache->primIndex = 0xFFFFFFFFu; cache->rx = lx; cache->ry = ly; }
            return true;
        }
        return false;
    }

    // ShapeKDTree::intersect(ray, idx, mint, maxt) (skdtree.h:310-337): shadow
    // rays; an instance runs Instance::rayIntersect(ray, mint, maxt)
    bool primIntersectShadow(const Ray &ray, uint32_t idx, float mint, float maxt, float &t, Counters *ctr) const {
        const mtsg_triaccel &ta = d.triaccel[idx];
        if (ta.k == MTSG_TRIACCEL_SHAPE && d.shapes[ta.shape_index].type == MTSG_SHAPE_INSTANCE)
            return instanceIntersect<true>(ray, ta.prim_index, mint, maxt, t, nullptr, ctr);
        return primIntersect(ray, idx, mint, maxt, t, nullptr);
    }

    // SAHKDTree3D::rayIntersectHavran (sahkdtree3.h:178-308), with the
    // 8-entry hashed mailbox (sahkdtree3.h:30-32,138-152)
    // Transform::operator()(Ray) (transform.h:262-278) with the instance's
    // inverse: o and d transformed, the reciprocal recomputed, mint / maxt kept
    Ray toInstance(const Ray &r, const mtsg_instance &in) const {
        const float *m = in.to_local;
        Ray l;
        l.o = Vec(m[0] * r.o.x + m[1] * r.o.y + m[2] * r.o.z + m[3], m[4] * r.o.x + m[5] * r.o.y + m[6] * r.o.z + m[7],
                  m[8] * r.o.x + m[9] * r.o.y + m[10] * r.o.z + m[11]);
        l.setDirection(Vec(m[0] * r.d.x + m[1] * r.d.y + m[2] * r.d.z, m[4] * r.d.x + m[5] * r.d.y + m[6] * r.d.z,
                           m[8] * r.d.x + m[9] * r.d.y + m[10] * r.d.z));
        l.mint = r.mint;
        l.maxt = r.maxt;
        return l;
    }
    // Instance::rayIntersect (instance.cpp:115-130) -> the group's
    // ShapeKDTree::rayIntersect(ray, mint, maxt, t, temp) (skdtree.h:431-458)
    template <bool shadowRay>
    bool instanceIntersect(const Ray &wr, uint32_t inst, float mint, float maxt, float &t, Cache *cache,
                           Counters *ctr) const {
        const mtsg_instance &in = d.instances[inst];
        const mtsg_group &G = d.groups[in.group];
        const Ray r = toInstance(wr, in);
        if (ctr) ctr->inst++;
        float nearT, farT;
        if (!aabbIntersect(r, G.aabb_min, G.aabb_max, nearT, farT)) return false;
        if (mint > nearT) nearT = mint;
        if (maxt < farT) farT = maxt;
        if (!(farT > nearT)) return false;
        const mtsg_kdnode *nodes = d.group_nodes + G.node_offset;
        const uint32_t *idx = d.group_indices + G.index_offset;
        float tt = std::numeric_limits<float>::infinity();
        Cache c;
        const bool hit = ctr ? havranTree<shadowRay, true>(nodes, idx, r, nearT, farT, tt, shadowRay ? nullptr : &c, ctr)
                             : havranTree<shadowRay, false>(nodes, idx, r, nearT, farT, tt, shadowRay ? nullptr : &c, nullptr);
        if (!hit) return false;
        t = tt;
        if (cache) { *cache = c; cache->inst = inst; }
        return true;
    }

    template <bool shadowRay, bool count>
    bool havran(const Ray &ray, float mint, float maxt, float &t, Cache *cache, Counters *ctr) const {
        return havranTree<shadowRay, count>(d.nodes, d.indices, ray, mint, maxt, t, cache, ctr);
    }

    template <bool shadowRay, bool count>
    bool havranTree(const mtsg_kdnode *nodes, const uint32_t *indices, const Ray &ray, float mint, float maxt, float &t,
                    Cache *cache, Counters *ctr) const {
        struct Entry { uint32_t node; float t; uint32_t prev; Vec p; };
        Entry stack[48];
        uint32_t mailbox[8];
        memset(mailbox, 0xFF, sizeof(mailbox));
        uint32_t enPt = 0;
        stack[enPt].t = mint;
        stack[enPt].p = ray(mint);
        uint32_t exPt = 1;
        stack[exPt].t = maxt;
        stack[exPt].p = ray(maxt);
        stack[exPt].node = 0xFFFFFFFFu;
        bool found = false;
        uint32_t cur = 0;
        Cache tmp;
        while (cur != 0xFFFFFFFFu) {
            for (;;) {
                if (count) ctr->nodes++;
                const mtsg_kdnode &node = nodes[cur];
                if (node.combined & 0x80000000u) break;
                float splitVal;
                memcpy(&splitVal, &node.data, 4);
                const int axis = (int)(node.combined & 3u);
                const uint32_t left = cur + ((node.combined & ~(3u | 0x40000000u)) >> 2);
                uint32_t farChild;
                if (stack[enPt].p[axis] <= splitVal) {
                    if (stack[exPt].p[axis] <= splitVal) { cur = left; continue; }
                    if (stack[enPt].p[axis] == splitVal) { cur = left + 1; continue; }
                    cur = left;
                    farChild = cur + 1;
                } else {
                    if (splitVal < stack[exPt].p[axis]) { cur = left + 1; continue; }
                    farChild = left;
                    cur = farChild + 1;
                }
                float distToSplit = (splitVal - ray.o[axis]) * ray.dRcp[axis];
                const uint32_t tmpPt = exPt++;
                if (exPt == enPt) ++exPt;
                if (exPt >= 48) { g_err = "kd-tree stack overflow"; return found; }
                stack[exPt].prev = tmpPt;
                stack[exPt].t = distToSplit;
                stack[exPt].node = farChild;
                stack[exPt].p = ray(distToSplit);
                stack[exPt].p[axis] = splitVal;
            }
            const mtsg_kdnode &leaf = nodes[cur];
            for (uint32_t entry = leaf.combined & 0x7FFFFFFFu, last = leaf.data; entry != last; entry++) {
                const uint32_t primIdx = indices[entry];
                if (count) ctr->refs++;
                if (mailbox[primIdx & 7] == primIdx) continue;
                if (count) ctr->tests++;
                bool result;
                if (!shadowRay) result = primIntersect(ray, primIdx, mint, maxt, t, &tmp, count ? ctr : nullptr);
                else { float tt; result = primIntersectShadow(ray, primIdx, mint, maxt, tt, count ? ctr : nullptr); }
                if (result) {
                    if (shadowRay) return true;
                    maxt = t;
                    found = true;
                    if (cache) *cache = tmp;
                }
                mailbox[primIdx & 7] = primIdx;
            }
            if (stack[exPt].t > maxt) break;
            enPt = exPt;
            cur = stack[exPt].node;
            exPt = stack[enPt].prev;
        }
        return found;
    }

    // ShapeKDTree::fillIntersectionRecord<BarycentricPos> (skdtree.h:343-428),
    // without the final computeShadingFrame / wi
    void fillShape(const Ray &ray, const Cache &c, Its &its, bool barycentricPos) const {
        its.shape = (int)c.shapeIndex;
        const mtsg_shape &sh = d.shapes[c.shapeIndex];
        if (c.primIndex != 0xFFFFFFFFu) {
            const uint32_t g = c.primIndex;
            const uint32_t i0 = d.tri_idx[3 * g], i1 = d.tri_idx[3 * g + 1], i2 = d.tri_idx[3 * g + 2];
            const float bx = 1 - c.u - c.v, by = c.u, bz = c.v;
            const Vec p0 = vtx(i0), p1 = vtx(i1), p2 = vtx(i2);
            its.p = barycentricPos ? p0 * bx + p1 * by + p2 * bz : ray(its.t);
            Vec side1 = p1 - p0, side2 = p2 - p0;
            Vec faceNormal = cross(side1, side2);
            float len = length(faceNormal);
            if (!(faceNormal.x == 0 && faceNormal.y == 0 && faceNormal.z == 0)) faceNormal = faceNormal / len;
            its.dpdu = Vec(d.tri_dpdu[3 * g], d.tri_dpdu[3 * g + 1], d.tri_dpdu[3 * g + 2]);
            // UV tangent dpdv or side2; uv interpolated from the vertices' texture
            // coordinates, Point2(b.y, b.z) without them (skdtree.h:373-405)
            its.dpdv = d.tri_dpdv ? Vec(d.tri_dpdv[3 * g], d.tri_dpdv[3 * g + 1], d.tri_dpdv[3 * g + 2]) : side2;
            if (d.tri_uv) {
                const float *t = d.tri_uv + 6 * (size_t)g;
                its.u = t[0] * bx + t[2] * by + t[4] * bz;
                its.v = t[1] * bx + t[3] * by + t[5] * bz;
            } else {
                its.u = by;
                its.v = bz;
            }
            if (!sh.face_normals) {
                const Vec n0 = nrm(i0), n1 = nrm(i1), n2 = nrm(i2);
                its.shFrame.n = normalize(n0 * bx + n1 * by + n2 * bz);
                if (dot(faceNormal, its.shFrame.n) < 0) faceNormal = -faceNormal;
            } else {
                its.shFrame.n = faceNormal;
            }
            its.geoFrame = Frame(faceNormal);
        } else {
            // Rectangle::fillIntersectionRecord (rectangle.cpp:145-158)
            const mtsg_rect &r = d.rects[sh.rect];
            its.geoFrame.s = Vec(r.frame_s[0], r.frame_s[1], r.frame_s[2]);
            its.geoFrame.t = Vec(r.frame_t[0], r.frame_t[1], r.frame_t[2]);
            its.geoFrame.n = Vec(r.frame_n[0], r.frame_n[1], r.frame_n[2]);
            its.shFrame.n = its.geoFrame.n;
            its.dpdu = Vec(r.dpdu[0], r.dpdu[1], r.dpdu[2]);
            its.dpdv = Vec(r.dpdv[0], r.dpdv[1], r.dpdv[2]);
            its.u = 0.5f * (c.rx + 1);
            its.v = 0.5f * (c.ry + 1);
            its.p = ray(its.t);
        }
    }

    // ShapeKDTree::fillIntersectionRecord<true> (skdtree.h:343-428)
    void fill(const Ray &ray, const Cache &c, Its &its) const {
        if (c.inst == 0xFFFFFFFFu) {
            fillShape(ray, c, its, true);
        } else {
            // Instance::fillIntersectionRecord (instance.cpp:146-160): the
            // group tree fills the record from the group-space ray
            // (BarycentricPos = false), then it is mapped back with toWorld;
            // normals by the inverse transpose (transform.h:203-211)
            const mtsg_instance &in = d.instances[c.inst];
            const Ray lr = toInstance(ray, in);
            fillShape(lr, c, its, false);
            const float *W = in.to_world, *L = in.to_local;
            auto normalT = [&](const Vec &v) {
                return Vec(L[0] * v.x + L[4] * v.y + L[8] * v.z, L[1] * v.x + L[5] * v.y + L[9] * v.z,
                           L[2] * v.x + L[6] * v.y + L[10] * v.z);
            };
            its.shFrame.n = normalize(normalT(its.shFrame.n));
            its.geoFrame = Frame(normalize(normalT(its.geoFrame.n)));
            its.dpdu = Vec(W[0] * its.dpdu.x + W[1] * its.dpdu.y + W[2] * its.dpdu.z,
                           W[4] * its.dpdu.x + W[5] * its.dpdu.y + W[6] * its.dpdu.z,
                           W[8] * its.dpdu.x + W[9] * its.dpdu.y + W[10] * its.dpdu.z);
            its.dpdv = Vec(W[0] * its.dpdv.x + W[1] * its.dpdv.y + W[2] * its.dpdv.z,
                           W[4] * its.dpdv.x + W[5] * its.dpdv.y + W[6] * its.dpdv.z,
                           W[8] * its.dpdv.x + W[9] * its.dpdv.y + W[10] * its.dpdv.z);
            its.p = Vec(W[0] * its.p.x + W[1] * its.p.y + W[2] * its.p.z + W[3],
                        W[4] * its.p.x + W[5] * its.p.y + W[6] * its.p.z + W[7],
                        W[8] * its.p.x + W[9] * its.p.y + W[10] * its.p.z + W[11]);
        }
        computeShadingFrame(its.shFrame.n, its.dpdu, its.shFrame);
        its.wi = its.toLocal(-ray.d);
    }

    // ShapeKDTree::rayIntersect (skdtree.cpp:112-142)
    template <bool count>
    bool rayIntersect(const Ray &ray, Its &its, Cache *outCache, Counters *ctr) const {
        if (g_rayLog) g_rayLog->insert(g_rayLog->end(), {ray.o.x, ray.o.y, ray.o.z, ray.d.x, ray.d.y, ray.d.z, ray.mint, ray.maxt});
        its.t = std::numeric_limits<float>::infinity();
        if (count) ctr->closest++;
        float mint, maxt;
        if (aabbIntersect(ray, mint, maxt)) {
            float rayMinT = ray.mint;
            if (rayMinT == kEpsilon)
                rayMinT *= std::max(std::max(std::max(std::abs(ray.o.x), std::abs(ray.o.y)), std::abs(ray.o.z)), kEpsilon);
            if (rayMinT > mint) mint = rayMinT;
            if (ray.maxt < maxt) maxt = ray.maxt;
            if (maxt > mint) {
                Cache c;
                float t = its.t;
                if (havran<false, count>(ray, mint, maxt, t, &c, ctr)) {
                    its.t = t;
                    fill(ray, c, its);
                    if (outCache) *outCache = c;
                    return true;
                }
            }
        }
        its.t = std::numeric_limits<float>::infinity();
        return false;
    }

    // ShapeKDTree::rayIntersect(const Ray&) shadow variant (skdtree.cpp:207-226)
    template <bool count>
    bool rayIntersectShadow(const Ray &ray, Counters *ctr) const {
        float mint, maxt, t = std::numeric_limits<float>::infinity();
        if (count) ctr->shadow++;
        if (aabbIntersect(ray, mint, maxt)) {
            float rayMinT = ray.mint;
            if (rayMinT == kEpsilon)
                rayMinT *= std::max(std::max(std::abs(ray.o.x), std::abs(ray.o.y)), std::abs(ray.o.z));
            if (rayMinT > mint) mint = rayMinT;
            if (ray.maxt < maxt) maxt = ray.maxt;
            if (maxt > mint)
                if (havran<true, count>(ray, mint, maxt, t, nullptr, ctr)) return true;
        }
        return false;
    }

    // ---- emitters -------------------------------------------------------
    // DiscreteDistribution::sample / sampleReuse (pmf.h:128-188)
    static size_t pmfSample(const float *cdf, size_t n, float x) {
        const float *entry = std::lower_bound(cdf, cdf + n + 1, x);
        size_t index = std::min(n - 1, (size_t)std::max((ptrdiff_t)0, entry - cdf - 1));
        while ((cdf[index + 1] - cdf[index]) == 0 && index < n) ++index;
        return index;
    }
    static size_t pmfSampleReuse(const float *cdf, size_t n, float &x, float &pdf) {
        size_t index = pmfSample(cdf, n, x);
        pdf = cdf[index + 1] - cdf[index];
        x = (x - cdf[index]) / (cdf[index + 1] - cdf[index]);
        return index;
    }

    struct DRec {   // DirectSamplingRecord (common.h:238-255)
        Vec p, n, ref, refN, d;
        float pdf = 0, dist = 0;
        int measureSolidAngle = 1;
        int emitter = -1;
    };

    // Shape::sampleDirect (shape.cpp:102-115) over TriMesh::samplePosition
    // (trimesh.cpp:412-423) / Rectangle::samplePosition (rectangle.cpp:200-207)
    void shapeSampleDirect(const mtsg_emitter &em, DRec &dRec, float sx, float sy) const {
        const mtsg_shape &sh = d.shapes[em.shape];
        if (sh.type == MTSG_SHAPE_MESH) {
            const float *cdf = d.emitter_tri_cdf + em.cdf_offset;
            float pdfDummy;
            size_t index = pmfSampleReuse(cdf, sh.tri_count, sy, pdfDummy);
            uint32_t g = sh.tri_begin + (uint32_t)index;
            const uint32_t i0 = d.tri_idx[3 * g], i1 = d.tri_idx[3 * g + 1], i2 = d.tri_idx[3 * g + 2];
            const Vec p0 = vtx(i0), p1 = vtx(i1), p2 = vtx(i2);
            // Triangle::sample (triangle.cpp:24-60), squareToUniformTriangle (warp.cpp:76-79)
            float a = safe_sqrt(1.0f - sx);
            float bx = 1 - a, by = a * sy;
            Vec sideA = p1 - p0, sideB = p2 - p0;
            dRec.p = p0 + (sideA * bx) + (sideB * by);
            if (!sh.face_normals) {
                dRec.n = normalize(nrm(i0) * (1.0f - bx - by) + nrm(i1) * bx + nrm(i2) * by);
            } else {
                dRec.n = normalize(cross(sideA, sideB));
            }
        } else {
            const mtsg_rect &r = d.rects[sh.rect];
            const float *m = r.to_world;
            float x = sx * 2 - 1, y = sy * 2 - 1;
            dRec.p = Vec(m[0] * x + m[1] * y + m[3], m[4] * x + m[5] * y + m[7], m[8] * x + m[9] * y + m[11]);
            dRec.n = Vec(r.frame_n[0], r.frame_n[1], r.frame_n[2]);
        }
        dRec.pdf = em.inv_area;
        dRec.d = dRec.p - dRec.ref;
        float distSquared = dot(dRec.d, dRec.d);
        dRec.dist = std::sqrt(distSquared);
        dRec.d = dRec.d / dRec.dist;
        float dp = absDot(dRec.d, dRec.n);
        dRec.pdf *= dp != 0 ? (distSquared / dp) : 0.0f;
        dRec.measureSolidAngle = 1;
    }

    // ------------------------------------------------------------------
    // EnvironmentMap (src/emitters/envmap.cpp) over TMIPMap (mipmap.h)
    // ------------------------------------------------------------------
    MipMap envMip() const { return MipMap{d.envmap.mip, d.env_texels}; }   // u repeats, v clamps

    // Intersection::computePartials (src/librender/intersection.cpp:5-80) for
    // a camera ray with (scaled) differentials rxD / ryD from origin o
    // (rxOrigin = ryOrigin = o for the perspective camera)
    static void computePartials(const Its &its, const Vec &o, const Vec &rxD, const Vec &ryD, float &dudx, float &dvdx,
                                float &dudy, float &dvdy) {
        dudx = dvdx = dudy = dvdy = 0.0f;
        const auto isZero = [](const Vec &v) { return v.x == 0 && v.y == 0 && v.z == 0; };
        if (isZero(its.dpdu) && isZero(its.dpdv)) return;
        const Vec &n = its.geoFrame.n;
        const float pp = dot(n, its.p), pox = dot(n, o), poy = dot(n, o), prx = dot(n, rxD), pry = dot(n, ryD);
        if (prx == 0 || pry == 0) return;
        const float tx = (pp - pox) / prx, ty = (pp - poy) / pry;
        const float absX = std::abs(n.x), absY = std::abs(n.y), absZ = std::abs(n.z);
        int axes[2];
        if (absX > absY && absX > absZ) { axes[0] = 1; axes[1] = 2; }
        else if (absY > absZ) { axes[0] = 0; axes[1] = 2; }
        else { axes[0] = 0; axes[1] = 1; }
        float A[2][2], Bx[2], By[2], x[2];
        A[0][0] = its.dpdu[axes[0]]; A[0][1] = its.dpdv[axes[0]];
        A[1][0] = its.dpdu[axes[1]]; A[1][1] = its.dpdv[axes[1]];
        const Vec px = o + rxD * tx, py = o + ryD * ty;
        Bx[0] = px[axes[0]] - its.p[axes[0]]; Bx[1] = px[axes[1]] - its.p[axes[1]];
        By[0] = py[axes[0]] - its.p[axes[0]]; By[1] = py[axes[1]] - its.p[axes[1]];
        // solveLinearSystem2x2 (src/libcore/util.cpp:527-539)
        auto solve = [&](const float b[2]) {
            const float det = A[0][0] * A[1][1] - A[0][1] * A[1][0];
            if (std::abs(det) <= 0x1p-128f) return false;   // RCPOVERFLOW
            const float inverse = 1.0f / det;
            x[0] = (A[1][1] * b[0] - A[0][1] * b[1]) * inverse;
            x[1] = (A[0][0] * b[1] - A[1][0] * b[0]) * inverse;
            return true;
        };
        if (solve(Bx)) { dudx = x[0]; dvdx = x[1]; }
        else { dudx = 1; dvdx = 0; }
        if (solve(By)) { dudy = x[0]; dvdy = x[1]; }
        else { dudy = 1; dvdy = 0; }   // the reference sets dudy twice and leaves dvdy unset
    }

    // The reflectance a BSDF record sees at a hit: its constant, or its bitmap
    // texture through Texture2D::eval(its) (texture.cpp:112-121) -> the
    // filtered lookup with UV partials when the ray carries differentials (the
    // camera ray, records.inl:69-75), BitmapTexture::eval(uv) otherwise
    // (bitmap.cpp:431-499) -> times the ScaleTexture of ensureEnergyConservation
    Spec reflectance(const mtsg_bsdf &b, const Its &its, const Vec &rayO, const struct RayDiff *diff) const;
    Vec envToLocal(const Vec &v) const {
        const float *m = d.envmap.to_local;
        return Vec(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z, m[6] * v.x + m[7] * v.y + m[8] * v.z);
    }
    Vec envToWorld(const Vec &v) const {
        const float *m = d.envmap.to_world;
        return Vec(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z, m[6] * v.x + m[7] * v.y + m[8] * v.z);
    }
    // EnvironmentMap::evalEnvironment (envmap.cpp:380-410)
    Spec envEvalEnvironment(const Ray &ray, bool hasDiff, const Vec &rxD, const Vec &ryD) const {
        const Vec v = envToLocal(ray.d);
        const float ux = std::atan2(v.x, -v.z) * kInvTwoPi, uy = std::acos(std::min(1.0f, std::max(-1.0f, v.y))) * kInvPi;
        Spec value;
        if (!hasDiff) {
            value = envMip().bilinear(0, ux, uy);
        } else {
            const Vec dvdx = envToLocal(rxD) - v, dvdy = envToLocal(ryD) - v;
            const float t1 = kInvTwoPi / (v.x * v.x + v.z * v.z),
                        t2 = -kInvPi / std::max(safe_sqrt(1.0f - v.y * v.y), kEpsilon);
            value = envMip().filtered(ux, uy, t1 * (dvdx.z * v.x - dvdx.x * v.z), t2 * dvdx.y, t1 * (dvdy.z * v.x - dvdy.x * v.z),
                                t2 * dvdy.y);
        }
        return value * d.envmap.scale;
    }
    // sampleReuse (envmap.cpp:628-633)
    static uint32_t envSampleReuse(const float *cdf, uint32_t size, float &sample) {
        const float *entry = std::lower_bound(cdf, cdf + size + 1, sample);
        const uint32_t index = std::min((uint32_t)std::max((ptrdiff_t)0, entry - cdf - 1), size - 1);
        sample = (sample - cdf[index]) / (cdf[index + 1] - cdf[index]);
        return index;
    }
    static float intervalToTent(float sample) {   // warp.cpp:143-155
        float sign;
        if (sample < 0.5f) { sign = 1; sample *= 2; }
        else { sign = -1; sample = 2 * (sample - 0.5f); }
        return sign * (1 - std::sqrt(sample));
    }
    // envmap.cpp:574-600
    void envInternalSample(float sx, float sy, Vec &dOut, Spec &value, float &pdf) const {
        const mtsg_envmap &E = d.envmap;
        const int W = E.mip.level_w[0], H = E.mip.level_h[0];
        const MipMap M = envMip();
        const uint32_t row = envSampleReuse(d.env_cdf_rows, H, sy);
        const uint32_t col = envSampleReuse(d.env_cdf_cols + row * (W + 1), W, sx);
        const float px = (float)col + intervalToTent(sx), py = (float)row + intervalToTent(sy);
        const int xPos = (int)std::floor(px), yPos = (int)std::floor(py);
        const float dx1 = px - xPos, dx2 = 1.0f - dx1, dy1 = py - yPos, dy2 = 1.0f - dy1;
        const Spec value1 = M.texel(0, xPos, yPos) * dx2 * dy2 + M.texel(0, xPos + 1, yPos) * dx1 * dy2;
        const Spec value2 = M.texel(0, xPos, yPos + 1) * dx2 * dy1 + M.texel(0, xPos + 1, yPos + 1) * dx1 * dy1;
        value = (value1 + value2) * E.scale;
        pdf = (value1.luminance() * d.env_row_weights[std::min(std::max(yPos, 0), H - 1)] +
               value2.luminance() * d.env_row_weights[std::min(std::max(yPos + 1, 0), H - 1)]) * E.normalization;
        const float sinPhi = std::sin(E.pixel_size[0] * (px + 0.5f)), cosPhi = std::cos(E.pixel_size[0] * (px + 0.5f));
        const float sinTheta = std::sin(E.pixel_size[1] * (py + 0.5f)), cosTheta = std::cos(E.pixel_size[1] * (py + 0.5f));
        dOut = Vec(sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta);
        pdf /= std::max(std::fabs(sinTheta), kEpsilon);
    }
    // envmap.cpp:603-633
    float envInternalPdf(const Vec &dl) const {
        const mtsg_envmap &E = d.envmap;
        const int W = E.mip.level_w[0], H = E.mip.level_h[0];
        const MipMap M = envMip();
        const float ux = std::atan2(dl.x, -dl.z) * kInvTwoPi, uy = std::acos(std::min(1.0f, std::max(-1.0f, dl.y))) * kInvPi;
        if (!std::isfinite(ux) || !std::isfinite(uy)) return 0.0f;
        const float u = ux * W - 0.5f, v = uy * H - 0.5f;
        const int xPos = (int)std::floor(u), yPos = (int)std::floor(v);
        const float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
        const Spec value1 = M.texel(0, xPos, yPos) * dx2 * dy2 + M.texel(0, xPos + 1, yPos) * dx1 * dy2;
        const Spec value2 = M.texel(0, xPos, yPos + 1) * dx2 * dy1 + M.texel(0, xPos + 1, yPos + 1) * dx1 * dy1;
        const float sinTheta = safe_sqrt(1 - dl.y * dl.y);
        return (value1.luminance() * d.env_row_weights[std::min(std::max(yPos, 0), H - 1)] +
                value2.luminance() * d.env_row_weights[std::min(std::max(yPos + 1, 0), H - 1)]) *
               E.normalization / std::max(std::fabs(sinTheta), kEpsilon);
    }
    // BSphere::rayIntersect (bsphere.h:88-95) + solveQuadratic (util.cpp:447-485)
    bool envSphere(const Vec &o, const Vec &dir, float &nearT, float &farT) const {
        const mtsg_envmap &E = d.envmap;
        const Vec oc = o - Vec(E.bsphere_center[0], E.bsphere_center[1], E.bsphere_center[2]);
        const float A = dot(dir, dir), B = 2 * dot(oc, dir), C = dot(oc, oc) - E.bsphere_radius * E.bsphere_radius;
        if (A == 0) {
            if (B != 0) { nearT = farT = -C / B; return true; }
            return false;
        }
        const float discrim = B * B - 4.0f * A * C;
        if (discrim < 0) return false;
        const float sq = std::sqrt(discrim), temp = B < 0 ? -0.5f * (B - sq) : -0.5f * (B + sq);
        nearT = temp / A;
        farT = C / temp;
        if (nearT > farT) std::swap(nearT, farT);
        return true;
    }
    // EnvironmentMap::sampleDirect (envmap.cpp:516-543)
    Spec envSampleDirect(DRec &dRec, float sx, float sy) const {
        Vec dl;
        Spec value;
        float pdf;
        envInternalSample(sx, sy, dl, value, pdf);
        const Vec dw = envToWorld(dl);
        Ray r;
        r.o = dRec.ref;
        r.setDirection(dw);
        float nearT, farT;
        if (value.isZero() || pdf == 0 || !envSphere(r.o, r.d, nearT, farT) || nearT >= 0 || farT <= 0) {
            dRec.pdf = 0.0f;
            return Spec(0.0f);
        }
        dRec.pdf = pdf;
        dRec.p = r.o + r.d * farT;
        dRec.d = r.d;
        dRec.dist = farT;
        dRec.measureSolidAngle = 1;
        return value / pdf;
    }

    // Scene::sampleEmitterDirect (scene.cpp:910-947) + AreaLight::sampleDirect (area.cpp:150-165)
    template <bool count>
    Spec sampleEmitterDirect(DRec &dRec, float sx, float sy, Counters *ctr, bool testVisibility = true) const {
        float emPdf;
        size_t index = pmfSampleReuse(d.emitter_cdf, d.n_emitters, sx, emPdf);
        const mtsg_emitter &em = d.emitters[index];
        Spec value;
        if (em.type == MTSG_EMITTER_ENVMAP) {
            value = envSampleDirect(dRec, sx, sy);
        } else {
            shapeSampleDirect(em, dRec, sx, sy);
            if (dot(dRec.d, dRec.refN) >= 0 && dot(dRec.d, dRec.n) < 0 && dRec.pdf != 0) {
                value = Spec::of(em.radiance) / dRec.pdf;
            } else {
                dRec.pdf = 0.0f;
                value = Spec(0.0f);
            }
        }
        if (dRec.pdf != 0) {
            Ray ray;
            ray.o = dRec.ref;
            ray.setDirection(dRec.d);
            ray.mint = kEpsilon;
            ray.maxt = dRec.dist * (1 - kShadowEpsilon);
            if (testVisibility && rayIntersectShadow<count>(ray, ctr)) return Spec(0.0f);
            dRec.emitter = (int)index;
            dRec.pdf *= emPdf;
            value = value / emPdf;
            return value;
        }
        return Spec(0.0f);
    }

    // Scene::pdfEmitterDirect (scene.cpp:1067-1071), AreaLight::pdfDirect (area.cpp:167-176),
    // Shape::pdfDirect (shape.cpp:117-126)
    float pdfEmitterDirect(const DRec &dRec) const {
        const mtsg_emitter &em = d.emitters[dRec.emitter];
        if (em.type == MTSG_EMITTER_ENVMAP)   // EnvironmentMap::pdfDirect, solid angle (envmap.cpp:545-556)
            return envInternalPdf(envToLocal(dRec.d)) * em.pdf_discrete;
        float pdf = 0.0f;
        if (dot(dRec.d, dRec.refN) >= 0 && dot(dRec.d, dRec.n) < 0) {
            float pdfPos = em.inv_area;
            pdf = pdfPos * (dRec.dist * dRec.dist) / absDot(dRec.d, dRec.n);
        }
        return pdf * em.pdf_discrete;
    }
};

// ---------------------------------------------------------------------------
// BSDFs
// ---------------------------------------------------------------------------
enum { EDeltaReflection = 4, EDeltaTransmission = 16, EGlossyReflection = 2, EDiffuseReflection = 1, EGlossyTransmission = 32 };   // own bit numbering of the bsdf.h:224-285 lobe types

struct BRec {   // BSDFSamplingRecord (bsdf.h:40-193)
    Vec wi, wo;
    float eta = 1.0f;
    int sampledType = 0;
};

// warp.cpp:81-102 + 43-52
Vec squareToCosineHemisphere(float sx, float sy) {
    float r1 = 2.0f * sx - 1.0f, r2 = 2.0f * sy - 1.0f;
    float phi, r;
    if (r1 == 0 && r2 == 0) { r = phi = 0; }
    else if (r1 * r1 > r2 * r2) { r = r1; phi = (float)(M_PI / 4.0f) * (r2 / r1); }
    else { r = r2; phi = (float)(M_PI / 2.0f) - (r1 / r2) * (float)(M_PI / 4.0f); }
    float cosPhi = std::cos(phi), sinPhi = std::sin(phi);
    float px = r * cosPhi, py = r * sinPhi;
    float z = safe_sqrt(1.0f - px * px - py * py);
    if (z == 0) z = 1e-10f;
    return Vec(px, py, z);
}

// MicrofacetDistribution (microfacet.h): Beckmann, GGX and Phong /
// Ashikhmin-Shirley, isotropic or anisotropic
struct Microfacet {
    int type;
    float au, av;
    bool sampleVisible;
    float eu = 0, ev = 0;   // Phong exponents
    Microfacet(int t, float u, float v, bool vis) : type(t), au(u), av(v), sampleVisible(vis) {
        if (type == MTSG_MF_PHONG) {   // microfacet.h:140-144, computePhongExponent :701-704
            sampleVisible = false;
            eu = std::max(2.0f / (au * au) - 2.0f, 0.0f);
            ev = std::max(2.0f / (av * av) - 2.0f, 0.0f);
        }
    }
    bool isotropic() const { return au == av; }
    void scaleAlpha(float v) {   // microfacet.h:178-183
        au *= v;
        av *= v;
        if (type == MTSG_MF_PHONG) {
            eu = std::max(2.0f / (au * au) - 2.0f, 0.0f);
            ev = std::max(2.0f / (av * av) - 2.0f, 0.0f);
        }
    }
    float phongExponent(const Vec &v) const {   // interpolatePhongExponent :554-565
        const float st2 = sinTheta2(v);
        if (isotropic() || st2 <= 2.93873587705571876e-39f) return eu;
        float inv = 1 / st2;
        return eu * (v.x * v.x * inv) + ev * (v.y * v.y * inv);
    }
    void sampleFirstQuadrant(float u1, float &phi, float &exponent) const {   // :707-715
        phi = std::atan(std::sqrt((eu + 2.0f) / (ev + 2.0f)) * std::tan((float)M_PI * u1 * 0.5f));
        float sinPhi = std::sin(phi), cosPhi = std::cos(phi);
        exponent = eu * cosPhi * cosPhi + ev * sinPhi * sinPhi;
    }
    float eval(const Vec &m) const {   // microfacet.h:191-234
        if (cosTheta(m) <= 0) return 0.0f;
        float ct2 = cosTheta2(m);
        float be = ((m.x * m.x) / (au * au) + (m.y * m.y) / (av * av)) / ct2;
        float result;
        if (type == MTSG_MF_BECKMANN) {
            result = fastexp(-be) / ((float)M_PI * au * av * ct2 * ct2);
        } else if (type == MTSG_MF_GGX) {
            float root = (1.0f + be) * ct2;
            result = 1.0f / ((float)M_PI * au * av * root * root);
        } else {
            result = std::sqrt((eu + 2) * (ev + 2)) * (float)(0.5 / M_PI) * std::pow(cosTheta(m), phongExponent(m));
        }
        if (result * cosTheta(m) < 1e-20f) result = 0;
        return result;
    }
    float projectRoughness(const Vec &v) const {   // microfacet.h (isotropic)
        float invSinTheta2 = 1 / sinTheta2(v);
        if (au == av || invSinTheta2 <= 0) return au;
        float cosPhi2 = v.x * v.x * invSinTheta2, sinPhi2 = v.y * v.y * invSinTheta2;
        return std::sqrt(cosPhi2 * au * au + sinPhi2 * av * av);
    }
    float smithG1(const Vec &v, const Vec &m) const {   // microfacet.h:477-514
        if (dot(v, m) * cosTheta(v) <= 0) return 0.0f;
        float tt = std::abs(tanTheta(v));
        if (tt == 0.0f) return 1.0f;
        float alpha = projectRoughness(v);
        if (type != MTSG_MF_GGX) {   // Phong uses the Beckmann approximation
            float a = 1.0f / (alpha * tt);
            if (a >= 1.6f) return 1.0f;
            float aSqr = a * a;
            return (3.535f * a + 2.181f * aSqr) / (1.0f + 2.276f * a + 2.577f * aSqr);
        }
        float root = alpha * tt;
        return 2.0f / (1.0f + hypot2(1.0f, root));
    }
    float G(const Vec &wi, const Vec &wo, const Vec &m) const { return smithG1(wi, m) * smithG1(wo, m); }
    void sampleVisible11(float thetaI, float sx, float sy, float &slx, float &sly) const {   // :573-697
        const float SQRT_PI_INV = 1 / std::sqrt((float)M_PI);
        if (type == MTSG_MF_BECKMANN) {
            if (thetaI < 1e-4f) {
                float r = std::sqrt(-fastlog(1.0f - sx));
                float sinPhi = std::sin(2 * (float)M_PI * sy), cosPhi = std::cos(2 * (float)M_PI * sy);
                slx = r * cosPhi; sly = r * sinPhi;
                return;
            }
            float tanThetaI = std::tan(thetaI);
            float cotThetaI = 1 / tanThetaI;
            float a = -1, c = erf(cotThetaI);
            float sample_x = std::max(sx, 1e-6f);
            float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
            float b = c - (1 + c) * std::pow(1 - sample_x, fit);
            float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * std::exp(-cotThetaI * cotThetaI));
            int it = 0;
            while (++it < 10) {
                if (!(b >= a && b <= c)) b = 0.5f * (a + c);
                float invErf = erfinv(b);
                float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * std::exp(-invErf * invErf)) - sample_x;
                float derivative = normalization * (1 - invErf * tanThetaI);
                if (std::abs(value) < 1e-5f) break;
                if (value > 0) c = b; else a = b;
                b -= value / derivative;
            }
            slx = erfinv(b);
            sly = erfinv(2.0f * std::max(sy, 1e-6f) - 1.0f);
            return;
        }
        // GGX
        if (thetaI < 1e-4f) {
            float r = safe_sqrt(sx / (1 - sx));
            float sinPhi = std::sin(2 * (float)M_PI * sy), cosPhi = std::cos(2 * (float)M_PI * sy);
            slx = r * cosPhi; sly = r * sinPhi;
            return;
        }
        float tanThetaI = std::tan(thetaI);
        float a = 1 / tanThetaI;
        float G1 = 2.0f / (1.0f + safe_sqrt(1.0f + 1.0f / (a * a)));
        float A = 2.0f * sx / G1 - 1.0f;
        if (std::abs(A) == 1) A -= signum(A) * kEpsilon;
        float tmp = 1.0f / (A * A - 1.0f);
        float B = tanThetaI;
        float D = safe_sqrt(B * B * tmp * tmp - (A * A - B * B) * tmp);
        float slope_x_1 = B * tmp - D, slope_x_2 = B * tmp + D;
        slx = (A < 0.0f || slope_x_2 > 1.0f / tanThetaI) ? slope_x_1 : slope_x_2;
        float S;
        if (sy > 0.5f) { S = 1.0f; sy = 2.0f * (sy - 0.5f); }
        else { S = -1.0f; sy = 2.0f * (0.5f - sy); }
        float z = (sy * (sy * (sy * (-0.365728915865723f) + 0.790235037209296f) - 0.424965825137544f) + 0.000152998850436920f) /
                  (sy * (sy * (sy * (sy * 0.169507819808272f - 0.397203533833404f) - 0.232500544458471f) + 1.0f) - 0.539825872510702f);
        sly = S * z * std::sqrt(1.0f + slx * slx);
    }
    Vec sampleVisibleN(const Vec &wi_, float sx, float sy) const {   // :421-459
        Vec wi = normalize(Vec(au * wi_.x, av * wi_.y, wi_.z));
        float theta = 0, phi = 0;
        if (wi.z < 0.99999f) { theta = std::acos(wi.z); phi = std::atan2(wi.y, wi.x); }
        float sinPhi = std::sin(phi), cosPhi = std::cos(phi);
        float slx, sly;
        sampleVisible11(theta, sx, sy, slx, sly);
        float rx = cosPhi * slx - sinPhi * sly;
        float ry = sinPhi * slx + cosPhi * sly;
        rx *= au; ry *= av;
        float normalization = 1.0f / std::sqrt(rx * rx + ry * ry + 1.0f);
        return Vec(-rx * normalization, -ry * normalization, normalization);
    }
    float pdfVisible(const Vec &wi, const Vec &m) const {   // :462-466
        if (cosTheta(wi) == 0) return 0.0f;
        return smithG1(wi, m) * absDot(wi, m) * eval(m) / std::abs(cosTheta(wi));
    }
    Vec sampleAll(float sx, float sy, float &pdf) const {   // :287-397
        float sinPhiM, cosPhiM, cosThetaM;
        if (type == MTSG_MF_PHONG) {
            float phiM, exponent;
            if (isotropic()) {
                phiM = (2.0f * (float)M_PI) * sy;
                exponent = eu;
            } else if (sy < 0.25f) {
                sampleFirstQuadrant(4 * sy, phiM, exponent);
            } else if (sy < 0.5f) {
                sampleFirstQuadrant(4 * (0.5f - sy), phiM, exponent);
                phiM = (float)M_PI - phiM;
            } else if (sy < 0.75f) {
                sampleFirstQuadrant(4 * (sy - 0.5f), phiM, exponent);
                phiM += (float)M_PI;
            } else {
                sampleFirstQuadrant(4 * (1 - sy), phiM, exponent);
                phiM = 2 * (float)M_PI - phiM;
            }
            sinPhiM = std::sin(phiM); cosPhiM = std::cos(phiM);
            cosThetaM = std::pow(sx, 1.0f / (exponent + 2.0f));
            pdf = std::sqrt((eu + 2.0f) * (ev + 2.0f)) * (float)(0.5 / M_PI) * std::pow(cosThetaM, exponent + 1.0f);
        } else {
            float alphaSqr;
            if (isotropic()) {
                sinPhiM = std::sin((2.0f * (float)M_PI) * sy); cosPhiM = std::cos((2.0f * (float)M_PI) * sy);
                alphaSqr = au * au;
            } else {
                float phiM = std::atan(av / au * std::tan((float)M_PI + 2 * (float)M_PI * sy)) + (float)M_PI * std::floor(2 * sy + 0.5f);
                sinPhiM = std::sin(phiM); cosPhiM = std::cos(phiM);
                float cosSc = cosPhiM / au, sinSc = sinPhiM / av;
                alphaSqr = 1.0f / (cosSc * cosSc + sinSc * sinSc);
            }
            if (type == MTSG_MF_BECKMANN) {
                float tanThetaMSqr = alphaSqr * -fastlog(1.0f - sx);
                cosThetaM = 1.0f / std::sqrt(1.0f + tanThetaMSqr);
                pdf = (1.0f - sx) / ((float)M_PI * au * av * cosThetaM * cosThetaM * cosThetaM);
            } else {
                float tanThetaMSqr = alphaSqr * sx / (1.0f - sx);
                cosThetaM = 1.0f / std::sqrt(1.0f + tanThetaMSqr);
                float temp = 1 + tanThetaMSqr / alphaSqr;
                pdf = kInvPi / (au * av * cosThetaM * cosThetaM * cosThetaM * temp * temp);
            }
        }
        if (pdf < 1e-20f) pdf = 0;
        float sinThetaM = std::sqrt(std::max(0.0f, 1 - cosThetaM * cosThetaM));
        return Vec(sinThetaM * cosPhiM, sinThetaM * sinPhiM, cosThetaM);
    }
    Vec sample(const Vec &wi, float sx, float sy, float &pdf) const {   // :240-251
        if (sampleVisible) {
            Vec m = sampleVisibleN(wi, sx, sy);
            pdf = pdfVisible(wi, m);
            return m;
        }
        return sampleAll(sx, sy, pdf);
    }
    float pdf(const Vec &wi, const Vec &m) const {
        return sampleVisible ? pdfVisible(wi, m) : eval(m) * cosTheta(m);
    }
};

inline Microfacet mfOf(const mtsg_bsdf &b) { return Microfacet(b.distribution, b.alpha_u, b.alpha_v, b.sample_visible != 0); }

// util.cpp:651-681
float fresnelDielectricExt(float cosThetaI_, float &cosThetaT_, float eta) {
    if (eta == 1) { cosThetaT_ = -cosThetaI_; return 0.0f; }
    float scale = (cosThetaI_ > 0) ? 1 / eta : eta, cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) { cosThetaT_ = 0.0f; return 1.0f; }
    float cosThetaI = std::abs(cosThetaI_), cosThetaT = std::sqrt(cosThetaTSqr);
    float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    cosThetaT_ = (cosThetaI_ > 0) ? -cosThetaT : cosThetaT;
    return 0.5f * (Rs * Rs + Rp * Rp);
}

// util.cpp:739-761
Spec fresnelConductorExact(float cosThetaI, const Spec &eta, const Spec &k) {
    float cosThetaI2 = cosThetaI * cosThetaI, sinThetaI2 = 1 - cosThetaI2, sinThetaI4 = sinThetaI2 * sinThetaI2;
    Spec temp1 = eta * eta - k * k - Spec(sinThetaI2);
    Spec a2pb2 = sqrtSafe(temp1 * temp1 + k * k * eta * eta * 4);
    Spec a = sqrtSafe((a2pb2 + temp1) * 0.5f);
    Spec term1 = a2pb2 + Spec(cosThetaI2), term2 = a * (2 * cosThetaI);
    Spec Rs2 = (term1 - term2) / (term1 + term2);
    Spec term3 = a2pb2 * cosThetaI2 + Spec(sinThetaI4), term4 = term2 * sinThetaI2;
    Spec Rp2 = Rs2 * (term3 - term4) / (term3 + term4);
    return (Rp2 + Rs2) * 0.5f;
}

inline Vec reflectM(const Vec &wi, const Vec &m) { return m * (2 * dot(wi, m)) - wi; }

float fresnelDielectricExt1(float cosThetaI, float eta) {
    float cosThetaT;
    return fresnelDielectricExt(cosThetaI, cosThetaT, eta);
}
// SmoothPlastic (plastic.cpp:93-140): m_invEta2, the internal-reflection
// renormalised diffuse base and the Fresnel-steered specular probability
inline float plasticInvEta2(const mtsg_bsdf &b) { return 1 / (b.ior_eta * b.ior_eta); }
Spec plasticDiffuse(const mtsg_bsdf &b, Spec diff) {
    if (b.nonlinear) return diff / (Spec(1.0f) - diff * b.fdr_int);
    return diff / (1 - b.fdr_int);
}
float plasticProbSpecular(const mtsg_bsdf &b, float Fi) {
    return (Fi * b.spec_sampling_weight) / (Fi * b.spec_sampling_weight + (1 - Fi) * (1 - b.spec_sampling_weight));
}

// evalCubicInterp1D (spline.cpp:23-60) on [0, 1]
float evalCubicInterp1D(float x, const float *values, size_t size) {
    if (!(x >= 0.0f && x <= 1.0f)) return 0.0f;
    float t = (x * (size - 1)) / 1.0f;
    size_t k = std::max((size_t)0, std::min((size_t)t, size - 2));
    float f0 = values[k], f1 = values[k + 1], d0, d1;
    if (k > 0) d0 = 0.5f * (values[k + 1] - values[k - 1]);
    else d0 = values[k + 1] - values[k];
    if (k + 2 < size) d1 = 0.5f * (values[k + 2] - values[k]);
    else d1 = values[k + 1] - values[k];
    t = t - (float)k;
    float t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
}
// RoughTransmittance::eval, m_alphaFixed && m_etaFixed (rtrans.h:169-181,205-206)
float roughTransmittance(const mtsg_bsdf &b, float cosTheta) {
    float warpedCosTheta = std::pow(std::abs(cosTheta), 0.25f);
    if (!(cosTheta >= 0)) return 0.0f;
    float result = evalCubicInterp1D(warpedCosTheta, b.rtrans, MTSG_RTRANS_SAMPLES);
    return std::min(1.0f, std::max(0.0f, result));
}
// RoughPlastic::eval / pdf (roughplastic.cpp:302-385), both components
Spec roughPlasticEval(const mtsg_bsdf &b, const Spec &alb, const BRec &r) {
    if (cosTheta(r.wi) <= 0 || cosTheta(r.wo) <= 0) return Spec(0.0f);
    Microfacet distr = mfOf(b);
    Spec result(0.0f);
    Vec H = normalize(r.wo + r.wi);
    float D = distr.eval(H);
    float F = fresnelDielectricExt1(dot(r.wi, H), b.ior_eta);
    float G = distr.G(r.wi, r.wo, H);
    float value = F * D * G / (4.0f * cosTheta(r.wi));
    result += Spec::of(b.spec_refl) * value;
    float T12 = roughTransmittance(b, cosTheta(r.wi)), T21 = roughTransmittance(b, cosTheta(r.wo));
    result += plasticDiffuse(b, alb) * (kInvPi * cosTheta(r.wo) * T12 * T21 * plasticInvEta2(b));
    return result;
}
float roughPlasticPdf(const mtsg_bsdf &b, const BRec &r) {
    if (cosTheta(r.wi) <= 0 || cosTheta(r.wo) <= 0) return 0.0f;
    Microfacet distr = mfOf(b);
    Vec H = normalize(r.wo + r.wi);
    float probSpecular = 1 - roughTransmittance(b, cosTheta(r.wi));
    probSpecular = plasticProbSpecular(b, probSpecular);
    float probDiffuse = 1 - probSpecular;
    float dwh_dwo = 1.0f / (4.0f * dot(r.wo, H));
    float prob = distr.pdf(r.wi, H);
    float result = prob * dwh_dwo * probSpecular;
    result += probDiffuse * (kInvPi * cosTheta(r.wo));
    return result;
}

// BSDF::eval (measure = ESolidAngle for smooth BSDFs; dielectric only
// evaluates EDiscrete, so it returns 0 here: dielectric.cpp:228-250)
// alb: the record's `reflectance` / `diffuseReflectance` at the hit (the
// constant, or its texture's value: SceneView::reflectance)
Spec bsdfEval(const mtsg_bsdf &b, const Spec &alb, const BRec &r) {
    if (b.type == MTSG_BSDF_DIFFUSE) {   // diffuse.cpp:107-116
        if (!b.smooth || cosTheta(r.wi) <= 0 || cosTheta(r.wo) <= 0) return Spec(0.0f);
        return alb * (kInvPi * cosTheta(r.wo));
    }
    if (b.type == MTSG_BSDF_ROUGHCONDUCTOR) {   // roughconductor.cpp:235-268
        if (cosTheta(r.wi) <= 0 || cosTheta(r.wo) <= 0) return Spec(0.0f);
        Vec H = normalize(r.wo + r.wi);
        Microfacet distr = mfOf(b);
        const float D = distr.eval(H);
        if (D == 0) return Spec(0.0f);
        const Spec F = fresnelConductorExact(dot(r.wi, H), Spec::of(b.eta), Spec::of(b.k)) * Spec::of(b.spec_refl);
        const float G = distr.G(r.wi, r.wo, H);
        float model = D * G / (4.0f * cosTheta(r.wi));
        return F * model;
    }
    if (b.type == MTSG_BSDF_ROUGHDIELECTRIC) {   // roughdielectric.cpp:265-335
        if (cosTheta(r.wi) == 0) return Spec(0.0f);
        bool reflect = cosTheta(r.wi) * cosTheta(r.wo) > 0;
        Vec H;
        if (reflect) {
            H = normalize(r.wo + r.wi);
        } else {
            float eta = cosTheta(r.wi) > 0 ? b.ior_eta : b.ior_inv_eta;
            H = normalize(r.wi + r.wo * eta);
        }
        H = H * signum(cosTheta(H));
        Microfacet distr = mfOf(b);
        const float D = distr.eval(H);
        if (D == 0) return Spec(0.0f);
        const float F = fresnelDielectricExt1(dot(r.wi, H), b.ior_eta);
        const float G = distr.G(r.wi, r.wo, H);
        if (reflect) {
            float value = F * D * G / (4.0f * std::abs(cosTheta(r.wi)));
            return Spec::of(b.spec_refl) * value;
        }
        float eta = cosTheta(r.wi) > 0.0f ? b.ior_eta : b.ior_inv_eta;
        float sqrtDenom = dot(r.wi, H) + eta * dot(r.wo, H);
        float value = ((1 - F) * D * G * eta * eta * dot(r.wi, H) * dot(r.wo, H)) / (cosTheta(r.wi) * sqrtDenom * sqrtDenom);
        float factor = cosTheta(r.wi) > 0 ? b.ior_inv_eta : b.ior_eta;   // ERadiance
        return Spec::of(b.spec_trans) * std::abs(value * factor * factor);
    }
    if (b.type == MTSG_BSDF_PLASTIC) {   // plastic.cpp:190-233 (ESolidAngle: the diffuse part)
        if (cosTheta(r.wo) <= 0 || cosTheta(r.wi) <= 0) return Spec(0.0f);
        float Fi = fresnelDielectricExt1(cosTheta(r.wi), b.ior_eta);
        float Fo = fresnelDielectricExt1(cosTheta(r.wo), b.ior_eta);
        return plasticDiffuse(b, alb) * (kInvPi * cosTheta(r.wo) * plasticInvEta2(b) * (1 - Fi) * (1 - Fo));
    }
    if (b.type == MTSG_BSDF_ROUGHPLASTIC) return roughPlasticEval(b, alb, r);
    return Spec(0.0f);   // dielectric / conductor: delta components only (EDiscrete)
}

float bsdfPdf(const mtsg_bsdf &b, const BRec &r) {
    if (b.type == MTSG_BSDF_DIFFUSE) {   // diffuse.cpp:118-126
        if (!b.smooth || cosTheta(r.wi) <= 0 || cosTheta(r.wo) <= 0) return 0.0f;
        return kInvPi * cosTheta(r.wo);
    }
    if (b.type == MTSG_BSDF_ROUGHCONDUCTOR) {   // roughconductor.cpp:270-293
        if (cosTheta(r.wi) <= 0 || cosTheta(r.wo) <= 0) return 0.0f;
        Vec H = normalize(r.wo + r.wi);
        Microfacet distr = mfOf(b);
        if (distr.sampleVisible) return distr.eval(H) * distr.smithG1(r.wi, H) / (4.0f * cosTheta(r.wi));
        return distr.pdf(r.wi, H) / (4 * absDot(r.wo, H));
    }
    if (b.type == MTSG_BSDF_ROUGHDIELECTRIC) {   // roughdielectric.cpp:337-400
        bool reflect = cosTheta(r.wi) * cosTheta(r.wo) > 0;
        Vec H;
        float dwh_dwo;
        if (reflect) {
            H = normalize(r.wo + r.wi);
            dwh_dwo = 1.0f / (4.0f * dot(r.wo, H));
        } else {
            float eta = cosTheta(r.wi) > 0 ? b.ior_eta : b.ior_inv_eta;
            H = normalize(r.wi + r.wo * eta);
            float sqrtDenom = dot(r.wi, H) + eta * dot(r.wo, H);
            dwh_dwo = (eta * eta * dot(r.wo, H)) / (sqrtDenom * sqrtDenom);
        }
        H = H * signum(cosTheta(H));
        Microfacet sampleDistr = mfOf(b);
        if (!sampleDistr.sampleVisible) sampleDistr.scaleAlpha(1.2f - 0.2f * std::sqrt(std::abs(cosTheta(r.wi))));
        float prob = sampleDistr.pdf(r.wi * signum(cosTheta(r.wi)), H);
        float F = fresnelDielectricExt1(dot(r.wi, H), b.ior_eta);
        prob *= reflect ? F : (1 - F);
        return std::abs(prob * dwh_dwo);
    }
    if (b.type == MTSG_BSDF_PLASTIC) {   // plastic.cpp:235-263
        if (cosTheta(r.wo) <= 0 || cosTheta(r.wi) <= 0) return 0.0f;
        float Fi = fresnelDielectricExt1(cosTheta(r.wi), b.ior_eta);
        return kInvPi * cosTheta(r.wo) * (1 - plasticProbSpecular(b, Fi));
    }
    if (b.type == MTSG_BSDF_ROUGHPLASTIC) return roughPlasticPdf(b, r);
    return 0.0f;
}

// BSDF::sample(bRec, pdf, sample); next1d: bRec.sampler->next1D(), drawn
// only where the reference draws it (roughdielectric.cpp:531-539)
template <class Next1D>
Spec bsdfSample(const mtsg_bsdf &b, const Spec &alb, BRec &r, float &pdf, float sx, float sy, Next1D &&next1d) {
    if (b.type == MTSG_BSDF_DIFFUSE) {   // diffuse.cpp:139-150
        if (cosTheta(r.wi) <= 0) return Spec(0.0f);
        r.wo = squareToCosineHemisphere(sx, sy);
        r.eta = 1.0f;
        r.sampledType = EDiffuseReflection;
        pdf = kInvPi * cosTheta(r.wo);
        return alb;
    }
    if (b.type == MTSG_BSDF_ROUGHCONDUCTOR) {   // roughconductor.cpp:345-394
        if (cosTheta(r.wi) < 0) return Spec(0.0f);
        Microfacet distr = mfOf(b);
        Vec m = distr.sample(r.wi, sx, sy, pdf);
        if (pdf == 0) return Spec(0.0f);
        r.wo = reflectM(r.wi, m);
        r.eta = 1.0f;
        r.sampledType = EGlossyReflection;
        if (cosTheta(r.wo) <= 0) return Spec(0.0f);
        Spec F = fresnelConductorExact(dot(r.wi, m), Spec::of(b.eta), Spec::of(b.k)) * Spec::of(b.spec_refl);
        float weight;
        if (distr.sampleVisible) weight = distr.smithG1(r.wo, m);
        else weight = distr.eval(m) * distr.G(r.wi, r.wo, m) * dot(r.wi, m) / (pdf * cosTheta(r.wi));
        pdf /= 4.0f * dot(r.wo, m);
        return F * weight;
    }
    if (b.type == MTSG_BSDF_DIELECTRIC) {   // dielectric.cpp:277-333 (both components)
        float cosThetaT;
        float F = fresnelDielectricExt(cosTheta(r.wi), cosThetaT, b.ior_eta);
        if (sx <= F) {
            r.sampledType = EDeltaReflection;
            r.wo = Vec(-r.wi.x, -r.wi.y, r.wi.z);
            r.eta = 1.0f;
            pdf = F;
            return Spec::of(b.spec_refl);
        }
        r.sampledType = EDeltaTransmission;
        float scale = -(cosThetaT < 0 ? b.ior_inv_eta : b.ior_eta);
        r.wo = Vec(scale * r.wi.x, scale * r.wi.y, cosThetaT);
        r.eta = cosThetaT < 0 ? b.ior_eta : b.ior_inv_eta;
        pdf = 1 - F;
        float factor = cosThetaT < 0 ? b.ior_inv_eta : b.ior_eta;   // ERadiance
        return Spec::of(b.spec_trans) * (factor * factor);
    }
    if (b.type == MTSG_BSDF_CONDUCTOR) {   // conductor.cpp:220-236
        if (cosTheta(r.wi) <= 0) return Spec(0.0f);
        r.sampledType = EDeltaReflection;
        r.wo = Vec(-r.wi.x, -r.wi.y, r.wi.z);
        r.eta = 1.0f;
        pdf = 1;
        return Spec::of(b.spec_refl) * fresnelConductorExact(cosTheta(r.wi), Spec::of(b.eta), Spec::of(b.k));
    }
    if (b.type == MTSG_BSDF_ROUGHDIELECTRIC) {   // roughdielectric.cpp:508-590 (both components)
        Microfacet distr = mfOf(b);
        Microfacet sampleDistr = distr;
        if (!distr.sampleVisible) sampleDistr.scaleAlpha(1.2f - 0.2f * std::sqrt(std::abs(cosTheta(r.wi))));
        float microfacetPDF;
        const Vec m = sampleDistr.sample(r.wi * signum(cosTheta(r.wi)), sx, sy, microfacetPDF);
        if (microfacetPDF == 0) return Spec(0.0f);
        pdf = microfacetPDF;
        float cosThetaT;
        float F = fresnelDielectricExt(dot(r.wi, m), cosThetaT, b.ior_eta);
        Spec weight(1.0f);
        bool sampleReflection = true;
        if (next1d() > F) {
            sampleReflection = false;
            pdf *= 1 - F;
        } else {
            pdf *= F;
        }
        float dwh_dwo;
        if (sampleReflection) {
            r.wo = reflectM(r.wi, m);
            r.eta = 1.0f;
            r.sampledType = EGlossyReflection;
            if (cosTheta(r.wi) * cosTheta(r.wo) <= 0) return Spec(0.0f);
            weight = weight * Spec::of(b.spec_refl);
            dwh_dwo = 1.0f / (4.0f * dot(r.wo, m));
        } else {
            if (cosThetaT == 0) return Spec(0.0f);
            float e = cosThetaT < 0 ? 1 / b.ior_eta : b.ior_eta;   // refract (util.cpp:767-772)
            r.wo = m * (dot(r.wi, m) * e + cosThetaT) - r.wi * e;
            r.eta = cosThetaT < 0 ? b.ior_eta : b.ior_inv_eta;
            r.sampledType = EGlossyTransmission;
            if (cosTheta(r.wi) * cosTheta(r.wo) >= 0) return Spec(0.0f);
            float factor = cosThetaT < 0 ? b.ior_inv_eta : b.ior_eta;   // ERadiance
            weight = weight * (Spec::of(b.spec_trans) * (factor * factor));
            float sqrtDenom = dot(r.wi, m) + r.eta * dot(r.wo, m);
            dwh_dwo = (r.eta * r.eta * dot(r.wo, m)) / (sqrtDenom * sqrtDenom);
        }
        if (distr.sampleVisible) weight = weight * distr.smithG1(r.wo, m);
        else weight = weight * std::abs(distr.eval(m) * distr.G(r.wi, r.wo, m) * dot(r.wi, m) / (microfacetPDF * cosTheta(r.wi)));
        pdf *= std::abs(dwh_dwo);
        return weight;
    }
    if (b.type == MTSG_BSDF_ROUGHPLASTIC) {   // roughplastic.cpp:387-455
        if (cosTheta(r.wi) <= 0) return Spec(0.0f);
        bool choseSpecular = true;
        float probSpecular = plasticProbSpecular(b, 1 - roughTransmittance(b, cosTheta(r.wi)));
        if (sy < probSpecular) {
            sy /= probSpecular;
        } else {
            sy = (sy - probSpecular) / (1 - probSpecular);
            choseSpecular = false;
        }
        if (choseSpecular) {
            Microfacet distr = mfOf(b);
            float mpdf;
            Vec m = distr.sample(r.wi, sx, sy, mpdf);
            r.wo = reflectM(r.wi, m);
            r.sampledType = EGlossyReflection;
            if (cosTheta(r.wo) <= 0) return Spec(0.0f);
        } else {
            r.sampledType = EDiffuseReflection;
            r.wo = squareToCosineHemisphere(sx, sy);
        }
        r.eta = 1.0f;
        pdf = roughPlasticPdf(b, r);
        if (pdf == 0) return Spec(0.0f);
        return roughPlasticEval(b, alb, r) / pdf;
    }
    if (b.type == MTSG_BSDF_PLASTIC) {   // plastic.cpp:344-390 (both components)
        if (cosTheta(r.wi) <= 0) return Spec(0.0f);
        float Fi = fresnelDielectricExt1(cosTheta(r.wi), b.ior_eta);
        r.eta = 1.0f;
        float probSpecular = plasticProbSpecular(b, Fi);
        if (sx < probSpecular) {
            r.sampledType = EDeltaReflection;
            r.wo = Vec(-r.wi.x, -r.wi.y, r.wi.z);
            pdf = probSpecular;
            return Spec::of(b.spec_refl) * Fi / probSpecular;
        }
        r.sampledType = EDiffuseReflection;
        r.wo = squareToCosineHemisphere((sx - probSpecular) / (1 - probSpecular), sy);
        float Fo = fresnelDielectricExt1(cosTheta(r.wo), b.ior_eta);
        pdf = (1 - probSpecular) * (kInvPi * cosTheta(r.wo));
        return plasticDiffuse(b, alb) * (plasticInvEta2(b) * (1 - Fi) * (1 - Fo) / (1 - probSpecular));
    }
    return Spec(0.0f);
}

// TwoSidedBRDF (twosided.cpp:103-170): a twosided front record hands
// back-side queries to bsdfs[back] with the z components negated
const mtsg_bsdf &bsdfSide(const mtsg_bsdf *all, const mtsg_bsdf &b, BRec &r, bool sampling, bool &flipped) {
    flipped = b.twosided && (sampling ? cosTheta(r.wi) < 0 : !(cosTheta(r.wi) > 0));
    if (!flipped) return b;
    r.wi.z *= -1;
    if (!sampling) r.wo.z *= -1;
    return all[b.back];
}
template <class Alb>
Spec bsdfEvalTS(const mtsg_bsdf *all, const mtsg_bsdf &b, BRec r, Alb &&alb) {
    bool f;
    const mtsg_bsdf &nb = bsdfSide(all, b, r, false, f);
    return bsdfEval(nb, alb(nb), r);
}
float bsdfPdfTS(const mtsg_bsdf *all, const mtsg_bsdf &b, BRec r) {
    bool f;
    return bsdfPdf(bsdfSide(all, b, r, false, f), r);
}
template <class Next1D, class Alb>
Spec bsdfSampleTS(const mtsg_bsdf *all, const mtsg_bsdf &b, BRec &r, float &pdf, float sx, float sy, Next1D &&next1d, Alb &&alb) {
    bool flipped;
    const mtsg_bsdf &nb = bsdfSide(all, b, r, true, flipped);
    Spec result = bsdfSample(nb, alb(nb), r, pdf, sx, sy, next1d);
    if (flipped) {
        r.wi.z *= -1;
        if (!result.isZero() && pdf != 0) r.wo.z *= -1;
    }
    return result;
}

inline float miWeight(float pdfA, float pdfB) {   // path.cpp:296-300
    pdfA *= pdfA;
    pdfB *= pdfB;
    return pdfA / (pdfA + pdfB);
}

// ---------------------------------------------------------------------------
// MIPathTracer::Li (src/integrators/path/path.cpp:119-294)
// ---------------------------------------------------------------------------
struct Integrator {
    int maxDepth, rrDepth;
    bool strictNormals, hideEmitters;
};

enum {
    EEmittedRadiance = 0x0001, EDirectSurfaceRadiance = 0x0004, EIndirectSurfaceRadiance = 0x0008,
    EIntersection = 0x0200, EOpacity = 0x0400
};

// Camera-ray differentials (PerspectiveCamera::sampleRayDifferential scaled
// by 1/sqrt(spp), integrator.cpp:148-149,188); used only by the environment
// lookup of primary rays that leave the scene.
struct RayDiff {
    bool has = false;
    Vec rx, ry;
};

Spec SceneView::reflectance(const mtsg_bsdf &b, const Its &its, const Vec &rayO, const RayDiff *diff) const {
    if (!b.texture) return Spec::of(b.reflectance);
    const mtsg_texture &T = d.textures[b.texture - 1];
    const MipMap M{T.mip, d.tex_texels};
    const float u = its.u * T.uv_scale[0] + T.uv_offset[0], v = its.v * T.uv_scale[1] + T.uv_offset[1];
    Spec value;
    if (diff && diff->has) {
        float dudx, dvdx, dudy, dvdy;
        computePartials(its, rayO, diff->rx, diff->ry, dudx, dvdx, dudy, dvdy);
        value = M.filtered(u, v, dudx * T.uv_scale[0], dvdx * T.uv_scale[1], dudy * T.uv_scale[0], dvdy * T.uv_scale[1]);
    } else {
        value = M.unfiltered(u, v);
    }
    return value * T.scale;
}

template <bool count>
Spec Li(const SceneView &scene, const Integrator &I, Ray ray, Sampler &sampler, float &alpha, int &depthOut, Counters *ctr,
        bool hasAlpha, const RayDiff &diff = RayDiff()) {
    Its its;
    Spec Li(0.0f);
    bool scattered = false;
    int type = EEmittedRadiance | EDirectSurfaceRadiance | EIndirectSurfaceRadiance | EIntersection | (hasAlpha ? EOpacity : 0);
    int depth = 1;
    // RadianceQueryRecord::rayIntersect (records.inl:117-143)
    scene.rayIntersect<count>(ray, its, nullptr, ctr);
    DBG("camera o=(%g %g %g) d=(%g %g %g) mint=%g maxt=%g -> t=%g shape=%d p=(%g %g %g)\n", ray.o.x, ray.o.y, ray.o.z, ray.d.x, ray.d.y, ray.d.z, ray.mint, ray.maxt, its.t, its.shape, its.p.x, its.p.y, its.p.z);
    alpha = 1.0f;
    if (type & EOpacity) alpha = its.valid() ? 1.0f : 0.0f;
    ray.mint = kEpsilon;
    Spec throughput(1.0f);
    float eta = 1.0f;
    while (depth <= I.maxDepth || I.maxDepth < 0) {
        if (!its.valid()) {
            // Scene::evalEnvironment of the (differential) camera ray
            if ((type & EEmittedRadiance) && (!I.hideEmitters || scattered) && scene.d.has_envmap)
                Li += throughput * scene.envEvalEnvironment(ray, diff.has, diff.rx, diff.ry);
            break;
        }
        const mtsg_shape &sh = scene.d.shapes[its.shape];
        const mtsg_bsdf &bsdf = scene.d.bsdfs[sh.bsdf];
        if (sh.emitter >= 0 && (type & EEmittedRadiance) && (!I.hideEmitters || scattered)) {
            // AreaLight::eval (area.cpp:104-109)
            if (dot(its.shFrame.n, -ray.d) > 0) Li += throughput * Spec::of(scene.d.emitters[sh.emitter].radiance);
        }
        if ((depth >= I.maxDepth && I.maxDepth > 0) ||
            (I.strictNormals && dot(ray.d, its.geoFrame.n) * cosTheta(its.wi) >= 0))
            break;

        // the hit's reflectance, with UV partials at the camera ray's hit only
        // (later rays are built without differentials, path.cpp:217)
        // (alb is used before the next rayIntersect overwrites its / ray)
        const RayDiff *hitDiff = depth == 1 ? &diff : nullptr;
        auto alb = [&](const mtsg_bsdf &rec) { return scene.reflectance(rec, its, ray.o, hitDiff); };
        // DirectSamplingRecord dRec(its) (records.inl:160-164)
        SceneView::DRec dRec;
        dRec.ref = its.p;
        dRec.refN = bsdf.ref_n_zero ? Vec(0.0f) : its.shFrame.n;
        if ((type & EDirectSurfaceRadiance) && bsdf.smooth) {
            float s0, s1;
            sampler.next2D(s0, s1);
            Spec value = scene.sampleEmitterDirect<count>(dRec, s0, s1, ctr);
            DBG("  depth %d NEE s=(%g %g) value=(%g %g %g) pdf=%g d=(%g %g %g) dist=%g\n", depth, s0, s1, value.s[0], value.s[1], value.s[2], dRec.pdf, dRec.d.x, dRec.d.y, dRec.d.z, dRec.dist);
            if (!value.isZero()) {
                BRec bRec;
                bRec.wi = its.wi;
                bRec.wo = its.toLocal(dRec.d);
                const Spec bsdfVal = bsdfEvalTS(scene.d.bsdfs, bsdf, bRec, alb);
                if (!bsdfVal.isZero() && (!I.strictNormals || dot(its.geoFrame.n, dRec.d) * cosTheta(bRec.wo) > 0)) {
                    float bsdfPdfV = bsdfPdfTS(scene.d.bsdfs, bsdf, bRec);   // area emitter: on surface, solid angle
                    float weight = miWeight(dRec.pdf, bsdfPdfV);
                    Li += throughput * value * bsdfVal * weight;
                }
            }
        }

        float bsdfPdfS;
        BRec bRec;
        bRec.wi = its.wi;
        float s0, s1;
        sampler.next2D(s0, s1);
        Spec bsdfWeight = bsdfSampleTS(scene.d.bsdfs, bsdf, bRec, bsdfPdfS, s0, s1, [&]() { return sampler.next1D(); }, alb);
        DBG("  depth %d bsdf type=%d s=(%g %g) wi=(%g %g %g) wo=(%g %g %g) w=(%g %g %g) pdf=%g sampled=%d\n", depth, bsdf.type, s0, s1, bRec.wi.x, bRec.wi.y, bRec.wi.z, bRec.wo.x, bRec.wo.y, bRec.wo.z, bsdfWeight.s[0], bsdfWeight.s[1], bsdfWeight.s[2], bsdfPdfS, bRec.sampledType);
        if (bsdfWeight.isZero()) break;
        scattered |= bRec.sampledType != 0;
        const Vec wo = its.toWorld(bRec.wo);
        float woDotGeoN = dot(its.geoFrame.n, wo);
        if (I.strictNormals && woDotGeoN * cosTheta(bRec.wo) <= 0) break;

        bool hitEmitter = false;
        Spec value;
        Ray next;
        next.o = its.p;
        next.setDirection(wo);
        next.mint = kEpsilon;
        next.maxt = std::numeric_limits<float>::infinity();
        ray = next;
        bool hitNext = scene.rayIntersect<count>(ray, its, nullptr, ctr);
        DBG("  trace o=(%g %g %g) d=(%g %g %g) -> hit=%d t=%g shape=%d p=(%g %g %g) n=(%g %g %g)\n", ray.o.x, ray.o.y, ray.o.z, ray.d.x, ray.d.y, ray.d.z, (int)hitNext, its.t, its.shape, its.p.x, its.p.y, its.p.z, its.shFrame.n.x, its.shFrame.n.y, its.shFrame.n.z);
        if (hitNext) {
            const mtsg_shape &hs = scene.d.shapes[its.shape];
            if (hs.emitter >= 0) {
                value = dot(its.shFrame.n, -ray.d) > 0 ? Spec::of(scene.d.emitters[hs.emitter].radiance) : Spec(0.0f);
                // dRec.setQuery(ray, its) (records.inl:170-176)
                dRec.p = its.p;
                dRec.n = its.shFrame.n;
                dRec.measureSolidAngle = 1;
                dRec.emitter = hs.emitter;
                dRec.d = ray.d;
                dRec.dist = its.t;
                hitEmitter = true;
            }
        } else if (scene.d.has_envmap) {
            if (I.hideEmitters && !scattered) break;
            value = scene.envEvalEnvironment(ray, false, Vec(0.0f), Vec(0.0f));
            // EnvironmentMap::fillDirectSamplingRecord (envmap.cpp:358-374)
            float nearT, farT;
            if (!scene.envSphere(ray.o, ray.d, nearT, farT) || nearT > 0 || farT < 0) break;
            dRec.p = ray.o + ray.d * farT;
            dRec.n = normalize(Vec(scene.d.envmap.bsphere_center[0], scene.d.envmap.bsphere_center[1],
                                   scene.d.envmap.bsphere_center[2]) - dRec.p);
            dRec.measureSolidAngle = 1;
            dRec.emitter = scene.d.envmap.emitter;
            dRec.d = ray.d;
            dRec.dist = farT;
            hitEmitter = true;
        } else {
            break;
        }
        throughput *= bsdfWeight;
        eta *= bRec.eta;
        if (hitEmitter && (type & EDirectSurfaceRadiance)) {
            const float lumPdf = !(bRec.sampledType & (EDeltaReflection | EDeltaTransmission)) ? scene.pdfEmitterDirect(dRec) : 0;
            Li += throughput * value * miWeight(bsdfPdfS, lumPdf);
        }
        if (!its.valid() || !(type & EIndirectSurfaceRadiance)) break;
        type = type & ~EEmittedRadiance & ~EOpacity;
        if (depth++ >= I.rrDepth) {
            float q = std::min(throughput.max() * eta * eta, 0.95f);
            if (sampler.next1D() >= q) break;
            throughput = throughput / q;
        }
    }
    depthOut = depth;
    DBG("  -> L=(%g %g %g) depth=%d\n", Li.s[0], Li.s[1], Li.s[2], depth);
    return Li;
}


// ---------------------------------------------------------------------------
// myPath2_OM (src/integrators/testOM/myPath2_OM.cpp:317-485) and the
// occupancy-map visibility it uses instead of shadow rays (myOM.h)
// ---------------------------------------------------------------------------
// OccupancyMap::nearestOMindex / direct2uv (myOM.h:603-615, helpers.h:6-44):
// flips d in place when d.z < 0, as the reference does
int omNearestIndex(Vec &d) {
    if (d.z < 0) d = -d;
    const float r = std::sqrt(1 - d.z);
    float phi = std::atan2(d.y, d.x);
    float u, v;
    if (r == 0) {
        u = 0;
        v = 0;
    } else {
        float a, b;
        if (phi < -M_PI / 4) phi += 2 * M_PI;
        if (phi < M_PI / 4) {
            a = r;
            b = phi * a / (M_PI / 4);
        } else if (phi < M_PI * 3 / 4) {
            b = r;
            a = -(phi - M_PI / 2) * b / (M_PI / 4);
        } else if (phi < M_PI * 5 / 4) {
            a = -r;
            b = (phi - M_PI) * a / (M_PI / 4);
        } else {
            b = -r;
            a = -(phi - M_PI * 3 / 2) * b / (M_PI / 4);
        }
        u = (a + 1) / 2;
        v = (b + 1) / 2;
    }
    if (u > 0.999999) u = 0.999999;
    if (v > 0.999999) v = 0.999999;
    return int(std::floor(u * MTSG_OM_SQRT)) * MTSG_OM_SQRT + int(std::floor(v * MTSG_OM_SQRT));
}

// OccupancyMap::Visible (myOM.h:383-503, 32-bit column path); x or y == 256
// (an out-of-range read in the reference) counts as visible
bool omVisible(const mtsg_scene_desc &d, int id, const Vec &o1, const Vec &o2) {
    const mtsg_om &O = *d.om;
    const Vec dir(O.dir[id][0], O.dir[id][1], O.dir[id][2]);
    const Vec o21 = o2 - o1;
    float length = std::sqrt(o21.x * o21.x + o21.y * o21.y + o21.z * o21.z);
    if (dot(dir, o21) < 0) length = -length;
    const float *m = O.rotate[id];
    const Vec c(O.center[0], O.center[1], O.center[2]);
    const Vec q = o1 - c;
    const Vec a1 = Vec(m[0] * q.x + m[1] * q.y + m[2] * q.z + 0.0f, m[3] * q.x + m[4] * q.y + m[5] * q.z + 0.0f,
                       m[6] * q.x + m[7] * q.y + m[8] * q.z + 0.0f) + c;
    const Vec a2 = a1 + dir * length;
    const float rc = O.grid_size_recp;
    const int x = (int)std::floor((a1.x - O.aabb_min[0]) * rc + kEpsilon), y = (int)std::floor((a1.y - O.aabb_min[1]) * rc + kEpsilon);
    if (x < 0 || x >= MTSG_OM_SIZE || y < 0 || y >= MTSG_OM_SIZE) return true;
    int z1 = (int)std::floor((a1.z - O.aabb_min[2]) * rc + kEpsilon), z2 = (int)std::floor((a2.z - O.aabb_min[2]) * rc + kEpsilon);
    if (z1 > z2) std::swap(z1, z2);
    if (z2 - z1 < 2) return true;
    z1 += 1;
    z2 -= 1;
    z1 = std::min(std::max(z1, 0), MTSG_OM_SIZE - 1);
    z2 = std::min(std::max(z2, 0), MTSG_OM_SIZE - 1);
    const uint32_t *col = d.om_bits + (((size_t)id * MTSG_OM_SIZE + x) * MTSG_OM_SIZE + y) * (MTSG_OM_SIZE / 32);
    const int p1 = z1 >> 5, p2 = z2 >> 5, r1 = z1 & 31, r2 = (31 - z2) & 31;
    if (p1 == p2) return ((col[p1] >> r1) << (r1 + r2)) == 0;
    if (col[p1] >> r1) return false;
    for (int i = p1 + 1; i < p2; ++i)
        if (col[i]) return false;
    return (col[p2] << r2) == 0;
}

struct OMParams { int maxDepthEye, strategy, mis; };

float omMis(const OMParams &P, float p1, float p2) {   // myPath2_OM.cpp:301-314
    if (P.mis == MTSG_OM_MIS_UNIFORM) return 0.5f;
    if (P.mis == MTSG_OM_MIS_BALANCE) return p1 / (p1 + p2);
    return (p1 * p1) / ((p1 * p1) + (p2 * p2));
}
// misWeight (myPath2_OM.cpp:270-299): which = 0 for the BSDF strategy, 1 for NEE
float omMisWeight(const OMParams &P, float pdfBSDF, float pdfDirect, int which) {
    if (which == 0) {
        if (P.strategy == MTSG_OM_STRATEGY_BSDF) return 1;
        if (P.strategy == MTSG_OM_STRATEGY_NEE) return 0;
        return omMis(P, pdfBSDF, pdfDirect);
    }
    if (P.strategy == MTSG_OM_STRATEGY_BSDF) return 0;
    if (P.strategy == MTSG_OM_STRATEGY_NEE) return 1;
    return omMis(P, pdfDirect, pdfBSDF);
}

// myPath2OMIntegrator::Li (myPath2_OM.cpp:386-485)
Spec LiOM(const SceneView &scene, const OMParams &P, Ray ray, Sampler &sampler) {
    Its its;
    Spec Li(0.0f), throughput(1.0f);
    float eta = 1.0f;
    scene.rayIntersect<false>(ray, its, nullptr, nullptr);
    ray.mint = kEpsilon;
    if (its.valid() && scene.d.shapes[its.shape].emitter >= 0) {   // its.Le(-ray.d)
        if (dot(its.shFrame.n, -ray.d) > 0) return Spec::of(scene.d.emitters[scene.d.shapes[its.shape].emitter].radiance);
        return Spec(0.0f);
    }
    int depth = 1;
    while (depth <= P.maxDepthEye) {
        if (!its.valid()) break;
        const mtsg_bsdf &bsdf = scene.d.bsdfs[scene.d.shapes[its.shape].bsdf];
        auto alb = [&](const mtsg_bsdf &rec) { return scene.reflectance(rec, its, ray.o, nullptr); };   // sampleRay: no differentials
        SceneView::DRec dRec;
        dRec.ref = its.p;
        dRec.refN = bsdf.ref_n_zero ? Vec(0.0f) : its.shFrame.n;
        if (bsdf.smooth) {
            float s0, s1;
            sampler.next2D(s0, s1);
            const Spec value = scene.sampleEmitterDirect<false>(dRec, s0, s1, nullptr, false);
            const int id = omNearestIndex(dRec.d);   // (twice in the reference, same answer)
            const bool vis = omVisible(scene.d, id, its.p + its.shFrame.n * 0.5f, dRec.p);
            if (vis && !value.isZero()) {
                BRec bRec;
                bRec.wi = its.wi;
                bRec.wo = its.toLocal(dRec.d);   // the possibly flipped direction
                const Spec bsdfVal = bsdfEvalTS(scene.d.bsdfs, bsdf, bRec, alb);
                if (!bsdfVal.isZero()) {
                    const bool onSurface = scene.d.emitters[dRec.emitter].type != MTSG_EMITTER_ENVMAP;
                    const float bsdfPdf = onSurface ? bsdfPdfTS(scene.d.bsdfs, bsdf, bRec) : 0.0f;
                    Li += throughput * value * bsdfVal * omMisWeight(P, bsdfPdf, dRec.pdf, 1);
                }
            }
        }
        float bsdfPdf;
        BRec bRec;
        bRec.wi = its.wi;
        float s0, s1;
        sampler.next2D(s0, s1);
        const Spec bsdfWeight = bsdfSampleTS(scene.d.bsdfs, bsdf, bRec, bsdfPdf, s0, s1, [&]() { return sampler.next1D(); }, alb);
        if (bsdfWeight.isZero()) break;
        const Vec wo = its.toWorld(bRec.wo);
        throughput *= bsdfWeight;
        eta *= bRec.eta;
        Ray next;
        next.o = its.p;
        next.setDirection(wo);
        next.mint = kEpsilon;
        next.maxt = std::numeric_limits<float>::infinity();
        ray = next;
        if (scene.rayIntersect<false>(ray, its, nullptr, nullptr)) {
            const int em = scene.d.shapes[its.shape].emitter;
            if (em >= 0) {
                const Spec value = dot(its.shFrame.n, -ray.d) > 0 ? Spec::of(scene.d.emitters[em].radiance) : Spec(0.0f);
                dRec.p = its.p;   // dRec.setQuery(ray, its) (records.inl:170-176)
                dRec.n = its.shFrame.n;
                dRec.emitter = em;
                dRec.d = ray.d;
                dRec.dist = its.t;
                const float lumPdf = !(bRec.sampledType & (EDeltaReflection | EDeltaTransmission)) ? scene.pdfEmitterDirect(dRec) : 0;
                Li += throughput * value * omMisWeight(P, bsdfPdf, lumPdf, 0);
                return Li;
            }
        }
        const float q = std::min(throughput.max() * eta * eta, 0.95f);
        if (sampler.next1D() >= q) break;
        throughput = throughput / q;
        ++depth;
    }
    return Li;
}

// PerspectiveCamera::sampleRayDifferential (perspective.cpp:271-298)
Ray cameraRay(const mtsg_camera &c, float px, float py, RayDiff *diff = nullptr, uint32_t spp = 1) {
    const float *m = c.sample_to_camera;
    float sx = px * c.inv_res_x, sy = py * c.inv_res_y;
    float x = m[0] * sx + m[1] * sy + m[3];
    float y = m[4] * sx + m[5] * sy + m[7];
    float z = m[8] * sx + m[9] * sy + m[11];
    float w = m[12] * sx + m[13] * sy + m[15];
    Vec nearP = w == 1.0f ? Vec(x, y, z) : Vec(x, y, z) / w;
    Vec d = normalize(nearP);
    float invZ = 1.0f / d.z;
    Ray ray;
    ray.mint = c.near_clip * invZ;
    ray.maxt = c.far_clip * invZ;
    const float *t = c.camera_to_world;
    ray.o = Vec(t[3], t[7], t[11]);
    ray.setDirection(Vec(t[0] * d.x + t[1] * d.y + t[2] * d.z, t[4] * d.x + t[5] * d.y + t[6] * d.z, t[8] * d.x + t[9] * d.y + t[10] * d.z));
    if (diff) {
        auto toWorld = [&](const Vec &v) {
            return Vec(t[0] * v.x + t[1] * v.y + t[2] * v.z, t[4] * v.x + t[5] * v.y + t[6] * v.z, t[8] * v.x + t[9] * v.y + t[10] * v.z);
        };
        const Vec rx = toWorld(normalize(nearP + Vec(c.dx[0], c.dx[1], c.dx[2])));
        const Vec ry = toWorld(normalize(nearP + Vec(c.dy[0], c.dy[1], c.dy[2])));
        const float scale = 1.0f / std::sqrt((float)spp);   // RayDifferential::scaleDifferential
        diff->has = true;
        diff->rx = ray.d + (rx - ray.d) * scale;
        diff->ry = ray.d + (ry - ray.d) * scale;
    }
    return ray;
}

// ImageBlock::put (imageblock.h:124-204) into a tile+border block
struct Block {
    int ox, oy, w, h, border;   // offset of the tile, tile size
    float *data;                // (w+2b)*(h+2b)*5
    const mtsg_camera *cam;
    bool put(float spx, float spy, const Spec &spec, float alpha) {
        float value[5] = {spec.s[0], spec.s[1], spec.s[2], alpha, 1.0f};
        for (int i = 0; i < 5; ++i)
            if (!std::isfinite(value[i]) || value[i] < 0) return false;
        const float r = cam->filter_radius;
        const int W = w + 2 * border, H = h + 2 * border;
        const float px = spx - 0.5f - (float)(ox - border), py = spy - 0.5f - (float)(oy - border);
        int minx = std::max((int)std::ceil(px - r), 0), miny = std::max((int)std::ceil(py - r), 0);
        int maxx = std::min((int)std::floor(px + r), W - 1), maxy = std::min((int)std::floor(py + r), H - 1);
        float wx[8], wy[8];
        auto disc = [&](float x) { return cam->filter_values[std::min((int)std::abs(x * cam->filter_scale), 31)]; };
        for (int x = minx, i = 0; x <= maxx && i < 8; ++x, ++i) wx[i] = disc((float)x - px);
        for (int y = miny, i = 0; y <= maxy && i < 8; ++y, ++i) wy[i] = disc((float)y - py);
        for (int y = miny, yr = 0; y <= maxy; ++y, ++yr) {
            float *dst = data + ((size_t)y * W + minx) * 5;
            for (int x = minx, xr = 0; x <= maxx; ++x, ++xr) {
                float weight = wx[xr] * wy[yr];
                for (int k = 0; k < 5; ++k) *dst++ += weight * value[k];
            }
        }
        return true;
    }
};

int hwThreads(int t) { return t > 0 ? t : std::max(1u, std::thread::hardware_concurrency()); }

}  // namespace

namespace {
Ray rayFrom(const float *r) {
    Ray ray;
    ray.o = Vec(r[0], r[1], r[2]);
    ray.setDirection(Vec(r[3], r[4], r[5]));
    ray.mint = r[6];
    ray.maxt = r[7];
    return ray;
}

template <class F>
void parallelFor(uint32_t n, int threads, F f) {
    int T = std::min<int>(hwThreads(threads), (int)std::max<uint32_t>(1, n / 1024 + 1));
    std::vector<std::thread> pool;
    std::atomic<uint32_t> next{0};
    for (int t = 0; t < T; ++t)
        pool.emplace_back([&]() {
            for (;;) {
                uint32_t b = next.fetch_add(1024);
                if (b >= n) break;
                uint32_t e = std::min(n, b + 1024);
                for (uint32_t i = b; i < e; ++i) f(i);
            }
        });
    for (auto &th : pool) th.join();
}

}  // namespace

// ===========================================================================
// C API
// ===========================================================================
struct oracle_sfmt { Sfmt s; };

extern "C" {

oracle_sfmt *oracle_sfmt_new(uint64_t seed) {
    auto *r = new oracle_sfmt;
    r->s.initGenRand(seed);
    return r;
}
oracle_sfmt *oracle_sfmt_clone(oracle_sfmt *parent) {
    auto *r = new oracle_sfmt;
    r->s.seedFrom(parent->s);
    return r;
}
uint64_t oracle_sfmt_next_ulong(oracle_sfmt *r) { return r->s.nextULong(); }
float oracle_sfmt_next_float(oracle_sfmt *r) { return r->s.nextFloat(); }
void oracle_sfmt_free(oracle_sfmt *r) { delete r; }

float oracle_counter_float(uint32_t seed, uint64_t sample_id, uint32_t dim) {
    return counterFloat(counterKey(seed, sample_id), dim);
}

const char *oracle_last_error(void) { return g_err.c_str(); }

int oracle_trace_closest(const mtsg_scene_desc *d, uint32_t n, const float *rays, float *t, float *u, float *v,
                         uint32_t *prim, int threads) {
    SceneView sv(*d);
    parallelFor(n, threads, [&](uint32_t i) {
        Ray ray = rayFrom(rays + 8 * i);
        Its its;
        Cache c;
        Counters dummy;
        if (sv.rayIntersect<false>(ray, its, &c, &dummy)) {
            t[i] = its.t;
            if (c.primIndex != 0xFFFFFFFFu) { u[i] = c.u; v[i] = c.v; prim[i] = c.primIndex; }
            else { u[i] = c.rx; v[i] = c.ry; prim[i] = 0x80000000u | d->shapes[c.shapeIndex].rect; }
        } else {
            t[i] = std::numeric_limits<float>::infinity();
            u[i] = v[i] = 0;
            prim[i] = 0xFFFFFFFFu;
        }
    });
    return 0;
}

int oracle_trace_shadow(const mtsg_scene_desc *d, uint32_t n, const float *rays, uint8_t *occ, int threads) {
    SceneView sv(*d);
    parallelFor(n, threads, [&](uint32_t i) {
        Counters dummy;
        occ[i] = sv.rayIntersectShadow<false>(rayFrom(rays + 8 * i), &dummy) ? 1 : 0;
    });
    return 0;
}

int oracle_trace_closest_brute(const mtsg_scene_desc *d, uint32_t n, const float *rays, float *t, uint32_t *prim) {
    SceneView sv(*d);
    // triangles of shape groups are only reachable through their instances
    std::vector<uint8_t> grouped(d->n_prims, 0);
    std::vector<std::vector<uint32_t>> groupPrims(d->n_groups);
    for (uint32_t g = 0; g < d->n_groups; ++g) {
        const mtsg_group &G = d->groups[g];
        for (uint32_t i = 0; i < G.n_indices; ++i) {
            const uint32_t p = d->group_indices[G.index_offset + i];
            if (!grouped[p]) groupPrims[g].push_back(p);
            grouped[p] = 1;
        }
    }
    parallelFor(n, 0, [&](uint32_t i) {
        Ray ray = rayFrom(rays + 8 * i);
        float mint, maxt;
        t[i] = std::numeric_limits<float>::infinity();
        prim[i] = 0xFFFFFFFFu;
        if (!sv.aabbIntersect(ray, mint, maxt)) return;
        float rayMinT = ray.mint;
        if (rayMinT == kEpsilon)
            rayMinT *= std::max(std::max(std::max(std::abs(ray.o.x), std::abs(ray.o.y)), std::abs(ray.o.z)), kEpsilon);
        if (rayMinT > mint) mint = rayMinT;
        if (ray.maxt < maxt) maxt = ray.maxt;
        if (!(maxt > mint)) return;
        for (uint32_t p = 0; p < d->n_prims; ++p) {
            if (grouped[p]) continue;
            const mtsg_triaccel &ta = d->triaccel[p];
            if (ta.k == MTSG_TRIACCEL_SHAPE && d->shapes[ta.shape_index].type == MTSG_SHAPE_INSTANCE) {
                // every primitive of the group with the instance-space ray
                const Ray lr = sv.toInstance(ray, d->instances[ta.prim_index]);
                for (uint32_t q : groupPrims[d->instances[ta.prim_index].group]) {
                    float tt;
                    Cache c;
                    if (sv.primIntersect(lr, q, mint, maxt, tt, &c)) {
                        maxt = tt;
                        t[i] = tt;
                        prim[i] = c.primIndex;
                    }
                }
                continue;
            }
            float tt;
            Cache c;
            if (sv.primIntersect(ray, p, mint, maxt, tt, &c)) {
                maxt = tt;
                t[i] = tt;
                prim[i] = c.primIndex != 0xFFFFFFFFu ? c.primIndex : (0x80000000u | d->triaccel[p].prim_index);
            }
        }
    });
    return 0;
}

int oracle_debug_path_rays(const mtsg_scene_desc *d, const mtsg_render_params *p, int x, int y, int s,
                           float *rays_out, int max_rays) {
    std::vector<float> log;
    g_rayLog = &log;
    SceneView sv(*d);
    Integrator I{p->max_depth, p->rr_depth, p->strict_normals != 0, p->hide_emitters != 0};
    Qmc qmc(*d, p->spp);
    Sampler smp;
    smp.mode = ORACLE_RNG_COUNTER;
    smp.begin(&qmc, p->seed, d->camera.film_w, p->spp, x, y, (uint32_t)s);
    float a, b;
    smp.next2D(a, b);
    RayDiff diff;
    Ray ray = cameraRay(d->camera, x + a, y + b, &diff, p->spp);
    float alpha;
    int depth;
    Counters c;
    Li<false>(sv, I, ray, smp, alpha, depth, &c, d->camera.has_alpha != 0, diff);
    g_rayLog = nullptr;
    int n = std::min<int>((int)log.size() / 8, max_rays);
    std::copy(log.begin(), log.begin() + 8 * n, rays_out);
    return n;
}

int oracle_debug_pixel_sample(const mtsg_scene_desc *d, const mtsg_render_params *p, int x, int y, int s) {
    std::vector<float> out(3 * p->spp);
    g_debug = 1;
    mtsg_render_params q = *p;
    SceneView sv(*d);
    Integrator I{p->max_depth, p->rr_depth, p->strict_normals != 0, p->hide_emitters != 0};
    Qmc qmc(*d, p->spp);
    Sampler smp;
    smp.mode = ORACLE_RNG_COUNTER;
    smp.begin(&qmc, p->seed, d->camera.film_w, p->spp, x, y, (uint32_t)s);
    float a, b;
    smp.next2D(a, b);
    RayDiff diff;
    Ray ray = cameraRay(d->camera, x + a, y + b, &diff, p->spp);
    float alpha;
    int depth;
    Counters c;
    Li<false>(sv, I, ray, smp, alpha, depth, &c, d->camera.has_alpha != 0, diff);
    g_debug = 0;
    (void)q;
    return 0;
}

int oracle_sampler_draws(const mtsg_scene_desc *d, const mtsg_render_params *p, int x, int y, uint32_t s,
                         uint32_t n, const int32_t *kinds, float *out) try {
    Qmc qmc(*d, p->spp);
    Sampler smp;
    smp.mode = ORACLE_RNG_COUNTER;
    smp.begin(&qmc, p->seed, d->camera.film_w, p->spp, x, y, s);
    for (uint32_t i = 0; i < n; ++i) {
        if (kinds[i] == 2) {
            smp.next2D(out[0], out[1]);
            out += 2;
        } else {
            *out++ = smp.next1D();
        }
    }
    return 0;
} catch (const std::exception &e) {
    g_err = e.what();
    return -1;
}

int oracle_pixel_samples(const mtsg_scene_desc *d, const mtsg_render_params *p, int x, int y, float *out) try {
    SceneView sv(*d);
    Integrator I{p->max_depth, p->rr_depth, p->strict_normals != 0, p->hide_emitters != 0};
    Qmc qmc(*d, p->spp);
    for (uint32_t s = 0; s < p->spp; ++s) {
        Sampler smp;
        smp.mode = ORACLE_RNG_COUNTER;
        smp.begin(&qmc, p->seed, d->camera.film_w, p->spp, x, y, s);
        float a, b;
        smp.next2D(a, b);
        RayDiff diff;
    Ray ray = cameraRay(d->camera, x + a, y + b, &diff, p->spp);
        float alpha;
        int depth;
        Counters c;
        Spec L = Li<false>(sv, I, ray, smp, alpha, depth, &c, d->camera.has_alpha != 0, diff);
        out[3 * s] = L.s[0]; out[3 * s + 1] = L.s[1]; out[3 * s + 2] = L.s[2];
    }
    return 0;
} catch (const std::exception &e) {
    g_err = e.what();
    return -1;
}

int oracle_render(const mtsg_scene_desc *d, const mtsg_render_params *p, int rng_mode, int threads, float *rgbaw,
                  oracle_stats *stats) {
    try {
        const mtsg_camera &cam = d->camera;
        const int B = cam.border;
        const int W = p->tile_w + 2 * B, H = p->tile_h + 2 * B;
        std::fill(rgbaw, rgbaw + (size_t)W * H * 5, 0.0f);
        SceneView sv(*d);
        Integrator I{p->max_depth, p->rr_depth, p->strict_normals != 0, p->hide_emitters != 0};
        const OMParams omp{p->max_depth, p->om_strategy, p->om_mis};
        if (p->integrator == MTSG_INTEGRATOR_PATH2_OM && !d->om) throw std::runtime_error("myPath2_OM: the scene has no occupancy maps");
        int T = hwThreads(threads);
        const int BS = 32;   // scene.cpp:27 block size
        int nbx = (p->tile_w + BS - 1) / BS, nby = (p->tile_h + BS - 1) / BS;
        // BlockedImageProcess spiral order (imageproc.cpp:28-78)
        std::vector<std::pair<int, int>> blocks;
        {
            int cx = nbx / 2, cy = nby / 2, dir = 0, stepsLeft = 1, numSteps = 1;
            int total = nbx * nby;
            while ((int)blocks.size() < total) {
                if (cx >= 0 && cy >= 0 && cx < nbx && cy < nby) blocks.emplace_back(cx, cy);
                if ((int)blocks.size() == total) break;
                switch (dir) { case 0: ++cx; break; case 1: ++cy; break; case 2: --cx; break; default: --cy; }
                if (--stepsLeft == 0) {
                    dir = (dir + 1) % 4;
                    if (dir == 0 || dir == 2) ++numSteps;
                    stepsLeft = numSteps;
                }
            }
        }
        Sfmt parent;
        parent.initGenRand(5489ULL + p->seed);   // seed 0: Mitsuba's default (random.cpp:486); others: independent streams for the tests
        std::vector<Sfmt> clones(T);
        for (int t = 0; t < T; ++t) clones[t].seedFrom(parent);   // renderjob.cpp:57-69

        std::atomic<size_t> nextBlock{0};
        std::mutex filmMutex;
        std::vector<Counters> ctrs(T);
        std::vector<uint64_t> pathVerts(T, 0), samples(T, 0);
        auto t0 = std::chrono::steady_clock::now();
        const Qmc qmc(*d, p->spp);
        auto worker = [&](int tid) {
            Sampler smp;
            smp.mode = rng_mode;
            smp.sfmt = &clones[tid];
            std::vector<float> local;
            for (;;) {
                size_t bi = nextBlock.fetch_add(1);
                if (bi >= blocks.size()) break;
                int bx0 = p->tile_x + blocks[bi].first * BS, by0 = p->tile_y + blocks[bi].second * BS;
                int bw = std::min(BS, p->tile_x + p->tile_w - bx0), bh = std::min(BS, p->tile_y + p->tile_h - by0);
                local.assign((size_t)(bw + 2 * B) * (bh + 2 * B) * 5, 0.0f);
                Block blk{bx0, by0, bw, bh, B, local.data(), &cam};
                const int tilesX = (p->tile_w + 15) / 16;
                for (int y = by0; y < by0 + bh; ++y)
                    for (int x = bx0; x < bx0 + bw; ++x) {
                        // multi-GPU contract (mtsg_render_params.tile_stride): this
                        // call owns the 16x16 tiles t of the rectangle with
                        // deal key % tile_stride == tile_offset, the key of tile
                        // (tx, ty) being ty * tilesX + (tx - ty) mod tilesX
                        if (p->tile_stride > 1) {
                            const int ty = (y - p->tile_y) / 16, tx = (x - p->tile_x) / 16;
                            const int key = ty * tilesX + ((tx - ty % tilesX) % tilesX + tilesX) % tilesX;
                            if (key % p->tile_stride != p->tile_offset) continue;
                        }
                        for (uint32_t s = 0; s < p->spp; ++s) {
                            smp.begin(&qmc, p->seed, cam.film_w, p->spp, x, y, s);
                            if (p->integrator == MTSG_INTEGRATOR_PATH2_OM) {
                                // myPath2_OM.cpp:243-256: jittered (or centred) sample, sensor->sampleRay
                                float a = 0.5f, b = 0.5f;
                                if (p->om_jitter) smp.next2D(a, b);
                                const float spx = x + a, spy = y + b;
                                const Spec L = LiOM(sv, omp, cameraRay(cam, spx, spy), smp);
                                samples[tid]++;
                                blk.put(spx, spy, L, 1.0f);
                                continue;
                            }
                            float a, b;
                            smp.next2D(a, b);
                            float spx = x + a, spy = y + b;
                            RayDiff diff;
                            Ray ray = cameraRay(cam, spx, spy, &diff, p->spp);
                            float alpha;
                            int depth;
                            Spec L = stats && (stats->threads < 0)
                                         ? Li<true>(sv, I, ray, smp, alpha, depth, &ctrs[tid], cam.has_alpha != 0, diff)
                                         : Li<false>(sv, I, ray, smp, alpha, depth, &ctrs[tid], cam.has_alpha != 0, diff);
                            pathVerts[tid] += depth;
                            samples[tid]++;
                            blk.put(spx, spy, L, alpha);
                        }
                    }
                // BlockedRenderProcess::processResult -> Film::put (renderproc.cpp:142-149)
                std::lock_guard<std::mutex> g(filmMutex);
                for (int yy = 0; yy < bh + 2 * B; ++yy) {
                    int fy = by0 - p->tile_y + yy;   // row in the tile block (border-relative)
                    int fx0 = bx0 - p->tile_x;
                    float *dst = rgbaw + ((size_t)fy * W + fx0) * 5;
                    const float *src = local.data() + (size_t)yy * (bw + 2 * B) * 5;
                    for (int k = 0; k < (bw + 2 * B) * 5; ++k) dst[k] += src[k];
                }
            }
        };
        std::vector<std::thread> pool;
        std::mutex errMutex;
        std::string workerErr;
        auto guarded = [&](int tid) {
            try {
                worker(tid);
            } catch (const std::exception &e) {   // e.g. the QMC dimension limit
                std::lock_guard<std::mutex> lk(errMutex);
                workerErr = e.what();
                nextBlock.store(blocks.size() + (size_t)T);
            }
        };
        for (int t = 0; t < T; ++t) pool.emplace_back(guarded, t);
        for (auto &th : pool) th.join();
        if (!workerErr.empty()) throw std::runtime_error(workerErr);
        double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (stats) {
            bool counting = stats->threads < 0;
            memset(stats, 0, sizeof(*stats));
            stats->seconds = secs;
            stats->threads = T;
            for (int t = 0; t < T; ++t) {
                stats->samples += samples[t];
                stats->path_vertices += pathVerts[t];
                if (counting) {
                    stats->rays_closest += ctrs[t].closest;
                    stats->rays_shadow += ctrs[t].shadow;
                    stats->nodes_visited += ctrs[t].nodes;
                    stats->leaf_refs += ctrs[t].refs;
                    stats->tri_tests += ctrs[t].tests;
                }
            }
        }
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

int oracle_bsdf_sample(const mtsg_bsdf *b, const float wi[3], float s0, float s1, float wo[3], float *pdf, float weight[3]) {
    return oracle_bsdf_sample3(b, wi, s0, s1, 0.5f, wo, pdf, weight);
}

int oracle_bsdf_sample3(const mtsg_bsdf *b, const float wi[3], float s0, float s1, float s2, float wo[3], float *pdf,
                        float weight[3]) {
    BRec r;
    r.wi = Vec(wi[0], wi[1], wi[2]);
    float p = 0;
    Spec w = bsdfSample(*b, Spec::of(b->reflectance), r, p, s0, s1, [&]() { return s2; });
    wo[0] = r.wo.x; wo[1] = r.wo.y; wo[2] = r.wo.z;
    *pdf = p;
    weight[0] = w.s[0]; weight[1] = w.s[1]; weight[2] = w.s[2];
    return r.sampledType;
}

int oracle_bsdf_eval(const mtsg_bsdf *b, const float wi[3], const float wo[3], float value[3], float *pdf) {
    BRec r;
    r.wi = Vec(wi[0], wi[1], wi[2]);
    r.wo = Vec(wo[0], wo[1], wo[2]);
    Spec v = bsdfEval(*b, Spec::of(b->reflectance), r);
    value[0] = v.s[0]; value[1] = v.s[1]; value[2] = v.s[2];
    *pdf = bsdfPdf(*b, r);
    return 0;
}

int oracle_bsdf_sample_n(const mtsg_bsdf *b, const float wi[3], uint32_t n, const float *u2, float *wo, float *pdf,
                         float *weight, int32_t *type) {
    for (uint32_t i = 0; i < n; ++i)
        type[i] = oracle_bsdf_sample(b, wi, u2[2 * i], u2[2 * i + 1], wo + 3 * i, pdf + i, weight + 3 * i);
    return 0;
}

int oracle_bsdf_sample3_n(const mtsg_bsdf *b, const float wi[3], uint32_t n, const float *u3, float *wo, float *pdf,
                          float *weight, int32_t *type) {
    for (uint32_t i = 0; i < n; ++i)
        type[i] = oracle_bsdf_sample3(b, wi, u3[3 * i], u3[3 * i + 1], u3[3 * i + 2], wo + 3 * i, pdf + i, weight + 3 * i);
    return 0;
}

int oracle_bsdf_eval_n(const mtsg_bsdf *b, const float wi[3], uint32_t n, const float *wo, float *value, float *pdf) {
    for (uint32_t i = 0; i < n; ++i) oracle_bsdf_eval(b, wi, wo + 3 * i, value + 3 * i, pdf + i);
    return 0;
}

// EnvironmentMap::sampleDirect / pdfDirect from a reference point (the
// EmitterAdapter of src/tests/test_chisquare.cpp:342-388)
int oracle_env_sample_direct_n(const mtsg_scene_desc *d, uint32_t n, const float *u2, const float ref[3], float *dir,
                               float *pdf, float *value) {
    if (!d || !d->has_envmap) { g_err = "scene has no environment emitter"; return -1; }
    SceneView sv(*d);
    for (uint32_t i = 0; i < n; ++i) {
        SceneView::DRec dRec;
        dRec.ref = Vec(ref[0], ref[1], ref[2]);
        Spec v = sv.envSampleDirect(dRec, u2[2 * i], u2[2 * i + 1]);
        dir[3 * i] = dRec.d.x; dir[3 * i + 1] = dRec.d.y; dir[3 * i + 2] = dRec.d.z;
        pdf[i] = dRec.pdf;
        value[3 * i] = v.s[0]; value[3 * i + 1] = v.s[1]; value[3 * i + 2] = v.s[2];
    }
    return 0;
}

int oracle_env_pdf_direct_n(const mtsg_scene_desc *d, uint32_t n, const float *dir, float *pdf) {
    if (!d || !d->has_envmap) { g_err = "scene has no environment emitter"; return -1; }
    SceneView sv(*d);
    for (uint32_t i = 0; i < n; ++i) pdf[i] = sv.envInternalPdf(sv.envToLocal(Vec(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2])));
    return 0;
}

/* Environment radiance along world directions (no differentials: bilinear
 * level 0) and with camera-style differentials (EWA). */
int oracle_env_eval_n(const mtsg_scene_desc *d, uint32_t n, const float *dir, const float *rx, const float *ry, float *out) {
    if (!d || !d->has_envmap) { g_err = "scene has no environment emitter"; return -1; }
    SceneView sv(*d);
    for (uint32_t i = 0; i < n; ++i) {
        Ray r;
        r.o = Vec(0.0f);
        r.setDirection(Vec(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]));
        const bool diff = rx && ry;
        const Spec v = sv.envEvalEnvironment(r, diff, diff ? Vec(rx[3 * i], rx[3 * i + 1], rx[3 * i + 2]) : Vec(0.0f),
                                             diff ? Vec(ry[3 * i], ry[3 * i + 1], ry[3 * i + 2]) : Vec(0.0f));
        out[3 * i] = v.s[0]; out[3 * i + 1] = v.s[1]; out[3 * i + 2] = v.s[2];
    }
    return 0;
}

/* myPath2_OM's visibility query (nearestOMindex + Visible), as mtsg_om_query */
int oracle_om_query_n(const mtsg_scene_desc *d, uint32_t n, const float *dirs, const float *o1, const float *o2, int32_t *ids,
                      int32_t *vis) {
    if (!d || !d->om) { g_err = "scene has no occupancy maps"; return -1; }
    for (uint32_t i = 0; i < n; ++i) {
        Vec dd(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
        ids[i] = omNearestIndex(dd);
        vis[i] = omVisible(*d, ids[i], Vec(o1[3 * i], o1[3 * i + 1], o1[3 * i + 2]), Vec(o2[3 * i], o2[3 * i + 1], o2[3 * i + 2])) ? 1 : 0;
    }
    return 0;
}

/* BitmapTexture::eval(uv) / eval(uv, d0, d1) (bitmap.cpp:431-499) of texture
 * `tex`: the MIP-level lookup the device's mtsg_tex_eval answers */
int oracle_tex_eval_n(const mtsg_scene_desc *d, int tex, uint32_t n, const float *uv, const float *duv, float *out) {
    if (!d || tex < 0 || (uint32_t)tex >= d->n_textures) { g_err = "texture index out of range"; return -1; }
    const MipMap M{d->textures[tex].mip, d->tex_texels};
    for (uint32_t i = 0; i < n; ++i) {
        const Spec v = duv ? M.filtered(uv[2 * i], uv[2 * i + 1], duv[4 * i], duv[4 * i + 1], duv[4 * i + 2], duv[4 * i + 3])
                           : M.unfiltered(uv[2 * i], uv[2 * i + 1]);
        out[3 * i] = v.s[0]; out[3 * i + 1] = v.s[1]; out[3 * i + 2] = v.s[2];
    }
    return 0;
}

/* MicrofacetDistribution sampling and densities for the reference's own
 * microfacet chi-square test (src/tests/test_microfacet.cpp:53-94,
 * MicrofacetAdapter): wi == NULL: sampleAll with its pdf, and pdfAll(m) =
 * D(m) cos(theta_m); else sampleVisible(wi) and pdfVisible(wi, m). */
int oracle_mf_sample_n(int type, float au, float av, const float *wi, uint32_t n, const float *u2, float *m, float *pdf) {
    const Microfacet mf(type, au, av, wi != nullptr);
    for (uint32_t i = 0; i < n; ++i) {
        float p = 0;
        const Vec v = wi ? mf.sampleVisibleN(Vec(wi[0], wi[1], wi[2]), u2[2 * i], u2[2 * i + 1])
                         : mf.sampleAll(u2[2 * i], u2[2 * i + 1], p);
        m[3 * i] = v.x; m[3 * i + 1] = v.y; m[3 * i + 2] = v.z;
        pdf[i] = wi ? mf.pdfVisible(Vec(wi[0], wi[1], wi[2]), v) : p;
    }
    return 0;
}

int oracle_mf_pdf_n(int type, float au, float av, const float *wi, uint32_t n, const float *m, float *pdf) {
    const Microfacet mf(type, au, av, wi != nullptr);
    for (uint32_t i = 0; i < n; ++i) {
        const Vec v(m[3 * i], m[3 * i + 1], m[3 * i + 2]);
        pdf[i] = wi ? mf.pdfVisible(Vec(wi[0], wi[1], wi[2]), v) : mf.eval(v) * cosTheta(v);
    }
    return 0;
}

}  // extern "C"
