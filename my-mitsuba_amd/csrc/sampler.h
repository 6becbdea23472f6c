// Device samplers: the per-sample random / quasi-random numbers of a path.
//
// Every draw is a pure function of (pixel, sample index, dimension), so a
// path's numbers can be produced in any kernel, by any lane, in any batch:
//   independent  counter-mode draws (device_math.h counterFloat)
//   halton       src/samplers/halton.cpp:240-386: radical inverse in the
//                dim-th prime base of offset(pixel) + stride * s, blocked space
//                partition (setFilmResolution, blocked = true, as
//                Integrator::configureSampler sets it, integrator.cpp:39-43)
//   hammersley   src/samplers/hammersley.cpp:181-283: dimension 0 = index / N,
//                then radical inverses in the prime bases
//   ldsampler    src/samplers/ldsampler.cpp:143-216: scrambled (0,2)-sequence
//                per dimension, 1D and 2D requests counted separately; the
//                per-pixel scramble and shuffle come from the counter RNG
// The radical inverse restates RINV / SCRAMBLED_RINV (src/libcore/qmc.cpp:
// 141-167) with a run-time base; the library is compiled without FMA
// contraction, so values are bit-identical to the oracle's.
#pragma once

#include "device_math.h"

namespace mtsg {

struct DevSampler {
    int type;                      // MTSG_SAMPLER_*
    int ldDim;                     // ldsampler: low-discrepancy dimensions
    uint32_t ldBits;               // log2(spp) (ldsampler)
    uint32_t stride;               // halton: prod of prime powers; hammersley: res.y
    uint32_t multInv[2];           // halton CRT coefficients
    uint32_t primePow[2], primeExp[2];
    uint32_t res[2], logH;         // hammersley tile resolution
    float factor;                  // hammersley 1 / (spp * res.x * res.y)
    uint16_t inv[2][3];            // inverse digit permutations of bases 2, 3
    const uint32_t *primes, *off;  // MTSG_QMC_PRIMES each
    const uint16_t *perm;          // nullptr: unscrambled
    // sobol (sobol.cpp, sobolseq.h): generator matrices, look_up tables,
    // bucketed resolution 2^logRes, TEA'd scramble
    const uint32_t *sobolM;
    const uint64_t *vdc, *vdcInv;
    uint32_t logRes;
    float sobolRes;
    uint64_t sobolScramble;
};

constexpr float kOneMinusEps = 0x1.fffffep-1f;   // ONE_MINUS_EPS_FLT (constants.h:56)
constexpr uint32_t kLdSalt = 0x6C64736Du;       // pixel keys of the ldsampler (as the oracle)

// RINV / SCRAMBLED_RINV (qmc.cpp:141-167); 32-bit digit arithmetic while the
// index fits (always, for the image sizes and sample counts of the configs)
DEV float radical_inverse(uint32_t base, uint64_t index, const uint16_t *perm) {
#pragma clang fp contract(off)
    const float radical = 1.0f / (float)base;
    uint64_t value = 0;
    float factor = 1.0f;
    if ((index >> 32) == 0) {
        uint32_t idx = (uint32_t)index;
        while (idx) {
            const uint32_t next = idx / base;
            const uint32_t digit = idx - next * base;
            value = value * base + (perm ? perm[digit] : digit);
            factor *= radical;
            idx = next;
        }
    } else {
        while (index) {
            const uint64_t next = index / base;
            const uint64_t digit = index - next * base;
            value = value * base + (perm ? perm[digit] : digit);
            factor *= radical;
            index = next;
        }
    }
    float inverse;
    if (perm) inverse = factor * ((float)value + radical * (float)perm[0] / (1 - radical));
    else inverse = (float)value * factor;
    return fminf(inverse, kOneMinusEps);
}

// halton.cpp:195-209
DEV uint32_t inverse_scrambled_radical_inverse(uint32_t base, uint32_t inverse, uint32_t digits, const uint16_t *invPerm) {
    uint32_t index = 0;
    while (digits) {
        uint32_t digit = inverse % base;
        if (invPerm) digit = invPerm[digit];
        inverse /= base;
        index = index * base + digit;
        --digits;
    }
    return index;
}

// qmc.h:43-58, 82-87
DEV float radical_inverse2_single(uint32_t n, uint32_t scramble) {
    n = __builtin_bitreverse32(n);
    n = (n >> (32 - 24)) ^ (scramble & ~(0xFFFFFFFFu << 24));
    return (float)n / (float)(1u << 24);
}
DEV float sobol2_single(uint32_t n, uint32_t scramble) {
    for (uint32_t v = 1u << 31; n != 0; n >>= 1, v ^= v >> 1)
        if (n & 1) scramble ^= v;
    return (float)scramble / 4294967296.0f;
}

// keyed bijection of [0, 2^bits): the ldsampler's per-pixel shuffle
DEV uint32_t ld_shuffle(uint32_t s, uint32_t bits, uint64_t h) {
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

// generate(pos): the pixel's subsequence offset (halton.cpp:277-293,
// hammersley.cpp:206-218)
DEV uint64_t qmc_pixel_offset(const DevSampler &S, int x, int y, uint32_t spp) {
    const uint32_t px = (uint32_t)x % 128u, py = (uint32_t)y % 128u;
    if (S.type == MTSG_SAMPLER_HALTON) {
        if (S.stride <= 1) return 0;
        const uint32_t v0 = inverse_scrambled_radical_inverse(2, px, S.primeExp[0], S.perm ? S.inv[0] : nullptr);
        const uint32_t v1 = inverse_scrambled_radical_inverse(3, py, S.primeExp[1], S.perm ? S.inv[1] : nullptr);
        const uint64_t o = (uint64_t)v0 * (S.stride / S.primePow[0]) * S.multInv[0] +
                           (uint64_t)v1 * (S.stride / S.primePow[1]) * S.multInv[1];
        return o % S.stride;
    }
    return (uint64_t)px * S.res[1] * spp + inverse_scrambled_radical_inverse(2, py, S.logH, S.perm ? S.inv[0] : nullptr);
}

// sobolseq.h:43-58 sampleSingle
DEV float sobol_sample(const DevSampler &S, uint64_t index, uint32_t dim) {
    uint32_t result = (uint32_t)S.sobolScramble;
    const uint32_t *col = S.sobolM + dim * MTSG_SOBOL_COLUMNS;
    uint32_t lo = (uint32_t)index, hi = (uint32_t)(index >> 32);
    for (; lo; lo &= lo - 1u) result ^= col[__builtin_ctz(lo)];
    for (; hi; hi &= hi - 1u) result ^= col[32 + __builtin_ctz(hi)];
    return fminf((float)result * (1.0f / 4294967296.0f), kOneMinusEps);
}

// sobolseq.h:99-131 look_up (single precision), as SobolSampler::setSampleIndex
// uses it when the film is bucketed (sobol.cpp:204-216)
DEV uint64_t sobol_index(const DevSampler &S, uint32_t frame, int x, int y) {
    if (!(S.logRes > 1 && x >= 0)) return (uint64_t)frame;
    const uint32_t m = S.logRes;
    uint64_t index = (uint64_t)frame << (2 * m);
    uint64_t delta = 0;
    const uint64_t *v = S.vdc + (size_t)(m - 1) * MTSG_SOBOL_COLUMNS, *vi = S.vdcInv + (size_t)(m - 1) * MTSG_SOBOL_COLUMNS;
    for (uint32_t f = frame; f; f &= f - 1u) delta ^= v[__builtin_ctz(f)];
    const uint64_t scramble = (S.sobolScramble & 0xFFFFFFFFull) >> (32 - m);
    uint64_t b = ((((uint64_t)(uint32_t)x ^ scramble) << m) | ((uint64_t)(uint32_t)y ^ scramble)) ^ delta;
    for (; b; b &= b - 1ull) index ^= vi[__builtin_ctzll(b)];
    return index;
}

// One path's draws.  `dim` = dimensions consumed so far (next1D: 1,
// next2D: 2), `n2` = next2D calls so far; both live in the path state.
struct PathSampler {
    uint64_t key;                  // counter key of (pixel, sample)
    uint32_t dim, n2, s;           // dimensions used, 2D requests, sample index
    int x, y;                      // film pixel
    bool dimError;                 // QMC dimension limit exceeded (Mitsuba: EError)
    uint64_t qidx;                 // sobol: the sample's index in the sequence (sobol_index)
};

template <int KIND>
DEV float qmc_float(const DevSampler &S, PathSampler &p, uint64_t idx) {
    const uint32_t d = p.dim++;
    if (KIND == MTSG_SAMPLER_HAMMERSLEY) {
        if (d == 0) return (float)idx * S.factor;
        return radical_inverse(S.primes[d - 1], idx, S.perm ? S.perm + S.off[d - 1] : nullptr);
    }
    return radical_inverse(S.primes[d], idx, S.perm ? S.perm + S.off[d] : nullptr);
}

// KIND: MTSG_SAMPLER_* of the render (a template parameter, so each kernel
// carries only its sampler's code)
template <int KIND>
DEV float smp_next1D(const DevSampler &S, PathSampler &p, uint32_t seed, uint64_t pixelIndex, uint32_t spp) {
    if (KIND == MTSG_SAMPLER_SOBOL) {   // sobol.cpp:218-228
        if (p.dim >= MTSG_SOBOL_DIMS) { p.dimError = true; p.dim++; return 0.0f; }
        return sobol_sample(S, p.qidx, p.dim++);
    }
    if (KIND == MTSG_SAMPLER_HALTON || KIND == MTSG_SAMPLER_HAMMERSLEY) {
        if (p.dim >= MTSG_QMC_PRIMES) { p.dimError = true; p.dim++; return 0.0f; }
        return qmc_float<KIND>(S, p, qmc_pixel_offset(S, p.x, p.y, spp) + (uint64_t)S.stride * p.s);
    }
    if (KIND == MTSG_SAMPLER_LDSAMPLER) {
        const uint32_t n1 = p.dim - 2 * p.n2;
        if ((int)n1 < S.ldDim) {
            const uint64_t h = mix64(counterKey(seed ^ kLdSalt, pixelIndex) + (uint64_t)(2 * n1 + 1) * 0xD1B54A32D192ED03ULL);
            ++p.dim;
            return radical_inverse2_single(ld_shuffle(p.s, S.ldBits, h), (uint32_t)(h >> 32));
        }
    }
    return counterFloat(p.key, p.dim++);
}

template <int KIND>
DEV void smp_next2D(const DevSampler &S, PathSampler &p, uint32_t seed, uint64_t pixelIndex, uint32_t spp, float &a, float &b) {
    if (KIND == MTSG_SAMPLER_SOBOL) {   // sobol.cpp:230-250
        if (p.dim + 1 >= MTSG_SOBOL_DIMS) { p.dimError = true; p.dim += 2; p.n2++; a = b = 0.0f; return; }
        if (p.dim == 0 && p.qidx != (uint64_t)p.s) {
            a = sobol_sample(S, p.qidx, p.dim++) * S.sobolRes - (float)p.x;
            b = sobol_sample(S, p.qidx, p.dim++) * S.sobolRes - (float)p.y;
        } else {
            a = sobol_sample(S, p.qidx, p.dim++);
            b = sobol_sample(S, p.qidx, p.dim++);
        }
        p.n2++;
        return;
    }
    if (KIND == MTSG_SAMPLER_HALTON || KIND == MTSG_SAMPLER_HAMMERSLEY) {
        if (p.dim + 1 >= MTSG_QMC_PRIMES) { p.dimError = true; p.dim += 2; p.n2++; a = b = 0.0f; return; }
        const uint64_t idx = qmc_pixel_offset(S, p.x, p.y, spp) + (uint64_t)S.stride * p.s;
        if (p.dim == 0) {
            const float v1 = qmc_float<KIND>(S, p, idx), v2 = qmc_float<KIND>(S, p, idx);
            const uint32_t sx = KIND == MTSG_SAMPLER_HALTON ? S.primePow[0] : S.res[0];
            const uint32_t sy = KIND == MTSG_SAMPLER_HALTON ? S.primePow[1] : S.res[1];
            a = v1 * (float)sx - (float)((uint32_t)p.x % 128u);
            b = v2 * (float)sy - (float)((uint32_t)p.y % 128u);
        } else {
            a = qmc_float<KIND>(S, p, idx);
            b = qmc_float<KIND>(S, p, idx);
        }
        p.n2++;
        return;
    }
    if (KIND == MTSG_SAMPLER_LDSAMPLER && (int)p.n2 < S.ldDim) {
        const uint64_t h = mix64(counterKey(seed ^ kLdSalt, pixelIndex) + (uint64_t)(2 * p.n2 + 2) * 0xD1B54A32D192ED03ULL);
        const uint64_t sc = mix64(h ^ 0x5851F42D4C957F2DULL);
        const uint32_t i = ld_shuffle(p.s, S.ldBits, h);
        a = radical_inverse2_single(i, (uint32_t)sc);
        b = sobol2_single(i, (uint32_t)(sc >> 32));
        p.dim += 2;
        p.n2++;
        return;
    }
    a = counterFloat(p.key, p.dim++);
    b = counterFloat(p.key, p.dim++);
    p.n2++;
}

}  // namespace mtsg
