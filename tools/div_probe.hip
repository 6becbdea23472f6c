// On the GPU: fast reciprocal / division sequences (v_rcp_f32 + FMA Newton
// and Markstein steps) against the IEEE-correct division the kernels compile
// (1.0f / x and a / b with -ffp-contract=off: v_div_scale / v_div_fmas /
// v_div_fixup), bit for bit.  The reciprocal runs over all 2^32 float bit
// patterns; the division over 2^32 hashed (a, b) pairs per class:
//   any    both from all finite floats
//   tri    the triangle test's operand ranges: a = a distance-like value in
//          [2^-20, 2^20], b = a cosine-like value in [2^-24, 2], both signs
// NaN results only need to be NaN on both sides.  Mismatch counts and the
// first mismatching operands are printed per variant.
// Build: make tools/div_probe   Run: tools/div_probe [log2 pairs per class] (default 32)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

__device__ __host__ inline float asf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
__device__ __host__ inline uint32_t asu(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

// y ~ 1/x (v_rcp_f32, 1 ulp) and one FMA Newton step
__device__ inline float rcp_nr1(float x) {
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}
// two Newton steps
__device__ inline float rcp_nr2(float x) {
    const float y = rcp_nr1(x);
    const float e = __builtin_fmaf(-x, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}
// the kernels' guarded form (my-mitsuba_amd/csrc/device_math.h rcp_exact):
// the Newton reciprocal for exponent fields 1..252, else the IEEE division
__device__ inline float rcp_guarded(float x) {
    const uint32_t e = (asu(x) >> 23) & 0xFFu;
    float y;
    if (__builtin_expect(e - 1u < 252u, 1)) {
        const float r = __builtin_amdgcn_rcpf(x);
        y = __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
    } else {
        y = 1.0f / x;
    }
    return y;
}
// a / b: the Newton reciprocal, a quotient and one Markstein correction
__device__ inline float div_m1(float a, float b) {
    const float y = rcp_nr1(b);
    const float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}
// the same with a second correction
__device__ inline float div_m2(float a, float b) {
    const float y = rcp_nr1(b);
    float q = a * y;
    float r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
    r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}

__device__ inline bool same(float a, float b) {
    if (a != a || b != b) return a != a && b != b;
    return asu(a) == asu(b);
}

__device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
// a finite float from u: any exponent 1..254 (no zero / denormal / inf)
__device__ inline float finite_from(uint32_t u) {
    return asf((u & 0x807fffffu) | (((u >> 7) % 254u + 1u) << 23));
}
// a float of magnitude in [2^lo, 2^hi), random sign
__device__ inline float range_from(uint32_t u, int lo, int hi) {
    const uint32_t e = (uint32_t)(lo + 127 + (int)((u >> 8) % (uint32_t)(hi - lo)));
    return asf((u & 0x80000000u) | (e << 23) | (hash32(u) & 0x7fffffu));
}

enum { NV = 7, KEEP = 8 };
// rcp_nr1 mismatches per exponent field of x (all 2^32 x): which inputs the
// kernels' guard (device_math.h rcp_exact) must send to the IEEE division
__device__ unsigned long long g_rcpByExp[256];
// variants: 0 rcp_nr1, 1 rcp_nr2 (all x); 2 div_m1 any, 3 div_m2 any, 4 div_m1 tri, 5 div_m2 tri;
// 6 rcp_guarded (all x)
__global__ void k_probe(uint64_t base, uint32_t n, unsigned long long *cnt, float *keep) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t u = (uint32_t)(base + i);
    bool bad[NV];
    float a1[NV], b1[NV];
    {
        const float x = asf(u), ref = 1.0f / x;
        bad[0] = !same(rcp_nr1(x), ref);
        if (bad[0]) atomicAdd(&g_rcpByExp[(u >> 23) & 0xFFu], 1ull);
        bad[1] = !same(rcp_nr2(x), ref);
        bad[6] = !same(rcp_guarded(x), ref);
        a1[0] = a1[1] = a1[6] = 1.0f;
        b1[0] = b1[1] = b1[6] = x;
    }
    {
        const float a = finite_from(hash32(u * 2u + 1u)), b = finite_from(hash32(u * 2u + 2u) ^ 0x5bd1e995u);
        const float ref = a / b;
        bad[2] = !same(div_m1(a, b), ref);
        bad[3] = !same(div_m2(a, b), ref);
        a1[2] = a1[3] = a;
        b1[2] = b1[3] = b;
    }
    {
        const float a = range_from(hash32(u ^ 0xA511E9B3u), -20, 20), b = range_from(hash32(u + 0x68E31DA4u), -24, 1);
        const float ref = a / b;
        bad[4] = !same(div_m1(a, b), ref);
        bad[5] = !same(div_m2(a, b), ref);
        a1[4] = a1[5] = a;
        b1[4] = b1[5] = b;
    }
    for (int k = 0; k < NV; ++k)
        if (bad[k]) {
            const unsigned long long c = atomicAdd(&cnt[k], 1ull);
            if (c < KEEP) {
                keep[(k * KEEP + c) * 2] = a1[k];
                keep[(k * KEEP + c) * 2 + 1] = b1[k];
            }
        }
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 32;
    const uint64_t total = 1ull << lg;
    const uint32_t chunk = 1u << 26;
    unsigned long long *dc;
    float *dk;
    if (hipMalloc(&dc, NV * sizeof(unsigned long long)) || hipMalloc(&dk, NV * KEEP * 2 * sizeof(float))) return 2;
    if (hipMemset(dc, 0, NV * sizeof(unsigned long long)) || hipMemset(dk, 0, NV * KEEP * 2 * sizeof(float))) return 2;
    for (uint64_t b = 0; b < total; b += chunk) {
        const uint32_t n = (uint32_t)((total - b) < chunk ? (total - b) : chunk);
        hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), 0, 0, b, n, dc, dk);
        if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 3; }
        if ((b / chunk) % 16 == 15) { printf("progress %.0f%%\n", 100.0 * (b + n) / total); fflush(stdout); }
    }
    unsigned long long c[NV];
    float k[NV * KEEP * 2];
    if (hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost) || hipMemcpy(k, dk, sizeof(k), hipMemcpyDeviceToHost)) return 2;
    unsigned long long byExp[256];
    if (hipMemcpyFromSymbol(byExp, HIP_SYMBOL(g_rcpByExp), sizeof(byExp))) return 2;
    printf("rcp_nr1 mismatches by exponent field of x:");
    for (int e = 0; e < 256; ++e)
        if (byExp[e]) printf(" [%d] %llu", e, byExp[e]);
    printf("\n");
    static const char *name[NV] = {"rcp_nr1 (all 2^32 x)", "rcp_nr2 (all 2^32 x)", "div_m1 any", "div_m2 any",
                                   "div_m1 tri", "div_m2 tri", "rcp_exact (all 2^32 x)"};
    for (int v = 0; v < NV; ++v) {
        printf("%-22s %llu of %llu differ", name[v], c[v], (unsigned long long)total);
        for (unsigned long long j = 0; j < c[v] && j < KEEP; ++j)
            printf("  (%a / %a)", k[(v * KEEP + j) * 2], k[(v * KEEP + j) * 2 + 1]);
        printf("\n");
    }
    return 0;
}
