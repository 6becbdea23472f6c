// On the GPU: the device's float transcendentals vs the host's glibc, bit for
// bit, over a strided sweep of all 2^32 float arguments (NaN results only need
// to be NaN on both sides).  Two device versions per function:
//   gmf::*  my-mitsuba_amd/csrc/glibc_mathf.h, glibc 2.35's algorithms (what the
//           path integrator calls, device_math.h mt_*)
//   ocml    ROCm's float library (sinf, expf, ...), for comparison
// atan2f takes y = the argument and x from a hash of it; powf takes |x| and
// an exponent in [-8, 8) from another hash (and 0.25, roughplastic's).  DESIGN §5.
// Build: make tools/math_probe   Run: tools/math_probe [stride]  (default 3)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <thread>
#include <vector>

#include "../my-mitsuba_amd/csrc/glibc_mathf.h"

enum { NF = 10 };
static const char *kName[NF] = {"sinf", "cosf", "tanf", "expf", "logf", "atanf", "acosf", "atan2f", "powf", "powf.25"};

__host__ __device__ inline float arg_y(uint32_t u) {
    uint32_t h = u * 0x9E3779B9u;
    h ^= h >> 16;
    return gmf::asfloat((h & 0x807fffffu) | (((h >> 7) % 254u + 1u) << 23));   // a finite float from u
}
// powf's exponent: uniform in [-8, 8) from a hash of u
__host__ __device__ inline float arg_p(uint32_t u) {
    uint32_t h = (u ^ 0x5bd1e995u) * 0x85EBCA6Bu;
    h ^= h >> 13;
    return -8.0f + 16.0f * (float)(h >> 8) * 0x1p-24f;
}

__global__ void k_probe(uint64_t start, uint64_t stride, uint32_t n, float *outG, float *outO) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t u = (uint32_t)(start + (uint64_t)i * stride);
    const float x = gmf::asfloat(u), y = arg_y(u);
    const float p = arg_p(u), ax = fabsf(x);
    const float g[NF] = {gmf::sinf(x), gmf::cosf(x), gmf::tanf(x), gmf::expf(x), gmf::logf(x), gmf::atanf(x),
                         gmf::acosf(x), gmf::atan2f(x, y), gmf::powf(ax, p), gmf::powf(ax, 0.25f)};
    const float o[NF] = {sinf(x), cosf(x), tanf(x), expf(x), logf(x), atanf(x), acosf(x), atan2f(x, y), powf(ax, p),
                         powf(ax, 0.25f)};
    for (int k = 0; k < NF; ++k) {
        outG[(size_t)k * n + i] = g[k];
        outO[(size_t)k * n + i] = o[k];
    }
}

static bool same(float a, float b) {
    if (a != a || b != b) return a != a && b != b;
    return gmf::asuint(a) == gmf::asuint(b);
}

int main(int argc, char **argv) {
    const uint64_t stride = argc > 1 ? strtoull(argv[1], nullptr, 0) : 3;
    const uint32_t chunk = 1u << 24;
    float *dG, *dO;
    if (hipMalloc(&dG, sizeof(float) * NF * chunk) || hipMalloc(&dO, sizeof(float) * NF * chunk)) return 2;
    std::vector<float> G((size_t)NF * chunk), O((size_t)NF * chunk);
    uint64_t badG[NF] = {0}, badO[NF] = {0}, total = 0;
    uint32_t firstG[NF];
    for (int k = 0; k < NF; ++k) firstG[k] = 0xffffffffu;
    const int nth = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    for (uint64_t start = 0; start < (1ull << 32); start += (uint64_t)chunk * stride) {
        const uint32_t n = (uint32_t)std::min<uint64_t>(chunk, ((1ull << 32) - start + stride - 1) / stride);
        hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), 0, 0, start, stride, n, dG, dO);
        if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 3; }
        hipMemcpy(G.data(), dG, sizeof(float) * NF * n, hipMemcpyDeviceToHost);
        hipMemcpy(O.data(), dO, sizeof(float) * NF * n, hipMemcpyDeviceToHost);
        std::vector<std::thread> th;
        std::vector<uint64_t> bG((size_t)nth * NF, 0), bO((size_t)nth * NF, 0);
        std::vector<uint32_t> fG((size_t)nth * NF, 0xffffffffu);
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t]() {
                for (uint32_t i = t; i < n; i += nth) {
                    const uint32_t u = (uint32_t)(start + (uint64_t)i * stride);
                    const float x = gmf::asfloat(u), y = arg_y(u);
                    const float p = arg_p(u), ax = fabsf(x);
                    const float ref[NF] = {::sinf(x), ::cosf(x), ::tanf(x), ::expf(x), ::logf(x), ::atanf(x), ::acosf(x),
                                           ::atan2f(x, y), ::powf(ax, p), ::powf(ax, 0.25f)};
                    for (int k = 0; k < NF; ++k) {
                        if (!same(G[(size_t)k * n + i], ref[k])) {
                            if (bG[t * NF + k]++ == 0) fG[t * NF + k] = u;
                        }
                        bO[t * NF + k] += !same(O[(size_t)k * n + i], ref[k]);
                    }
                }
            });
        for (auto &x : th) x.join();
        for (int t = 0; t < nth; ++t)
            for (int k = 0; k < NF; ++k) {
                badG[k] += bG[t * NF + k];
                badO[k] += bO[t * NF + k];
                if (fG[t * NF + k] < firstG[k]) firstG[k] = fG[t * NF + k];
            }
        total += n;
        fprintf(stderr, "\r%.0f%%", 100.0 * (double)(start + (uint64_t)chunk * stride) / 4294967296.0);
    }
    fprintf(stderr, "\n");
    printf("%llu arguments (every %llu-th float bit pattern), device vs this host's glibc, bit for bit\n",
           (unsigned long long)total, (unsigned long long)stride);
    printf("%-7s %16s %16s\n", "fn", "gmf!=glibc", "ocml!=glibc");
    int fails = 0;
    for (int k = 0; k < NF; ++k) {
        printf("%-7s %16llu %16llu", kName[k], (unsigned long long)badG[k], (unsigned long long)badO[k]);
        if (badG[k]) { printf("   first 0x%08x", firstG[k]); ++fails; }
        printf("\n");
    }
    hipFree(dG);
    hipFree(dO);
    return fails ? 1 : 0;
}
