// Throughput of the device's float transcendentals: glibc_mathf.h (gmf::, the
// path integrator's default) vs ROCm's float library, on the argument ranges
// the shading code gives them (angles in [-pi, pi], cosines in [-1, 1], ...).
// Each thread evaluates a dependent chain, so the figure is issue cost per
// call, not memory.  Build: make tools/math_bench   Run: tools/math_bench
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "../my-mitsuba_amd/csrc/glibc_mathf.h"

constexpr int ITERS = 256;

// y feeds the next argument through a cheap map back into the function's range
#define KERNEL(NAME, EXPR, FOLD)                                                           \
    __global__ void NAME(float *out, float seed) {                                         \
        float x = seed + (blockIdx.x * blockDim.x + threadIdx.x) * 1e-7f;                  \
        float acc = 0.0f;                                                                   \
        for (int i = 0; i < ITERS; ++i) {                                                   \
            const float y = EXPR;                                                           \
            acc += y;                                                                       \
            x = FOLD;                                                                       \
        }                                                                                   \
        out[blockIdx.x * blockDim.x + threadIdx.x] = acc;                                   \
    }

#define ANGLE (x * 0.999f + 0.37f > 3.14159f ? x * 0.999f + 0.37f - 6.28318f : x * 0.999f + 0.37f)
#define UNIT (x * 0.73f + 0.29f > 1.0f ? x * 0.73f + 0.29f - 2.0f : x * 0.73f + 0.29f)

__device__ inline float sc_g(float x) { float s, c; gmf::sincosf(x, &s, &c); return s + c; }
__device__ inline float sc_o(float x) { float s, c; sincosf(x, &s, &c); return s + c; }

KERNEL(k_sincos_g, sc_g(x), ANGLE)
KERNEL(k_sincos_o, sc_o(x), ANGLE)
KERNEL(k_tan_g, gmf::tanf(x * 0.45f), ANGLE)
KERNEL(k_tan_o, tanf(x * 0.45f), ANGLE)
KERNEL(k_acos_g, gmf::acosf(x), UNIT)
KERNEL(k_acos_o, acosf(x), UNIT)
KERNEL(k_atan2_g, gmf::atan2f(x, 0.5f - x * x), UNIT)
KERNEL(k_atan2_o, atan2f(x, 0.5f - x * x), UNIT)
KERNEL(k_atan_g, gmf::atanf(x * 4.0f), UNIT)
KERNEL(k_atan_o, atanf(x * 4.0f), UNIT)
KERNEL(k_exp_g, gmf::expf(-x * x), UNIT)
KERNEL(k_exp_o, expf(-x * x), UNIT)
KERNEL(k_log_g, gmf::logf(x * x + 0.01f), UNIT)
KERNEL(k_log_o, logf(x * x + 0.01f), UNIT)
KERNEL(k_div_f, 1.0f / (x + 2.5f), UNIT)
KERNEL(k_base, x * 1.0001f, UNIT)

typedef void (*K)(float *, float);
int main() {
    const int blocks = 256 * 8 * 4, threads = 256;
    float *out;
    if (hipMalloc(&out, sizeof(float) * blocks * threads)) return 2;
    struct { const char *name; K g, o; } ks[] = {
        {"sincosf", k_sincos_g, k_sincos_o}, {"tanf", k_tan_g, k_tan_o}, {"acosf", k_acos_g, k_acos_o},
        {"atan2f", k_atan2_g, k_atan2_o},   {"atanf", k_atan_g, k_atan_o}, {"expf", k_exp_g, k_exp_o},
        {"logf", k_log_g, k_log_o},         {"1/x", k_div_f, k_div_f},     {"loop", k_base, k_base}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const double calls = (double)blocks * threads * ITERS;
    printf("%-8s %12s %12s   (ns per 1e3 calls, whole GPU; %.0f calls per launch)\n", "fn", "gmf", "ocml", calls);
    for (auto &k : ks) {
        float ms[2];
        for (int v = 0; v < 2; ++v) {
            K f = v ? k.o : k.g;
            hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, out, 0.1f);
            hipEventRecord(a, 0);
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, out, 0.1f + r);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms[v], a, b);
            ms[v] /= 5;
        }
        printf("%-8s %12.4f %12.4f\n", k.name, ms[0] * 1e6 / calls * 1e3, ms[1] * 1e6 / calls * 1e3);
    }
    hipFree(out);
    return 0;
}
