// Device vs glibc float transcendentals: how often does the device library's
// float function (ROCm OCML) and a double-evaluated, rounded-to-float version
// differ from glibc's float result on the same arguments?  (DESIGN §9, C5's
// per-pixel tail.)  Build: hipcc --offload-arch=gfx950 -O2 -ffp-contract=off
// -o tools/math_probe tools/math_probe.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

enum { NF = 9 };
static const char *kName[NF] = {"sin", "cos", "acos", "atan2", "exp", "log", "pow", "tan", "atan"};

__global__ void k_probe(const float4 *in, float *outF, float *outD, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 a = in[i];
    const float x = a.x, y = a.y, z = a.z, p = a.w;
    const float q = fabsf(a.w) * 0.375f + 1e-3f;   // log / pow base in (0, 1.5]
    float s, c;
    sincosf(x, &s, &c);
    float f[NF] = {s, c, acosf(y), atan2f(y, z), expf(x), logf(q), powf(q, p), tanf(x * 0.25f), atanf(x)};
    float d[NF] = {(float)sin((double)x), (float)cos((double)x), (float)acos((double)y), (float)atan2((double)y, (double)z),
                   (float)exp((double)x), (float)log((double)q), (float)pow((double)q, (double)p),
                   (float)tan((double)(x * 0.25f)), (float)atan((double)x)};
    for (int k = 0; k < NF; ++k) {
        outF[(size_t)k * n + i] = f[k];
        outD[(size_t)k * n + i] = d[k];
    }
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4000000;
    std::vector<float4> in(n);
    uint64_t st = 88172645463325252ull;
    auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (st >> 11) * (1.0 / 9007199254740992.0); };
    for (int i = 0; i < n; ++i)
        in[i] = make_float4((float)((rnd() * 2 - 1) * 6.3), (float)(rnd() * 2 - 1), (float)(rnd() * 2 - 1), (float)(rnd() * 4));
    float4 *din; float *dF, *dD;
    if (hipMalloc(&din, sizeof(float4) * n) || hipMalloc(&dF, sizeof(float) * NF * n) || hipMalloc(&dD, sizeof(float) * NF * n)) return 2;
    hipMemcpy(din, in.data(), sizeof(float4) * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), 0, 0, din, dF, dD, n);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    std::vector<float> F((size_t)NF * n), D((size_t)NF * n);
    hipMemcpy(F.data(), dF, sizeof(float) * NF * n, hipMemcpyDeviceToHost);
    hipMemcpy(D.data(), dD, sizeof(float) * NF * n, hipMemcpyDeviceToHost);
    long mF[NF] = {0}, mD[NF] = {0}, mFD[NF] = {0};
    for (int i = 0; i < n; ++i) {
        const float x = in[i].x, y = in[i].y, z = in[i].z, p = in[i].w, q = fabsf(in[i].w) * 0.375f + 1e-3f;
        float s, c;
        sincosf(x, &s, &c);
        const float g[NF] = {s, c, acosf(y), atan2f(y, z), expf(x), logf(q), powf(q, p), tanf(x * 0.25f), atanf(x)};
        for (int k = 0; k < NF; ++k) {
            const float f = F[(size_t)k * n + i], d = D[(size_t)k * n + i];
            mF[k] += f != g[k];
            mD[k] += d != g[k];
            mFD[k] += f != d;
        }
    }
    printf("%-6s %14s %14s %14s\n", "fn", "ocml!=glibc", "cr!=glibc", "ocml!=cr");
    for (int k = 0; k < NF; ++k)
        printf("%-6s %14.3e %14.3e %14.3e\n", kName[k], mF[k] / (double)n, mD[k] / (double)n, mFD[k] / (double)n);
    hipFree(din); hipFree(dF); hipFree(dD);
    return 0;
}
