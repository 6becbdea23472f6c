// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE for the traversal's
// access shapes.  MI355X_MICROARCH.md ("HBM")
// documents FETCH_SIZE = TCC_EA0_RDREQ x 64 B reading exactly 1/2 of a wide
// coalesced 16-B/lane stream (128-B requests tallied at 64 B); gathers are
// uncalibrated there.  Each kernel below reads a known set of bytes once from
// a 4-GiB buffer (far beyond the 256-MiB Infinity Cache, no line read twice),
// so FETCH_SIZE per launch against those bytes gives the correction for that
// shape:
//   stream16   every lane 16 B, coalesced                  (the guide's case)
//   g16        one 16-B load per 128-B line, random lines  (a node-pair fetch)
//   g16x2      two 16-B loads per line, at +0 and +64      (two halves of one line)
//   g32        one 32-B load per line                      (a grandchild pair)
//   g48@0/@48  one 48-B TriAccel-sized record per random line, inside one
//              64-B sector / across two sectors of the line (the primitive fetch)
// g16x2 tells the fill granularity: if the second half-line load costs no
// extra request, the L2 fills whole 128-B lines (and a 64-B tally per request
// means x2); if it doubles FETCH_SIZE, requests are 64-B sectors.
// Run: rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/fetch_calib
// (tools/fetch_calib_summary.py turns the two csv files into the table).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr size_t BUF_BYTES = size_t(4) << 30;       // 4 GiB
constexpr size_t LINES = BUF_BYTES / 128;            // 2^25 128-B lines
constexpr uint32_t N = 1u << 24;                      // accesses per kernel

// a bijection of [0, 2^25): odd multiplier, then a xor-shift
__device__ inline uint32_t perm_line(uint32_t i, uint32_t salt) {
    uint32_t x = (i * 2654435761u + salt) & (uint32_t)(LINES - 1);
    x ^= x >> 13;
    return (x * 0x9E3779B1u) & (uint32_t)(LINES - 1);
}

__global__ void k_stream16(const float4 *__restrict__ b, float *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const float4 v = b[i];
    if (v.x == 1.5f) out[i] = v.y;   // never (the buffer is zero): keeps the load
}
__global__ void k_g16(const float4 *__restrict__ b, float *out, uint32_t salt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const float4 v = b[(size_t)perm_line(i, salt) * 8];
    if (v.x == 1.5f) out[i] = v.y;
}
__global__ void k_g16x2(const float4 *__restrict__ b, float *out, uint32_t salt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const size_t l = (size_t)perm_line(i, salt) * 8;
    const float4 v = b[l], w = b[l + 4];
    if (v.x + w.x == 1.5f) out[i] = v.y;
}
__global__ void k_g32(const float4 *__restrict__ b, float *out, uint32_t salt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const size_t l = (size_t)perm_line(i, salt) * 8;
    const float4 v = b[l], w = b[l + 1];
    if (v.x + w.x == 1.5f) out[i] = v.y;
}
// a 48-B record inside one random line: at byte 0 (one 64-B sector) or at
// byte 48 (across the sector boundary: two sectors of the same line)
__global__ void k_g48(const float4 *__restrict__ b, float *out, uint32_t salt, uint32_t off16) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const size_t r = (size_t)perm_line(i, salt) * 8 + off16;
    const float4 x = b[r], y = b[r + 1], z = b[r + 2];
    if (x.x + y.x + z.x == 1.5f) out[i] = x.y;
}

#define CHECK(e) do { hipError_t err_ = (e); if (err_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #e, hipGetErrorString(err_)); return 1; } } while (0)

int main() {
    float4 *b = nullptr;
    float *out = nullptr;
    CHECK(hipMalloc((void **)&b, BUF_BYTES));
    CHECK(hipMalloc((void **)&out, (size_t)N * sizeof(float)));
    CHECK(hipMemset(b, 0, BUF_BYTES));
    CHECK(hipDeviceSynchronize());
    const dim3 g(N / 256), blk(256);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // bytes each kernel asks for (the lanes' loads), and the distinct 128-B lines it touches
    struct K { const char *name; double bytes, lines, sectors; } ks[] = {
        {"k_stream16", 16.0 * N, 16.0 * N / 128, 16.0 * N / 64}, {"k_g16", 16.0 * N, (double)N, (double)N},
        {"k_g16x2", 32.0 * N, (double)N, 2.0 * N}, {"k_g32", 32.0 * N, (double)N, (double)N},
        {"k_g48@0", 48.0 * N, (double)N, (double)N}, {"k_g48@48", 48.0 * N, (double)N, 2.0 * N}};
    printf("N %u accesses per kernel; 4-GiB buffer; kernels in launch order (two repetitions)\n", N);
    for (int rep = 0; rep < 2; ++rep) {
        for (int k = 0; k < 6; ++k) {
            const uint32_t salt = 0x1234567u * (uint32_t)(2 * k + rep + 1);
            CHECK(hipEventRecord(e0));
            switch (k) {
                case 0: hipLaunchKernelGGL(k_stream16, g, blk, 0, 0, b + (size_t)rep * N, out); break;
                case 1: hipLaunchKernelGGL(k_g16, g, blk, 0, 0, b, out, salt); break;
                case 2: hipLaunchKernelGGL(k_g16x2, g, blk, 0, 0, b, out, salt); break;
                case 3: hipLaunchKernelGGL(k_g32, g, blk, 0, 0, b, out, salt); break;
                case 4: hipLaunchKernelGGL(k_g48, g, blk, 0, 0, b, out, salt, 0u); break;
                case 5: hipLaunchKernelGGL(k_g48, g, blk, 0, 0, b, out, salt, 3u); break;
            }
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("%s rep %d: %.3f ms, %.0f bytes requested, %.0f 128-B lines, %.0f 64-B sectors, %.1f GB/s requested\n",
                   ks[k].name, rep, ms, ks[k].bytes, ks[k].lines, ks[k].sectors, ks[k].bytes / (ms * 1e-3) / 1e9);
        }
    }
    CHECK(hipGetLastError());
    (void)hipFree(b);
    (void)hipFree(out);
    return 0;
}
