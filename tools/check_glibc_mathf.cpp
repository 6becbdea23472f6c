// Host check of my-mitsuba_amd/csrc/glibc_mathf.h against this machine's libm
// (the glibc Mitsuba links): every float argument (or a stride of them), bit
// for bit; NaN results only need to be NaN on both sides.
//   tools/check_glibc_mathf [stride] [fn...]     (stride 1 = all 2^32 floats;
//   fn: sinf cosf sincosf.s sincosf.c tanf expf logf atanf acosf atan2f powf)
// Build: hipcc -O2 -mfma -ffp-contract=off (Makefile target check_glibc_mathf).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <atomic>
#include <thread>
#include <vector>
#include "../my-mitsuba_amd/csrc/glibc_mathf.h"

typedef float (*F1)(float);
static float ref_sin(float x) { return ::sinf(x); }
static float ref_cos(float x) { return ::cosf(x); }
static float ref_sincos_s(float x) { float s, c; ::sincosf(x, &s, &c); return s; }
static float ref_sincos_c(float x) { float s, c; ::sincosf(x, &s, &c); return c; }
static float ref_tan(float x) { return ::tanf(x); }
static float ref_exp(float x) { return ::expf(x); }
static float ref_log(float x) { return ::logf(x); }
static float ref_atan(float x) { return ::atanf(x); }
static float ref_acos(float x) { return ::acosf(x); }
static float my_sin(float x) { return gmf::sinf(x); }
static float my_cos(float x) { return gmf::cosf(x); }
static float my_sincos_s(float x) { float s, c; gmf::sincosf(x, &s, &c); return s; }
static float my_sincos_c(float x) { float s, c; gmf::sincosf(x, &s, &c); return c; }
static float my_tan(float x) { return gmf::tanf(x); }
static float my_exp(float x) { return gmf::expf(x); }
static float my_log(float x) { return gmf::logf(x); }
static float my_atan(float x) { return gmf::atanf(x); }
static float my_acos(float x) { return gmf::acosf(x); }

struct Fn { const char *name; F1 ref, mine; };
static const Fn kFns[] = {{"sinf", ref_sin, my_sin}, {"cosf", ref_cos, my_cos}, {"sincosf.s", ref_sincos_s, my_sincos_s},
                          {"sincosf.c", ref_sincos_c, my_sincos_c}, {"tanf", ref_tan, my_tan}, {"expf", ref_exp, my_exp},
                          {"logf", ref_log, my_log}, {"atanf", ref_atan, my_atan}, {"acosf", ref_acos, my_acos}};

static bool same(float a, float b) {
    if (a != a || b != b) return a != a && b != b;
    return gmf::asuint(a) == gmf::asuint(b);
}

int main(int argc, char **argv) {
    const uint64_t stride = argc > 1 ? strtoull(argv[1], nullptr, 0) : 1;
    const int nth = std::max(1u, std::thread::hardware_concurrency());
    int fails = 0;
    for (const Fn &f : kFns) {
        bool want = argc <= 2;
        for (int a = 2; a < argc; ++a) want |= strcmp(argv[a], f.name) == 0 || strcmp(argv[a], "atan2f") == 0 && 0;
        if (!want) continue;
        std::atomic<uint64_t> bad{0}, tested{0};
        std::atomic<uint32_t> first{0xffffffffu};
        std::vector<std::thread> th;
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t]() {
                uint64_t b = 0, n = 0;
                for (uint64_t u = (uint64_t)t * stride; u < (1ull << 32); u += (uint64_t)nth * stride) {
                    const float x = gmf::asfloat((uint32_t)u);
                    ++n;
                    if (!same(f.ref(x), f.mine(x))) {
                        if (b++ == 0) {
                            uint32_t cur = first.load();
                            while ((uint32_t)u < cur && !first.compare_exchange_weak(cur, (uint32_t)u)) {}
                        }
                    }
                }
                bad += b;
                tested += n;
            });
        for (auto &x : th) x.join();
        printf("%-10s %llu arguments, %llu differ", f.name, (unsigned long long)tested.load(), (unsigned long long)bad.load());
        if (bad) {
            const float x = gmf::asfloat(first.load());
            printf(" (first 0x%08x = %a: libm %a, restated %a)", first.load(), x, f.ref(x), f.mine(x));
            ++fails;
        }
        printf("\n");
    }
    // atan2f: every first argument of a stride against a set of second ones
    bool want2 = argc <= 2;
    for (int a = 2; a < argc; ++a) want2 |= strcmp(argv[a], "atan2f") == 0;
    if (want2) {
        const float xs[] = {1.0f, -1.0f, 0.5f, -0.5f, 2.0f, -3.0f, 1e-20f, -1e-20f, 1e20f, -1e20f, 0.0f, -0.0f, INFINITY,
                            -INFINITY, 0.7071068f, -0.9999999f, 1e-39f, 3.4e38f, 12345.678f, -0.001f};
        std::atomic<uint64_t> bad{0}, tested{0};
        std::vector<std::thread> th;
        const uint64_t st2 = stride * 16;
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t]() {
                uint64_t b = 0, n = 0;
                uint64_t seed = 0x9E3779B97F4A7C15ull * (t + 1);
                for (uint64_t u = (uint64_t)t * st2; u < (1ull << 32); u += (uint64_t)nth * st2) {
                    const float y = gmf::asfloat((uint32_t)u);
                    seed = seed * 6364136223846793005ull + 1442695040888963407ull;
                    const float xr = gmf::asfloat((uint32_t)(seed >> 32));
                    for (float x : xs) { ++n; b += !same(::atan2f(y, x), gmf::atan2f(y, x)); }
                    ++n;
                    b += !same(::atan2f(y, xr), gmf::atan2f(y, xr));
                }
                bad += b;
                tested += n;
            });
        for (auto &x : th) x.join();
        printf("%-10s %llu argument pairs, %llu differ\n", "atan2f", (unsigned long long)tested.load(), (unsigned long long)bad.load());
        if (bad) ++fails;
    }
    // powf: every x (of the stride) against the exponents the shading code
    // passes (rtrans 0.25; Phong exponents 2 / alpha^2 - 2 and their pdf /
    // sampling forms; Beckmann's visible-normal fit 1 + t(-0.876 + t(0.4265 -
    // 0.0594 t)) over theta), then random (x, y) pairs: random bit patterns
    // and y uniform in [-8, 8]
    bool want3 = argc <= 2;
    for (int a = 2; a < argc; ++a) want3 |= strcmp(argv[a], "powf") == 0;
    if (want3) {
        std::vector<float> ys = {0.25f, 0.5f, 2.0f, 3.0f, -1.0f, 1.0f / 3.0f, 1.0f, 0.0f, -0.0f, 1e-8f, 100.0f, -2.5f, 7.0f,
                                 INFINITY, -INFINITY, NAN};
        for (float a : {0.1f, 0.2f, 0.3f, 0.5f, 0.05f}) {   // Phong: alpha -> exponent
            const float e = 2.0f / (a * a) - 2.0f;
            ys.push_back(e);
            ys.push_back(e + 1.0f);
            ys.push_back(1.0f / (e + 2.0f));
        }
        for (int k = 0; k <= 16; ++k) {   // Beckmann's fit over thetaI in [0, pi/2]
            const float t = (float)k * 1.5707963f / 16.0f;
            ys.push_back(1 + t * (-0.876f + t * (0.4265f - 0.0594f * t)));
        }
        for (float y : ys) {
            std::atomic<uint64_t> bad{0}, tested{0};
            std::atomic<uint32_t> first{0xffffffffu};
            std::vector<std::thread> th;
            for (int t = 0; t < nth; ++t)
                th.emplace_back([&, t]() {
                    uint64_t b = 0, n = 0;
                    for (uint64_t u = (uint64_t)t * stride; u < (1ull << 32); u += (uint64_t)nth * stride) {
                        const float x = gmf::asfloat((uint32_t)u);
                        ++n;
                        if (!same(::powf(x, y), gmf::powf(x, y))) {
                            if (b++ == 0) {
                                uint32_t cur = first.load();
                                while ((uint32_t)u < cur && !first.compare_exchange_weak(cur, (uint32_t)u)) {}
                            }
                        }
                    }
                    bad += b;
                    tested += n;
                });
            for (auto &x : th) x.join();
            printf("powf(x, %-13a) %llu arguments, %llu differ", y, (unsigned long long)tested.load(),
                   (unsigned long long)bad.load());
            if (bad) {
                const float x = gmf::asfloat(first.load());
                printf(" (first x = %a: libm %a, restated %a)", x, ::powf(x, y), gmf::powf(x, y));
                ++fails;
            }
            printf("\n");
        }
        std::atomic<uint64_t> bad{0}, tested{0};
        std::vector<std::thread> th;
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t]() {
                uint64_t b = 0, n = 0;
                uint64_t seed = 0xD1B54A32D192ED03ull * (t + 7);
                for (uint64_t u = (uint64_t)t * stride; u < (1ull << 32); u += (uint64_t)nth * stride) {
                    seed = seed * 6364136223846793005ull + 1442695040888963407ull;
                    const float x = gmf::asfloat((uint32_t)(seed >> 32));
                    const float yb = gmf::asfloat((uint32_t)seed);
                    const float yu = -8.0f + 16.0f * (float)((seed >> 8) & 0xffffff) * 0x1p-24f;
                    const float xa = fabsf(x);
                    n += 3;
                    b += !same(::powf(x, yb), gmf::powf(x, yb));
                    b += !same(::powf(x, yu), gmf::powf(x, yu));
                    b += !same(::powf(xa, yu), gmf::powf(xa, yu));
                }
                bad += b;
                tested += n;
            });
        for (auto &x : th) x.join();
        printf("%-10s %llu random argument pairs, %llu differ\n", "powf", (unsigned long long)tested.load(),
               (unsigned long long)bad.load());
        if (bad) ++fails;
    }
    return fails ? 1 : 0;
}
