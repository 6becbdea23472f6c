// Rough dielectric transmittance for `roughplastic` (src/bsdfs/rtrans.h).
//
// Mitsuba ships this function precomputed over (eta, alpha, cos theta)
// (data/microfacet/{beckmann,ggx,phong}.dat: 50 x 50 x 100 samples on
// 4th-root warped axes) and reduces the table to the material's (eta, alpha)
// by cubic interpolation (RoughTransmittance::setEta/setAlpha,
// rtrans.h:292-388).  The tables are not available where this library runs,
// so the material's 1D slice is computed here directly, by quadrature of the
// integral the reference validates its tables against
// (src/tests/test_rtrans.cpp:25-33,49-113): the energy a `roughdielectric`
// interface transmits, i.e. the mean sample weight of
// BSDF::sample(bRec{typeMask = ETransmission, EImportance}) over [0,1]^2.
//
// Writing that weight in microfacet space (roughdielectric.cpp:508-590):
//   T(wi) = \int (1 - F(wi.m)) G1(wi,m) G1(wo(m),m) <wi.m>+ D(m) / cos(wi) dm
// with wo(m) = refract(wi, m) on the far side.  m is drawn from D(m) cos(m)
// (the closed-form `sampleAll` warps, microfacet.h:287-397, isotropic), so the
// integrand is smooth and bounded and a midpoint grid over the sample square
// converges quickly; phi is integrated over [0, pi] only (the integrand is
// symmetric in phi about the plane of incidence).
//
// The table is sampled at the reference's nodes: cos(theta_k) = (k/(n-1))^4
// (rtrans.h:177-183), evaluated by evalCubicInterp1D on the warped axis.
// Diffuse transmittance = \int_0^1 2 mu T(mu) dmu (test_rtrans.cpp:35-38).
#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "scene.h"

namespace mtsh {
namespace {

struct D3 { double x, y, z; };
inline double dot(const D3 &a, const D3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// smithG1, isotropic (microfacet.h:477-514); Phong uses the Beckmann
// rational approximation
double smithG1(int type, double alpha, const D3 &v, const D3 &m) {
    if (dot(v, m) * v.z <= 0) return 0.0;
    const double st2 = std::max(0.0, 1 - v.z * v.z);
    if (st2 <= 0) return 1.0;
    const double tt = std::abs(std::sqrt(st2) / v.z);
    if (tt == 0.0) return 1.0;
    if (type != MTSG_MF_GGX) {
        const double a = 1.0 / (alpha * tt);
        if (a >= 1.6) return 1.0;
        return (3.535 * a + 2.181 * a * a) / (1.0 + 2.276 * a + 2.577 * a * a);
    }
    const double root = alpha * tt;
    return 2.0 / (1.0 + std::sqrt(1.0 + root * root));
}

// fresnelDielectricExt (util.cpp:651-681)
double fresnel(double cosThetaI_, double &cosThetaT_, double eta) {
    if (eta == 1) { cosThetaT_ = -cosThetaI_; return 0.0; }
    const double scale = cosThetaI_ > 0 ? 1 / eta : eta;
    const double c2 = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (c2 <= 0.0) { cosThetaT_ = 0.0; return 1.0; }
    const double ci = std::abs(cosThetaI_), ct = std::sqrt(c2);
    const double Rs = (ci - eta * ct) / (ci + eta * ct), Rp = (eta * ci - ct) / (eta * ci + ct);
    cosThetaT_ = cosThetaI_ > 0 ? -ct : ct;
    return 0.5 * (Rs * Rs + Rp * Rp);
}

// cos(theta_m) of the sampleAll warp for u1 (microfacet.h:287-397, isotropic)
double sampleCosThetaM(int type, double alpha, double u1) {
    if (type == MTSG_MF_BECKMANN) return 1.0 / std::sqrt(1.0 - alpha * alpha * std::log(1.0 - u1));
    if (type == MTSG_MF_GGX) return 1.0 / std::sqrt(1.0 + alpha * alpha * u1 / (1.0 - u1));
    const double e = std::max(2.0 / (alpha * alpha) - 2.0, 0.0);   // computePhongExponent
    return std::pow(u1, 1.0 / (e + 2.0));
}

constexpr int kThetaGrid = 512, kPhiGrid = 64;

double transmittance(int type, double alpha, double eta, double mu) {
    // the reference's tables hold the grazing limit at cos = 0; its own
    // check clamps cos to 1e-5 (test_rtrans.cpp:84-85)
    mu = std::max(mu, 1e-5);
    const D3 wi{std::sqrt(std::max(0.0, 1 - mu * mu)), 0.0, mu};
    double sum = 0;
    for (int i = 0; i < kThetaGrid; ++i) {
        // u1 = 1 - (1 - v)^2: the integrand grows like 1/cos(theta_m) ~
        // (1 - u1)^(-1/2) for grazing microfacets (heavy GGX tails); the
        // Jacobian 2 (1 - v) cancels that singularity
        const double v = (i + 0.5) / kThetaGrid, jac = 2 * (1 - v);
        const double cm = sampleCosThetaM(type, alpha, 1 - (1 - v) * (1 - v));
        const double sm = std::sqrt(std::max(0.0, 1 - cm * cm));
        for (int j = 0; j < kPhiGrid; ++j) {
            const double phi = M_PI * (j + 0.5) / kPhiGrid;
            const D3 m{sm * std::cos(phi), sm * std::sin(phi), cm};
            const double wim = dot(wi, m);
            if (wim <= 0) continue;
            double cosThetaT;
            const double F = fresnel(wim, cosThetaT, eta);
            if (F >= 1.0 || cosThetaT == 0) continue;
            // refract (util.cpp:767-772)
            const double e = cosThetaT < 0 ? 1 / eta : eta;
            const double k = wim * e + cosThetaT;
            const D3 wo{m.x * k - wi.x * e, m.y * k - wi.y * e, m.z * k - wi.z * e};
            if (wi.z * wo.z >= 0) continue;
            const double g = smithG1(type, alpha, wi, m) * smithG1(type, alpha, wo, m);
            sum += jac * (1 - F) * g * wim / (mu * cm);
        }
    }
    return sum / ((double)kThetaGrid * kPhiGrid);
}

// T at n abscissae, spread over up to 16 host threads (the quadrature of one
// material's tables is ~10^7 integrand evaluations)
void transmittanceMany(int type, double alpha, double eta, const std::vector<double> &mu, std::vector<double> &out) {
    out.assign(mu.size(), 0.0);
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nt; ++t)
        pool.emplace_back([&, t] {
            for (size_t i = t; i < mu.size(); i += nt) out[i] = transmittance(type, alpha, eta, mu[i]);
        });
    for (auto &th : pool) th.join();
}

}  // namespace

void roughTransmittanceSlice(int type, float alpha, float eta, int n, float *trans) {
    std::vector<double> mu(n), t;
    for (int k = 0; k < n; ++k) {
        const double w = (double)k / (n - 1);
        mu[k] = w * w * w * w;
    }
    transmittanceMany(type, alpha, eta, mu, t);
    for (int k = 0; k < n; ++k) trans[k] = (float)std::min(1.0, std::max(0.0, t[k]));
}

float roughDiffuseTransmittance(int type, float alpha, float eta) {
    // \int_0^1 2 mu T(mu) dmu, midpoint rule
    constexpr int kMu = 256;
    std::vector<double> mu(kMu), t;
    for (int i = 0; i < kMu; ++i) mu[i] = (i + 0.5) / kMu;
    transmittanceMany(type, alpha, eta, mu, t);
    double sum = 0;
    for (int i = 0; i < kMu; ++i) sum += 2 * mu[i] * t[i];
    return (float)std::min(1.0, std::max(0.0, sum / kMu));
}

}  // namespace mtsh
