// Plugin construction from Properties: the part of Mitsuba's scene loading
// that turns each object's parameters into the device scene.  Two clients:
//   - the XML loader (loader.cpp), which parses a scene file into Properties
//     the way SceneHandler does (src/librender/scenehandler.cpp:461-625) and
//     calls these factories in document order;
//   - the in-memory builder C-ABI (mtsh_scene_begin / mtsh_scene_add_* /
//     mtsh_scene_finish, include/mtsh.h), which a Mitsuba-side plugin drives
//     from the objects Mitsuba already holds: each object's substituted
//     Properties (ConfigurableObject::getProperties, cobject.h:77) and the
//     TriMesh arrays (trimesh.h:127-153).
// Each factory restates its plugin's constructor / configure():
//   bsdfs   diffuse (diffuse.cpp:75-84), roughconductor (roughconductor.cpp:168-203,
//           microfacet.h:99-146), dielectric (dielectric.cpp:148-170),
//           roughdielectric (roughdielectric.cpp:160-205), conductor
//           (conductor.cpp:98-130), plastic (plastic.cpp:93-140), roughplastic
//           (roughplastic.cpp:198-300), twosided (twosided.cpp:52-80)
//   texture bitmap (bitmap.cpp:179-302)
//   emitter area (area.cpp:67-78), envmap (envmap.cpp:105-185)
//   shapes  ply, obj, serialized, cube, rectangle, shapegroup / instance
//   sensor  perspective (perspective.cpp, sensor.cpp:150-262), film hdrfilm
//           (hdrfilm.cpp:209-220), rfilter gaussian / box
//   sampler independent, halton, hammersley, ldsampler, sobol
//   integrator path (integrator.cpp:199-234), myPath2_OM (myPath2_OM.cpp:61-85)
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstring>
#include <fstream>

#include "scene.h"

namespace mtsh {

static std::runtime_error err(const std::string &m) { return std::runtime_error(m); }
static std::string lower(std::string s) {
    for (auto &c : s) c = (char)tolower((unsigned char)c);
    return s;
}
static std::string at(int line) { return line > 0 ? "line " + std::to_string(line) + ": " : std::string(); }

// ---------------------------------------------------------------------------
// Properties (include/mitsuba/core/properties.h)
// ---------------------------------------------------------------------------
float Properties::getFloat(const std::string &n, float def) const {
    auto it = floats.find(n);
    if (it != floats.end()) return it->second;
    auto ii = ints.find(n);
    if (ii != ints.end()) return (float)ii->second;
    return def;
}
float Properties::getFloat(const std::string &n) const {
    if (!floats.count(n) && !ints.count(n)) throw err("Property \"" + n + "\" has not been specified!");
    return getFloat(n, 0.0f);
}
long long Properties::getInt(const std::string &n, long long def) const {
    auto it = ints.find(n);
    return it != ints.end() ? it->second : def;
}
bool Properties::getBool(const std::string &n, bool def) const {
    auto it = bools.find(n);
    return it != bools.end() ? it->second : def;
}
std::string Properties::getString(const std::string &n, const std::string &def) const {
    auto it = strings.find(n);
    return it != strings.end() ? it->second : def;
}
V3 Properties::getSpectrum(const std::string &n, const V3 &def) const {
    auto it = spectra.find(n);
    if (it != spectra.end()) return it->second;
    auto f = floats.find(n);
    if (f != floats.end()) return V3(f->second);
    return def;
}
Transform Properties::getTransform(const std::string &n, const Transform &def) const {
    auto it = transforms.find(n);
    return it != transforms.end() ? it->second : def;
}

// ---------------------------------------------------------------------------
// IOR tables
// ---------------------------------------------------------------------------
namespace {
struct ConductorEntry { const char *name; float eta[3]; float k[3]; };
const ConductorEntry kConductors[] = {
#include "ior_table.inc"
};
// src/bsdfs/ior.h:38-66
const struct { const char *name; float value; } kIOR[] = {
    {"vacuum", 1.0f}, {"helium", 1.000036f}, {"hydrogen", 1.000132f}, {"air", 1.000277f},
    {"carbon dioxide", 1.00045f}, {"water", 1.3330f}, {"acetone", 1.36f}, {"ethanol", 1.361f},
    {"carbon tetrachloride", 1.461f}, {"glycerol", 1.4729f}, {"benzene", 1.501f},
    {"silicone oil", 1.52045f}, {"bromine", 1.661f}, {"water ice", 1.31f}, {"fused quartz", 1.458f},
    {"pyrex", 1.470f}, {"acrylic glass", 1.49f}, {"polypropylene", 1.49f}, {"bk7", 1.5046f},
    {"sodium chloride", 1.544f}, {"amber", 1.55f}, {"pet", 1.5750f}, {"diamond", 2.419f}};
}  // namespace

bool lookupConductor(const std::string &name, V3 &eta, V3 &k) {
    for (auto &c : kConductors)
        if (name == c.name) { eta = V3(c.eta[0], c.eta[1], c.eta[2]); k = V3(c.k[0], c.k[1], c.k[2]); return true; }
    return false;
}

float lookupIOR(const std::string &name) {
    std::string l = lower(name);
    for (auto &e : kIOR) if (l == e.name) return e.value;
    throw err("Unable to find an IOR value for \"" + l + "\"!");
}

static float lookupIORProp(const Properties &props, const std::string &n, const std::string &def) {
    if (props.floats.count(n)) return props.floats.at(n);
    return lookupIOR(props.getString(n, def));
}

// ---------------------------------------------------------------------------
// helpers of the BSDF constructors
// ---------------------------------------------------------------------------
namespace {
// util.cpp:651-681 (double precision, for the quadrature below)
double fresnelDielectricD(double cosThetaI, double eta) {
    if (eta == 1) return 0.0;
    double scale = cosThetaI > 0 ? 1 / eta : eta;
    double cosThetaTSqr = 1 - (1 - cosThetaI * cosThetaI) * (scale * scale);
    if (cosThetaTSqr <= 0.0) return 1.0;
    double ci = std::abs(cosThetaI), ct = std::sqrt(cosThetaTSqr);
    double Rs = (ci - eta * ct) / (ci + eta * ct), Rp = (eta * ci - ct) / (eta * ci + ct);
    return 0.5 * (Rs * Rs + Rp * Rp);
}
// fresnelDiffuseReflectance(eta, fast = false) (util.cpp:814-860): the
// integral over xi in [0, 1] of F(sqrt(xi)); Mitsuba uses adaptive
// Gauss-Lobatto with relative error 1e-5, restated here as adaptive
// Simpson in double precision to 1e-10 (identical to float precision)
double simpson(double eta, double a, double b, double fa, double fm, double fb, double whole, int depth) {
    const double m = 0.5 * (a + b), lm = 0.5 * (a + m), rm = 0.5 * (m + b);
    const double flm = fresnelDielectricD(std::sqrt(lm), eta), frm = fresnelDielectricD(std::sqrt(rm), eta);
    const double left = (m - a) / 6 * (fa + 4 * flm + fm), right = (b - m) / 6 * (fm + 4 * frm + fb);
    if (depth <= 0 || std::abs(left + right - whole) <= 1e-10) return left + right + (left + right - whole) / 15;
    return simpson(eta, a, m, fa, flm, fm, left, depth - 1) + simpson(eta, m, b, fm, frm, fb, right, depth - 1);
}
float fresnelDiffuseReflectance(float eta) {
    const double fa = fresnelDielectricD(0.0, eta), fm = fresnelDielectricD(std::sqrt(0.5), eta), fb = fresnelDielectricD(1.0, eta);
    return (float)simpson(eta, 0.0, 1.0, fa, fm, fb, (fa + 4 * fm + fb) / 6, 40);
}
// BSDF::ensureEnergyConservation(texture, name, 1) (bsdf.cpp:88-113): a
// constant whose largest component exceeds 1 is scaled by 0.99 / max
V3 energyConserving(const Properties &props, V3 v) {
    if (!props.getBool("ensureEnergyConservation", true)) return v;
    float mx = std::max(v.x, std::max(v.y, v.z));
    return mx > 1.0f ? v * (0.99f * (1.0f / mx)) : v;
}
float luminance(V3 v) { return v.x * 0.212671f + v.y * 0.715160f + v.z * 0.072169f; }   // spectrum.h:638-640
// conductor material: the data/ior/<name>.{eta,k}.spd lookup (RGB), eta/k overrides, / extEta
void conductorIOR(const Properties &props, mtsg_bsdf &d, const char *who) {
    std::string material = props.getString("material", "Cu");
    V3 intEta, intK;
    if (lower(material) == "none") { intEta = V3(0.0f); intK = V3(1.0f); }
    else if (!lookupConductor(material, intEta, intK)) throw err(std::string(who) + ": unknown material \"" + material + "\"");
    float extEta = lookupIORProp(props, "extEta", "air");
    V3 eta = props.getSpectrum("eta", intEta) / extEta;
    V3 k = props.getSpectrum("k", intK) / extEta;
    for (int i = 0; i < 3; ++i) { d.eta[i] = eta[i]; d.k[i] = k[i]; }
}
// MicrofacetDistribution(props) (microfacet.h:99-146)
void microfacetProps(const Properties &props, mtsg_bsdf &d) {
    int distr = MTSG_MF_BECKMANN;
    if (props.strings.count("distribution")) {
        std::string dn = lower(props.strings.at("distribution"));
        if (dn == "beckmann") distr = MTSG_MF_BECKMANN;
        else if (dn == "ggx") distr = MTSG_MF_GGX;
        else if (dn == "phong" || dn == "as") distr = MTSG_MF_PHONG;
        else throw err("Specified an invalid microfacet distribution \"" + dn + "\", must be \"beckmann\", \"ggx\", or \"phong\"/\"as\"!");
    }
    float au = 0.1f, av = 0.1f;
    if (props.has("alpha")) {
        if (props.has("alphaU") || props.has("alphaV")) throw err("Microfacet model: please specify either 'alpha' or 'alphaU'/'alphaV'.");
        au = av = props.getFloat("alpha");
    } else if (props.has("alphaU") || props.has("alphaV")) {
        if (!props.has("alphaU") || !props.has("alphaV")) throw err("Microfacet model: both 'alphaU' and 'alphaV' must be specified.");
        au = props.getFloat("alphaU"); av = props.getFloat("alphaV");
    }
    au = std::max(au, 1e-4f); av = std::max(av, 1e-4f);
    d.distribution = distr;
    // visible-normal sampling is not supported for Phong (microfacet.h:140-144)
    d.sample_visible = (props.getBool("sampleVisible", true) && distr != MTSG_MF_PHONG) ? 1 : 0;
    d.alpha_u = au; d.alpha_v = av;
}
}  // namespace

// ---------------------------------------------------------------------------
// SceneBuilder
// ---------------------------------------------------------------------------
SceneBuilder::SceneBuilder(Scene &s) : scene(s) {}

std::unique_ptr<Scene> SceneBuilder::newScene() {
    auto scene = std::make_unique<Scene>();
    scene->kd.threads = g_defaultKDThreads;
    scene->groupKd = scene->kd;
    scene->twoLevel = g_instancing == 1;
    return scene;
}

// Scene::Scene(const Properties &) (scene.cpp:47-83): the scene's kd-tree
// build parameters (the setters of gkdtree.h:760-925).  Unlike Mitsuba, which
// logs unqueried properties, a name it would not read is an error here.
void SceneBuilder::sceneProps(const Properties &props, int line) {
    KDBuildParams &k = scene.kd;
    static const std::map<std::string, const char *> kinds = {
        {"kdIntersectionCost", "float"}, {"kdTraversalCost", "float"}, {"kdEmptySpaceBonus", "float"},
        {"kdStopPrims", "integer"}, {"kdMaxDepth", "integer"}, {"kdExactPrimitiveThreshold", "integer"},
        {"kdMaxBadRefines", "integer"}, {"kdClip", "boolean"}, {"kdRetract", "boolean"}, {"kdParallelBuild", "boolean"}};
    // every property must be one Scene(props) reads, with its type
    auto check = [&](const std::string &n, const char *type) {
        auto it = kinds.find(n);
        if (it == kinds.end()) throw err(at(line) + "unknown scene property '" + n + "'");
        if (std::string(it->second) != type) throw err(at(line) + "scene property '" + n + "' must be of type " + it->second);
    };
    for (const auto &kv : props.strings) check(kv.first, "string");
    for (const auto &kv : props.spectra) check(kv.first, "spectrum");
    for (const auto &kv : props.points) check(kv.first, "point");
    for (const auto &kv : props.transforms) check(kv.first, "transform");
    for (const auto &kv : props.floats) {
        check(kv.first, "float");
        if (kv.first == "kdIntersectionCost") k.queryCost = kv.second;
        else if (kv.first == "kdTraversalCost") k.traversalCost = kv.second;
        else k.emptySpaceBonus = kv.second;
    }
    for (const auto &kv : props.ints) {
        check(kv.first, "integer");
        const std::string &n = kv.first;
        const long long v = kv.second;
        if (n == "kdStopPrims") {
            if (v < 1) throw err(at(line) + "kdStopPrims must be >= 1");
            k.stopPrims = (int)v;
        } else if (n == "kdMaxDepth") {
            if (v < 0 || v > 64) throw err(at(line) + "kdMaxDepth must lie in [0, 64]");
            k.maxDepth = (int)v;
        } else if (n == "kdExactPrimitiveThreshold") {
            if (v < 0) throw err(at(line) + "kdExactPrimitiveThreshold must be >= 0");
            k.exactPrimThreshold = k.exactSweepLimit = (int)std::min<long long>(v, 1 << 30);
        } else {
            if (v < 0) throw err(at(line) + "kdMaxBadRefines must be >= 0");
            k.maxBadRefines = (int)v;
        }
    }
    for (const auto &kv : props.bools) {
        check(kv.first, "boolean");
        if (kv.first == "kdClip") k.clip = kv.second;
        else if (kv.first == "kdRetract") k.retract = kv.second;
        // kdParallelBuild: accepted; the host build's threads are mtsh_set_kd_threads
    }
}

std::string SceneBuilder::resolve(const std::string &f) const {
    if (!f.empty() && f[0] == '/') return f;
    for (auto it = dirStack.rbegin(); it != dirStack.rend(); ++it) {
        std::string p = *it + "/" + f;
        std::ifstream t(p);
        if (t.good()) return p;
    }
    return (dirStack.empty() ? std::string(".") : dirStack.back()) + "/" + f;
}

// `bitmap` texture (src/textures/bitmap.cpp:179-302, Texture2D(props),
// src/librender/texture.cpp:84-98); returns its index in scene.textures
int SceneBuilder::texture(const std::string &type_, const Properties &props, const std::string &id, int line) {
    const std::string type = lower(type_);
    if (type != "bitmap")
        throw err(at(line) + "texture plugin \"" + type + "\" is outside this build's scope (only 'bitmap')");
    if (lower(props.getString("coordinates", "uv")) != "uv") throw err("Only UV coordinates are supported at the moment!");
    if (!props.getString("channel", "").empty()) throw err("bitmap: the 'channel' parameter is not supported by this build");
    const std::string file = props.getString("filename", "");
    if (file.empty()) throw err("bitmap: missing 'filename'");
    const std::string path = resolve(file);
    const std::string filterType = lower(props.getString("filterType", "ewa"));
    int filter;
    if (filterType == "ewa") filter = MTSG_MIP_EWA;
    else if (filterType == "bilinear") filter = MTSG_MIP_BILINEAR;
    else if (filterType == "trilinear") filter = MTSG_MIP_TRILINEAR;
    else if (filterType == "nearest") filter = MTSG_MIP_NEAREST;
    else throw err("Unknown filter type '" + filterType + "' -- must be 'ewa', 'trilinear', or 'nearest'!");
    auto wrap = [&](const std::string &w) {   // bitmap.cpp:324-339
        if (w == "repeat") return (int)MTSG_WRAP_REPEAT;
        if (w == "clamp") return (int)MTSG_WRAP_CLAMP;
        if (w == "mirror") return (int)MTSG_WRAP_MIRROR;
        if (w == "zero" || w == "black") return (int)MTSG_WRAP_ZERO;
        if (w == "one" || w == "white") return (int)MTSG_WRAP_ONE;
        throw err("Unknown wrap mode '" + w + "' -- must be 'repeat', 'clamp', 'black', or 'white'!");
    };
    const std::string wrapMode = props.getString("wrapMode", "repeat");
    const int wrapU = wrap(props.getString("wrapModeU", wrapMode)), wrapV = wrap(props.getString("wrapModeV", wrapMode));
    const float gamma = props.getFloat("gamma", 0.0f);
    const float maxAniso = props.getFloat("maxAnisotropy", 20.0f);
    Texture t;
    t.id = id;
    mtsg_texture &d = t.d;
    const float uvscale = props.getFloat("uvscale", 1.0f);
    d.uv_offset[0] = props.getFloat("uoffset", 0.0f);
    d.uv_offset[1] = props.getFloat("voffset", 0.0f);
    d.uv_scale[0] = props.getFloat("uscale", uvscale);
    d.uv_scale[1] = props.getFloat("vscale", uvscale);
    d.scale = 1.0f;
    int w = 0, h = 0;
    std::vector<float> rgb;
    loadTextureImage(path, gamma, w, h, rgb);
    // TMIPMap(bitmap, ..., maxValue = 1) (mipmap.h:155-170)
    buildMipmap(std::move(rgb), w, h, filter, wrapU, wrapV, 1.0f, maxAniso, scene.texTexels, d.mip, d.average, d.maximum);
    scene.textures.push_back(t);
    return (int)scene.textures.size() - 1;
}

// The texture given for one of a BSDF's parameters: only the parameters the
// device evaluates per hit may be textured; returns its index or -1
static int texturedParam(const std::map<std::string, int> &textures, const std::vector<std::string> &names,
                         const std::string &bsdfType, int line, int nTextures) {
    int found = -1;
    for (auto &kv : textures) {
        if (std::find(names.begin(), names.end(), kv.first) == names.end())
            throw err(at(line) + bsdfType + ": a texture for parameter \"" + kv.first + "\" is outside this build's scope");
        if (kv.second < 0 || kv.second >= nTextures) throw err(bsdfType + ": invalid texture id for \"" + kv.first + "\"");
        found = kv.second;
    }
    return found;
}

// Constant or textured reflectance of diffuse / plastic / roughplastic:
// ensureEnergyConservation scales a texture by 0.99 / max through a
// ScaleTexture (bsdf.cpp:88-113); returns the value used for getAverage()
// (the texture's average x scale) and sets d.texture
V3 SceneBuilder::reflectance(const Properties &props, int tex, const V3 &constant, mtsg_bsdf &d, float &maxOut) {
    if (tex < 0) {
        const V3 r = energyConserving(props, constant);
        maxOut = std::max(r.x, std::max(r.y, r.z));
        d.texture = 0;
        return r;
    }
    mtsg_texture &t = scene.textures[tex].d;
    float mx = std::max(t.maximum[0], std::max(t.maximum[1], t.maximum[2]));
    if (props.getBool("ensureEnergyConservation", true) && mx * t.scale > 1.0f) {
        // a second BSDF sharing the texture gets its own scaled copy
        Texture copy = scene.textures[tex];
        copy.id.clear();
        copy.d.scale = t.scale * (0.99f * (1.0f / (mx * t.scale)));
        scene.textures.push_back(copy);
        tex = (int)scene.textures.size() - 1;
    }
    const mtsg_texture &tt = scene.textures[tex].d;
    d.texture = tex + 1;
    maxOut = std::max(tt.maximum[0], std::max(tt.maximum[1], tt.maximum[2])) * tt.scale;
    return V3(tt.average[0], tt.average[1], tt.average[2]) * tt.scale;
}

int SceneBuilder::bsdf(const std::string &type_, const Properties &props, const std::map<std::string, int> &textures,
                       const std::vector<int> &nested, const std::string &id, int line) {
    const std::string type = lower(type_);
    const int nTex = (int)scene.textures.size();
    Bsdf b;
    b.id = id;
    mtsg_bsdf &d = b.d;
    if (type != "twosided" && !nested.empty()) throw err(at(line) + type + ": nested BSDFs are only accepted by 'twosided'");
    if (type == "diffuse") {
        // diffuse.cpp:77-84, configure() keeps the component iff max > 0
        float mx;
        const int tex = texturedParam(textures, {"reflectance", "diffuseReflectance"}, type, line, nTex);
        V3 r = reflectance(props, tex,
                           props.getSpectrum(props.has("reflectance") ? "reflectance" : "diffuseReflectance", V3(0.5f)), d, mx);
        d.type = MTSG_BSDF_DIFFUSE;
        d.reflectance[0] = r.x; d.reflectance[1] = r.y; d.reflectance[2] = r.z;
        d.smooth = mx > 0;
        d.ref_n_zero = 0;
    } else if (type == "roughconductor") {
        // roughconductor.cpp:168-203
        texturedParam(textures, {}, type, line, nTex);
        V3 spec = energyConserving(props, props.getSpectrum("specularReflectance", V3(1.0f)));
        conductorIOR(props, d, "roughconductor");
        microfacetProps(props, d);
        d.type = MTSG_BSDF_ROUGHCONDUCTOR;
        for (int i = 0; i < 3; ++i) d.spec_refl[i] = spec[i];
        d.smooth = 1;
        d.ref_n_zero = 0;
    } else if (type == "dielectric") {
        // dielectric.cpp:148-170
        texturedParam(textures, {}, type, line, nTex);
        float intIOR = lookupIORProp(props, "intIOR", "bk7");
        float extIOR = lookupIORProp(props, "extIOR", "air");
        if (intIOR < 0 || extIOR < 0) throw err("The interior and exterior indices of refraction must be positive!");
        V3 sr = energyConserving(props, props.getSpectrum("specularReflectance", V3(1.0f)));
        V3 st = energyConserving(props, props.getSpectrum("specularTransmittance", V3(1.0f)));
        d.type = MTSG_BSDF_DIELECTRIC;
        d.ior_eta = intIOR / extIOR;
        d.ior_inv_eta = 1 / d.ior_eta;
        for (int i = 0; i < 3; ++i) { d.spec_refl[i] = sr[i]; d.spec_trans[i] = st[i]; }
        d.smooth = 0;        // delta components only
        d.ref_n_zero = 1;    // ETransmission | EBackSide
    } else if (type == "roughdielectric") {
        // roughdielectric.cpp:160-205: microfacet reflection + transmission
        texturedParam(textures, {}, type, line, nTex);
        float intIOR = lookupIORProp(props, "intIOR", "bk7");
        float extIOR = lookupIORProp(props, "extIOR", "air");
        if (intIOR < 0 || extIOR < 0 || intIOR == extIOR)
            throw err("The interior and exterior indices of refraction must be positive and differ!");
        V3 sr = energyConserving(props, props.getSpectrum("specularReflectance", V3(1.0f)));
        V3 st = energyConserving(props, props.getSpectrum("specularTransmittance", V3(1.0f)));
        microfacetProps(props, d);
        d.type = MTSG_BSDF_ROUGHDIELECTRIC;
        d.ior_eta = intIOR / extIOR;
        d.ior_inv_eta = 1 / d.ior_eta;
        for (int i = 0; i < 3; ++i) { d.spec_refl[i] = sr[i]; d.spec_trans[i] = st[i]; }
        d.smooth = 1;        // glossy components: direct sampling
        d.ref_n_zero = 1;    // ETransmission | EBackSide
    } else if (type == "conductor") {
        // conductor.cpp:98-130: ideal mirror with the exact conductor Fresnel term
        texturedParam(textures, {}, type, line, nTex);
        V3 spec = energyConserving(props, props.getSpectrum("specularReflectance", V3(1.0f)));
        conductorIOR(props, d, "conductor");
        d.type = MTSG_BSDF_CONDUCTOR;
        for (int i = 0; i < 3; ++i) d.spec_refl[i] = spec[i];
        d.smooth = 0;        // delta reflection only: no direct sampling (path.cpp:174)
        d.ref_n_zero = 0;
    } else if (type == "plastic") {
        // plastic.cpp:93-140: smooth dielectric coating over a diffuse base
        float intIOR = lookupIORProp(props, "intIOR", "polypropylene");
        float extIOR = lookupIORProp(props, "extIOR", "air");
        if (intIOR < 0 || extIOR < 0) throw err("The interior and exterior indices of refraction must be positive!");
        V3 sr = energyConserving(props, props.getSpectrum("specularReflectance", V3(1.0f)));
        float dmx;
        const int tex = texturedParam(textures, {"diffuseReflectance"}, type, line, nTex);
        V3 dr = reflectance(props, tex, props.getSpectrum("diffuseReflectance", V3(0.5f)), d, dmx);
        d.type = MTSG_BSDF_PLASTIC;
        d.ior_eta = intIOR / extIOR;
        d.ior_inv_eta = 1 / d.ior_eta;
        d.nonlinear = props.getBool("nonlinear", false) ? 1 : 0;
        d.fdr_int = fresnelDiffuseReflectance(1 / d.ior_eta);
        const float dAvg = luminance(dr), sAvg = luminance(sr);
        d.spec_sampling_weight = sAvg / (dAvg + sAvg);
        for (int i = 0; i < 3; ++i) { d.spec_refl[i] = sr[i]; d.reflectance[i] = dr[i]; }
        d.smooth = 1;        // diffuse component
        d.ref_n_zero = 0;
    } else if (type == "roughplastic") {
        // roughplastic.cpp:198-300: microfacet dielectric coating over a
        // diffuse base; rough transmittance through the interface
        float intIOR = lookupIORProp(props, "intIOR", "polypropylene");
        float extIOR = lookupIORProp(props, "extIOR", "air");
        if (intIOR < 0 || extIOR < 0 || intIOR == extIOR)
            throw err("The interior and exterior indices of refraction must be positive and differ!");
        microfacetProps(props, d);
        if (d.alpha_u != d.alpha_v)
            throw err("The 'roughplastic' plugin currently does not support anisotropic microfacet distributions!");
        // RoughTransmittance::checkEta/checkAlpha (rtrans.h:222-258): the
        // range the reference's tables cover (eta in [1.0001, 4] after
        // inverting eta < 1, alpha in [0, 4], [0, 0.5] for Phong)
        const float etaChk = intIOR / extIOR < 1 ? extIOR / intIOR : intIOR / extIOR;
        if (etaChk < 1.0001f || etaChk > 4.0f)
            throw err("Error: the requested relative index of refraction is out of the supported range [1.0001, 4]");
        const float alphaMax = d.distribution == MTSG_MF_PHONG ? 0.5f : 4.0f;   // phong.dat covers [0, 0.5]
        if (d.alpha_u > alphaMax)
            throw err("Error: the requested roughness value is out of the supported range");
        V3 sr = energyConserving(props, props.getSpectrum("specularReflectance", V3(1.0f)));
        float dmx;
        const int tex = texturedParam(textures, {"diffuseReflectance"}, type, line, nTex);
        V3 dr = reflectance(props, tex, props.getSpectrum("diffuseReflectance", V3(0.5f)), d, dmx);
        d.type = MTSG_BSDF_ROUGHPLASTIC;
        d.ior_eta = intIOR / extIOR;
        d.ior_inv_eta = 1 / d.ior_eta;
        d.nonlinear = props.getBool("nonlinear", false) ? 1 : 0;
        const float dAvg = luminance(dr), sAvg = luminance(sr);
        d.spec_sampling_weight = sAvg / (dAvg + sAvg);
        for (int i = 0; i < 3; ++i) { d.spec_refl[i] = sr[i]; d.reflectance[i] = dr[i]; }
        // external slice at (eta, alpha); internal diffuse transmittance at 1/eta
        roughTransmittanceSlice(d.distribution, d.alpha_u, d.ior_eta, MTSG_RTRANS_SAMPLES, d.rtrans);
        d.fdr_int = 1 - roughDiffuseTransmittance(d.distribution, d.alpha_u, d.ior_inv_eta);
        d.smooth = 1;        // glossy + diffuse components
        d.ref_n_zero = 0;
    } else if (type == "twosided") {
        // twosided.cpp:52-80: one or two nested BRDFs, front and back
        texturedParam(textures, {}, type, line, nTex);
        if (nested.empty()) throw err("A nested one-sided material is required!");
        if (nested.size() > 2) throw err("No more than two nested BRDFs can be added!");
        for (int k : nested) {
            if (k < 0 || k >= (int)scene.bsdfs.size()) throw err("twosided: invalid nested BSDF id");
            const mtsg_bsdf &kd = scene.bsdfs[k].d;
            if (kd.type == MTSG_BSDF_DIELECTRIC || kd.type == MTSG_BSDF_ROUGHDIELECTRIC)
                throw err("Only materials without a transmission component can be nested!");
            if (kd.twosided) throw err("twosided: a nested twosided material is not supported by this build");
        }
        const int backIdx = nested.size() == 2 ? nested[1] : nested[0];
        d = scene.bsdfs[nested[0]].d;
        d.twosided = 1;
        d.back = backIdx;
        d.smooth = scene.bsdfs[nested[0]].d.smooth || scene.bsdfs[backIdx].d.smooth;
        d.ref_n_zero = 1;    // EBackSide component (records.inl:160-164)
    } else {
        throw err(at(line) + "BSDF plugin \"" + type + "\" is outside this build's scope");
    }
    scene.bsdfs.push_back(b);
    return (int)scene.bsdfs.size() - 1;
}

int SceneBuilder::defaultBsdf(bool emitter) {
    // Shape::configure (src/librender/shape.cpp:47-70): all-absorbing
    // diffuse on emitters, 0.5 Lambertian otherwise
    Bsdf b;
    float r = emitter ? 0.0f : 0.5f;
    b.d.type = MTSG_BSDF_DIFFUSE;
    b.d.reflectance[0] = b.d.reflectance[1] = b.d.reflectance[2] = r;
    b.d.smooth = r > 0;
    scene.bsdfs.push_back(b);
    return (int)scene.bsdfs.size() - 1;
}

int SceneBuilder::emitter(const std::string &type_, const Properties &props, int line) {
    const std::string type = lower(type_);
    if (type == "area") {
        // AreaLight(props) (area.cpp:67-78): attached to the shape that names it
        if (props.transforms.count("toWorld"))
            throw err("Found a 'toWorld' transformation -- this is not allowed -- the area light inherits this transformation from its parent shape");
        Emitter e;
        e.radiance = props.getSpectrum("radiance", V3(1.0f));   // D65 == 1 in RGB mode
        e.samplingWeight = props.getFloat("samplingWeight", 1.0f);
        scene.emitters.push_back(e);
        return (int)scene.emitters.size() - 1;
    }
    if (type != "envmap")
        throw err(at(line) + "emitter plugin \"" + type + "\" is outside this build's scope (only 'area' and 'envmap')");
    // EnvironmentMap(props) (envmap.cpp:105-185)
    for (auto &e : scene.emitters)
        if (e.type == MTSG_EMITTER_ENVMAP) throw err("only one environment emitter is supported (Scene::m_environmentEmitter)");
    Emitter e;
    e.type = MTSG_EMITTER_ENVMAP;
    e.samplingWeight = props.getFloat("samplingWeight", 1.0f);
    e.scale = props.getFloat("scale", 1.0f);
    if (props.has("intensityScale")) throw err("The 'intensityScale' parameter has been deprecated and is now called scale.");
    e.toWorld = props.getTransform("toWorld", Transform());
    std::string file = props.getString("filename", "");
    if (file.empty()) throw err("envmap: missing 'filename'");
    std::string path = resolve(file);
    std::string ext = lower(path.size() > 4 ? path.substr(path.size() - 4) : path);
    std::string e2;
    if (ext == ".pfm") {
        if (!readPFM(path, e.width, e.height, e.rgb, e2)) throw err("envmap \"" + file + "\": " + e2);
    } else if (ext == ".exr") {
        if (!readEXR(path, e.width, e.height, e.rgb, e2)) throw err("envmap \"" + file + "\": " + e2);
    } else {
        throw err("envmap \"" + file + "\": only OpenEXR and PFM images are supported by this build");
    }
    if (std::max(e.width, e.height) > 0xFFFF) throw err("Environment maps images must be smaller than 65536 pixels in width and height");
    scene.emitters.push_back(std::move(e));
    return (int)scene.emitters.size() - 1;
}

void SceneBuilder::checkEmitter(int emitter, bool inGroup, bool claim) {
    if (emitter < 0) return;
    if (inGroup) throw err("emitters inside shapegroups are not supported");
    if (emitter >= (int)scene.emitters.size() || scene.emitters[emitter].type != MTSG_EMITTER_AREA)
        throw err("a shape's emitter must be an 'area' emitter");
    if (scene.emitters[emitter].shape >= 0 || claimed.count(emitter))
        throw err("an area emitter can only be attached to one shape");
    if (claim) claimed.insert(emitter);
}

int SceneBuilder::group(const std::string &id) {
    if (id.empty()) throw err("shapegroup needs an id");
    ShapeGroup g;
    g.id = id;
    if (scene.twoLevel) {
        // ShapeGroup::addChild / configure (shapegroup.cpp:94-138): the
        // group's shapes get their own kd-tree in group space
        g.index = (int)scene.groups.size();
        GroupDef gd;
        gd.id = id;
        scene.groups.push_back(std::move(gd));
    }
    groups.push_back(std::move(g));
    return (int)groups.size() - 1;
}

ShapeGroup &SceneBuilder::groupAt(int group) {
    if (group < 0 || group >= (int)groups.size()) throw err("invalid shape group id");
    return groups[group];
}

void SceneBuilder::addRect(Rect r, int group) {
    if (group < 0) {
        scene.rects.push_back(r);
        const int si = (int)scene.shapes.size();
        scene.shapes.push_back({MTSG_SHAPE_RECT, (int)scene.rects.size() - 1});
        if (r.emitter >= 0) scene.emitters[r.emitter].shape = si;
        return;
    }
    ShapeGroup &g = groupAt(group);
    if (scene.twoLevel)
        throw err("shapegroup \"" + g.id + "\": rectangles inside shape groups are outside the two-level "
                  "variant of this build (use the flattening mode)");
    g.rects.push_back(r);
}

void SceneBuilder::addMesh(Mesh &&m, int group) {
    if (m.idx.empty() || m.idx.size() % 3) throw err("\"" + m.name + "\": a triangle mesh needs 3 indices per triangle");
    for (uint32_t i : m.idx)
        if (i >= m.p.size()) throw err("\"" + m.name + "\": triangle index out of range");
    if (group < 0) {
        scene.meshes.push_back(std::move(m));
        const int si = (int)scene.shapes.size();
        scene.shapes.push_back({MTSG_SHAPE_MESH, (int)scene.meshes.size() - 1});
        if (scene.meshes.back().emitter >= 0) scene.emitters[scene.meshes.back().emitter].shape = si;
        return;
    }
    ShapeGroup &g = groupAt(group);
    if (scene.twoLevel) {
        m.group = g.index;
        scene.meshes.push_back(std::move(m));
        scene.groups[g.index].shapes.push_back((int)scene.shapes.size());
        scene.shapes.push_back({MTSG_SHAPE_MESH, (int)scene.meshes.size() - 1});
    } else {
        g.meshes.push_back(std::move(m));   // object space, transformed per instance
    }
}

// TriMesh arrays as Mitsuba holds them after TriMesh::configure
// (trimesh.cpp:362-386): toWorld (if any) is applied to positions and
// normals, then computeNormals (trimesh.cpp:608-681) computes missing vertex
// normals or flips given ones (flipNormals)
void SceneBuilder::mesh(Mesh &&m, const Transform *toWorld, bool flip, int bsdf, int emitter, int group) {
    checkEmitter(emitter, group >= 0, true);
    if (bsdf >= (int)scene.bsdfs.size()) throw err("invalid BSDF id");
    if (bsdf < 0) bsdf = defaultBsdf(emitter >= 0);
    if (toWorld) {
        for (auto &p : m.p) p = toWorld->point(p);
        for (auto &nn : m.n) nn = normalize(toWorld->normal(nn));
    }
    computeNormals(m, flip);
    m.bsdf = bsdf;
    m.emitter = emitter;
    addMesh(std::move(m), group);
}

void SceneBuilder::shape(const std::string &type_, const Properties &props, int bsdf, int emitter, int group, int line) {
    const std::string type = lower(type_);
    if (type == "shapegroup" || type == "instance")
        throw err(at(line) + "'" + type + "' is built with mtsh_scene_add_group / mtsh_scene_add_instance");
    checkEmitter(emitter, group >= 0, type == "rectangle");   // meshes claim it in mesh()
    if (bsdf >= (int)scene.bsdfs.size()) throw err("invalid BSDF id");
    const Transform toWorld = props.getTransform("toWorld", Transform());
    const bool flip = props.getBool("flipNormals", false);
    if (type == "rectangle") {
        // Rectangle(props) (rectangle.cpp:57-76): flipNormals mirrors z
        if (bsdf < 0) bsdf = defaultBsdf(emitter >= 0);
        Rect r;
        r.toWorld = toWorld;
        if (flip) r.toWorld = r.toWorld * Transform::scale(V3(1, 1, -1));
        r.bsdf = bsdf;
        r.emitter = emitter;
        addRect(r, group);
        return;
    }
    Mesh m;
    if (type == "ply") {
        loadPLY(resolve(props.getString("filename", "")), m);
    } else if (type == "obj") {
        loadOBJ(resolve(props.getString("filename", "")), m, props.getBool("flipTexCoords", true));
    } else if (type == "cube") {
        buildCube(m);
    } else if (type == "serialized") {
        // serialized.cpp:146-196: the file's face-normal flag is overridden
        // by the property; an orientation-reversing toWorld swaps the
        // first two indices of every triangle
        if (props.has("maxSmoothAngle"))
            throw err("serialized: 'maxSmoothAngle' (TriMesh::rebuildTopology) is outside this build's scope");
        loadSerialized(resolve(props.getString("filename", "")), (int)props.getInt("shapeIndex", 0), m);
        const auto &M = toWorld.m;
        const double det = (double)M[0][0] * ((double)M[1][1] * M[2][2] - (double)M[1][2] * M[2][1]) -
                           (double)M[0][1] * ((double)M[1][0] * M[2][2] - (double)M[1][2] * M[2][0]) +
                           (double)M[0][2] * ((double)M[1][0] * M[2][1] - (double)M[1][1] * M[2][0]);
        if (det < 0)
            for (size_t t = 0; t + 2 < m.idx.size(); t += 3) std::swap(m.idx[t], m.idx[t + 1]);
    } else {
        throw err(at(line) + "shape plugin \"" + type + "\" is outside this build's scope");
    }
    m.faceNormals = props.getBool("faceNormals", false);
    mesh(std::move(m), &toWorld, flip, bsdf, emitter, group);
}

void SceneBuilder::instance(int group, const Transform &toWorld) {
    const ShapeGroup &g = groupAt(group);
    if (scene.twoLevel) {
        // Instance (instance.cpp:57-130): a top-level primitive that
        // transforms rays into the group's space
        InstanceDef idf;
        idf.group = g.index;
        idf.toWorld = toWorld;
        scene.instances.push_back(idf);
        scene.shapes.push_back({MTSG_SHAPE_INSTANCE, (int)scene.instances.size() - 1});
        return;
    }
    // flattened: the group's shapes in world space join the scene
    for (const Mesh &m0 : g.meshes) {
        Mesh m = m0;
        m.instanced = true;   // an Instance in the reference: not one of Scene::getMeshes()
        for (auto &p : m.p) p = toWorld.point(p);
        for (auto &nn : m.n) nn = normalize(toWorld.normal(nn));
        addMesh(std::move(m), -1);
    }
    for (const Rect &r0 : g.rects) {
        Rect r = r0;
        r.toWorld = toWorld * r0.toWorld;
        addRect(r, -1);
    }
}

void SceneBuilder::buildCube(Mesh &m) {
    // src/shapes/cube.cpp:24-30 data, restated as 6 faces of 4 vertices
    // with per-face normals and [0,1]^2 texcoords
    static const float P[24][3] = {
        {1, -1, -1}, {1, -1, 1}, {-1, -1, 1}, {-1, -1, -1}, {1, 1, -1}, {-1, 1, -1}, {-1, 1, 1}, {1, 1, 1},
        {1, -1, -1}, {1, 1, -1}, {1, 1, 1}, {1, -1, 1}, {1, -1, 1}, {1, 1, 1}, {-1, 1, 1}, {-1, -1, 1},
        {-1, -1, 1}, {-1, 1, 1}, {-1, 1, -1}, {-1, -1, -1}, {1, 1, -1}, {1, -1, -1}, {-1, -1, -1}, {-1, 1, -1}};
    static const float N[24][3] = {
        {0, -1, 0}, {0, -1, 0}, {0, -1, 0}, {0, -1, 0}, {0, 1, 0}, {0, 1, 0}, {0, 1, 0}, {0, 1, 0},
        {1, 0, 0}, {1, 0, 0}, {1, 0, 0}, {1, 0, 0}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1},
        {-1, 0, 0}, {-1, 0, 0}, {-1, 0, 0}, {-1, 0, 0}, {0, 0, -1}, {0, 0, -1}, {0, 0, -1}, {0, 0, -1}};
    static const float T[24][2] = {
        {0, 1}, {1, 1}, {1, 0}, {0, 0}, {0, 1}, {1, 1}, {1, 0}, {0, 0}, {0, 1}, {1, 1}, {1, 0}, {0, 0},
        {0, 1}, {1, 1}, {1, 0}, {0, 0}, {0, 1}, {1, 1}, {1, 0}, {0, 0}, {0, 1}, {1, 1}, {1, 0}, {0, 0}};
    for (int i = 0; i < 24; ++i) {
        m.p.emplace_back(P[i][0], P[i][1], P[i][2]);
        m.n.emplace_back(N[i][0], N[i][1], N[i][2]);
        m.uv.push_back(T[i][0]);
        m.uv.push_back(T[i][1]);
    }
    for (uint32_t f = 0; f < 6; ++f) {
        uint32_t b = 4 * f;
        m.idx.insert(m.idx.end(), {b + 0, b + 1, b + 2, b + 3, b + 0, b + 2});
    }
}

void SceneBuilder::integrator(const std::string &type, const Properties &props, int line) {
    IntegratorProps &ip = scene.integrator;
    if (type == "myPath2_OM") {
        // myPath2OMIntegrator(props) (myPath2_OM.cpp:61-85)
        ip = IntegratorProps();
        ip.type = type;
        ip.maxDepth = (int)props.getInt("maxDepthEye", 50);
        ip.rrDepth = 1;
        const std::string st = props.getString("strategy", "mis"), mm = props.getString("MISmode", "balance");
        if (st == "bsdf") ip.omStrategy = MTSG_OM_STRATEGY_BSDF;
        else if (st == "nee") ip.omStrategy = MTSG_OM_STRATEGY_NEE;
        else if (st == "mis") ip.omStrategy = MTSG_OM_STRATEGY_MIS;
        else throw err("Unknown strategy: " + st);
        if (mm == "uniform") ip.omMis = MTSG_OM_MIS_UNIFORM;
        else if (mm == "balance") ip.omMis = MTSG_OM_MIS_BALANCE;
        else if (mm == "power") ip.omMis = MTSG_OM_MIS_POWER;
        else throw err("Unknown MIS mode: " + mm);
        ip.omJitter = props.getBool("jitterSample", true);
        if (ip.maxDepth < 1) throw err("myPath2_OM: 'maxDepthEye' must be at least 1");
        return;
    }
    const std::string t = lower(type);
    if (t != "path") throw err(at(line) + "integrator \"" + t + "\" is outside this build's scope (only 'path' and 'myPath2_OM')");
    // MonteCarloIntegrator(props) (integrator.cpp:199-234)
    ip = IntegratorProps();
    ip.type = t;
    ip.rrDepth = (int)props.getInt("rrDepth", 5);
    ip.maxDepth = (int)props.getInt("maxDepth", -1);
    ip.strictNormals = props.getBool("strictNormals", false);
    ip.hideEmitters = props.getBool("hideEmitters", false);
    if (ip.rrDepth <= 0) throw err("'rrDepth' must be set to a value greater than zero!");
    if (ip.maxDepth <= 0 && ip.maxDepth != -1) throw err("'maxDepth' must be set to -1 (infinite) or a value greater than zero!");
}

void SceneBuilder::sensor(const std::string &type_, const Properties &props, int line) {
    const std::string type = lower(type_);
    if (type != "perspective") throw err(at(line) + "sensor \"" + type + "\" is outside this build's scope");
    Sensor &s = scene.sensor;
    s.present = true;
    s.toWorld = props.getTransform("toWorld", Transform());
    s.nearClip = props.getFloat("nearClip", 1e-2f);
    s.farClip = props.getFloat("farClip", 1e4f);
    if (s.nearClip <= 0) throw err("The 'nearClip' parameter must be greater than zero!");
    if (s.nearClip >= s.farClip) throw err("The 'nearClip' parameter must be smaller than 'farClip'.");
    if (props.has("fov")) s.fov = props.getFloat("fov");
    else if (props.strings.count("focalLength")) throw err("focalLength is not supported by this loader; use fov");
    else s.fov = -1;  // default focal length 50mm handled in finalize
    s.fovAxis = lower(props.getString("fovAxis", "x"));
}

void SceneBuilder::sampler(const std::string &type, const Properties &sp) {
    const std::string st = lower(type);
    mtsg_sampler &smp = scene.sampler;
    scene.sampleCount = (int)sp.getInt("sampleCount", 4);
    if (st == "independent") {
        smp.type = MTSG_SAMPLER_INDEPENDENT;
    } else if (st == "halton" || st == "hammersley") {
        // halton.cpp:113-121, hammersley.cpp:93-101
        smp.type = st == "halton" ? MTSG_SAMPLER_HALTON : MTSG_SAMPLER_HAMMERSLEY;
        smp.scramble = (int)sp.getInt("scramble", -1);
    } else if (st == "ldsampler") {
        // ldsampler.cpp:82-95: the count is rounded up to a power of two
        smp.type = MTSG_SAMPLER_LDSAMPLER;
        smp.dimension = (int)sp.getInt("dimension", 4);
        if (smp.dimension < 0) throw err("ldsampler: 'dimension' must be >= 0");
        uint32_t c = (uint32_t)std::max(1, scene.sampleCount), r = 1;
        while (r < c) r <<= 1;
        scene.sampleCount = (int)r;
    } else if (st == "sobol") {
        // sobol.cpp:86-107
        smp.type = MTSG_SAMPLER_SOBOL;
        scene.sobolScrambleProp = (uint64_t)sp.getInt("scramble", 0);
    } else {
        throw err("sampler \"" + st + "\" is outside this build's scope "
                  "(independent, halton, hammersley, ldsampler, sobol)");
    }
    if (scene.sampleCount <= 0) throw err("sampleCount must be > 0");
    scene.samplerType = st;
}

void SceneBuilder::film(const std::string &type_, const Properties &props) {
    const std::string type = lower(type_);
    if (type != "hdrfilm") throw err("film \"" + type + "\" is outside this build's scope (only 'hdrfilm')");
    Film &f = scene.film;
    const std::string filter = f.filter;
    const float stddev = f.stddev, radius = f.boxRadius;
    f = Film();
    f.filter = filter; f.stddev = stddev; f.boxRadius = radius;   // an rfilter given before the film's values stays
    f.width = (int)props.getInt("width", 768);
    f.height = (int)props.getInt("height", 576);
    f.cropX = (int)props.getInt("cropOffsetX", 0);
    f.cropY = (int)props.getInt("cropOffsetY", 0);
    f.cropW = (int)props.getInt("cropWidth", f.width);
    f.cropH = (int)props.getInt("cropHeight", f.height);
    f.pixelFormat = lower(props.getString("pixelFormat", "rgb"));
    f.hasAlpha = f.pixelFormat.find('a') != std::string::npos;
}

void SceneBuilder::rfilter(const std::string &type_, const Properties &fp) {
    const std::string ft = lower(type_);
    Film &f = scene.film;
    if (ft == "gaussian") { f.filter = ft; f.stddev = fp.getFloat("stddev", 0.5f); }
    else if (ft == "box") { f.filter = ft; f.boxRadius = fp.getFloat("radius", 0.5f); }
    else throw err("rfilter \"" + ft + "\" is outside this build's scope");
}

void SceneBuilder::finish(const mtsh_scene_overrides *ov) {
    if (!scene.sensor.present) throw err("scene has no <sensor>");
    for (auto &e : scene.emitters)
        if (e.type == MTSG_EMITTER_AREA && e.shape < 0) throw err("area emitter without a parent shape");
    if (ov) {
        // the in-memory values of a Mitsuba plugin (mtsh.h mtsh_scene_overrides)
        if (ov->mask & (MTSH_OVERRIDE_FILM_SIZE | MTSH_OVERRIDE_FILM_CROP)) {
            Film &f = scene.film;
            if (ov->mask & MTSH_OVERRIDE_FILM_SIZE) {
                if (ov->film_width <= 0 || ov->film_height <= 0) throw err("override: film size must be positive");
                // a new size without a crop: the crop is the whole film (the
                // XML's crop no longer fits a film of another size)
                if (!(ov->mask & MTSH_OVERRIDE_FILM_CROP) &&
                    (f.cropX != 0 || f.cropY != 0 || f.cropW != f.width || f.cropH != f.height) &&
                    (ov->film_width != f.width || ov->film_height != f.height))
                    throw err("override: the film size changes but the XML's crop window is kept; pass the crop "
                              "(MTSH_OVERRIDE_FILM_CROP) too");
                if (!(ov->mask & MTSH_OVERRIDE_FILM_CROP) && f.cropW == f.width && f.cropH == f.height) {
                    f.cropW = ov->film_width;
                    f.cropH = ov->film_height;
                }
                f.width = ov->film_width;
                f.height = ov->film_height;
            }
            if (ov->mask & MTSH_OVERRIDE_FILM_CROP) {
                f.cropX = ov->crop_x;
                f.cropY = ov->crop_y;
                f.cropW = ov->crop_width;
                f.cropH = ov->crop_height;
            }
        }
        if (ov->mask & MTSH_OVERRIDE_SAMPLE_COUNT) {
            if (ov->sample_count <= 0) throw err("sampleCount must be > 0");
            scene.sampleCount = ov->sample_count;
            if (scene.sampler.type == MTSG_SAMPLER_LDSAMPLER) {   // ldsampler.cpp:82-95
                uint32_t r = 1;
                while (r < (uint32_t)ov->sample_count) r <<= 1;
                scene.sampleCount = (int)r;
            }
        }
        if (ov->mask & MTSH_OVERRIDE_INTEGRATOR) {
            IntegratorProps &ip = scene.integrator;
            if (ip.type != "path") throw err("integrator overrides apply to the `path` integrator");
            // MonteCarloIntegrator's own checks (integrator.cpp:184-196)
            if (ov->rr_depth <= 0) throw err("'rrDepth' must be set to a value greater than zero!");
            if (ov->max_depth <= 0 && ov->max_depth != -1) throw err("'maxDepth' must be set to -1 (infinite) or a value greater than zero!");
            ip.maxDepth = ov->max_depth;
            ip.rrDepth = ov->rr_depth;
            ip.strictNormals = ov->strict_normals != 0;
            ip.hideEmitters = ov->hide_emitters != 0;
        }
    }
    scene.finalize();
}

}  // namespace mtsh
