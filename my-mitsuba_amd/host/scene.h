// Host-side scene model: the Mitsuba-mirror side of the drop-in boundary.
// It stands in for the parts of Mitsuba that stay on the CPU in the
// reference (XML SceneHandler, shape plugins, Scene::initialize, the SAH
// kd-tree build) and produces the flat mtsg_scene_desc handed to libmtsg.
#pragma once
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "hmath.h"
#include "../../include/mtsg.h"
#include "../../include/mtsh.h"

namespace mtsh {

struct Properties {
    // typed property bag (include/mitsuba/core/properties.h)
    std::map<std::string, float> floats;
    std::map<std::string, long long> ints;
    std::map<std::string, bool> bools;
    std::map<std::string, std::string> strings;
    std::map<std::string, V3> spectra;   // RGB mode: 3 samples
    std::map<std::string, V3> points;
    std::map<std::string, Transform> transforms;
    std::map<std::string, bool> queried;

    bool has(const std::string &n) const {
        return floats.count(n) || ints.count(n) || bools.count(n) || strings.count(n) ||
               spectra.count(n) || points.count(n) || transforms.count(n);
    }
    float getFloat(const std::string &n, float def) const;
    float getFloat(const std::string &n) const;
    long long getInt(const std::string &n, long long def) const;
    bool getBool(const std::string &n, bool def) const;
    std::string getString(const std::string &n, const std::string &def) const;
    V3 getSpectrum(const std::string &n, const V3 &def) const;
    Transform getTransform(const std::string &n, const Transform &def) const;
};

struct Mesh {
    std::string name;
    std::vector<V3> p, n;            // n empty when faceNormals
    std::vector<float> uv;           // 2 per vertex, may be empty
    std::vector<uint32_t> idx;       // 3 per triangle
    bool faceNormals = false;
    int bsdf = -1, emitter = -1;
    int group = -1;                  // two-level: the shape group it belongs to (group space)
    bool instanced = false;          // flattened from an instance (not a Scene::getMeshes() TriMesh)
};

struct Rect {
    Transform toWorld;
    int bsdf = -1, emitter = -1;
};

struct Bsdf {
    mtsg_bsdf d{};
    std::string id;
};

struct Emitter {
    int type = MTSG_EMITTER_AREA;
    V3 radiance{1, 1, 1};
    float samplingWeight = 1.0f;
    int shape = -1;                  // index into Scene::shapes (area lights)
    // envmap (src/emitters/envmap.cpp)
    int width = 0, height = 0;       // level-0 size
    std::vector<float> rgb;          // level 0, RGB float, top row first (after the PFM flip)
    float scale = 1.0f;
    Transform toWorld;
};

// `bitmap` texture (src/textures/bitmap.cpp): its pyramid lives in
// Scene::texTexels, the header in desc
struct Texture {
    std::string id;
    mtsg_texture d{};
};

struct ShapeRef {                    // m_shapes order in the kd-tree
    int type;                        // MTSG_SHAPE_*
    int index;                       // into meshes / rects / instances
};

// Two-level instancing (src/shapes/shapegroup.cpp, instance.cpp)
struct GroupDef {
    std::string id;
    std::vector<int> shapes;         // its meshes' entries in Scene::shapes
};
struct InstanceDef {
    int group = -1;
    Transform toWorld;
};

struct Sensor {
    Transform toWorld;
    float fov = -1;
    std::string fovAxis = "x";
    float nearClip = 1e-2f, farClip = 1e4f;
    bool present = false;
};

struct Film {
    int width = 768, height = 576;
    int cropX = 0, cropY = 0, cropW = -1, cropH = -1;
    std::string filter = "gaussian";
    float stddev = 0.5f, boxRadius = 0.5f;
    bool hasAlpha = false;
    std::string pixelFormat = "rgb";
};

struct IntegratorProps {
    std::string type = "path";
    int maxDepth = -1, rrDepth = 5;
    bool strictNormals = false, hideEmitters = false;
    // myPath2_OM (myPath2_OM.cpp:61-85)
    int omStrategy = MTSG_OM_STRATEGY_MIS, omMis = MTSG_OM_MIS_BALANCE;
    bool omJitter = true;
};

struct KDBuildParams {                // gkdtree.h:734-744 defaults, except stopPrims
    float traversalCost = 15, queryCost = 20, emptySpaceBonus = 0.9f;
    // stopPrims: 4 instead of Mitsuba's 6 (gkdtree.h:738).  The GPU traversal
    // tests one primitive per iteration while it descends, so a primitive test
    // costs it more, relative to a node step, than Mitsuba's cost model
    // assumes: C3 1501 -> 1538 Msamples/s (5.99 instead of 7.24 tests per ray,
    // DESIGN §3).  Hits do not depend on the tree; the scene's kdStopPrims
    // property (scene.cpp:64) sets it, e.g. 6 for Mitsuba's own tree (the CPU
    // baseline in bench.py is timed on that one).
    int stopPrims = 4, maxBadRefines = 3, minMaxBins = 128;
    int exactPrimThreshold = 65536;
    int exactSweepLimit = 65536;      // exact O(n log n) sweep below exactPrimThreshold (gkdtree.h:980, 1510), binned above
    bool clip = true;
    bool retract = true;              // m_retract (gkdtree.h:742)
    int maxDepth = 0;                 // 0 = 8 + 1.3 log2(N) (gkdtree.h:986-988)
    int threads = 0;                  // 0 = hardware concurrency
};

struct KDTree {
    std::vector<mtsg_kdnode> nodes;
    std::vector<uint32_t> indices;
    AABB aabb;                         // enlarged
    AABB tightAABB;
    uint32_t maxDepth = 0;
    double buildSeconds = 0;
    double sahCost = 0;
    size_t leafCount = 0, nonEmptyLeaves = 0, retractedSplits = 0;
};

struct Scene {
    std::vector<Mesh> meshes;
    std::vector<Rect> rects;
    std::vector<ShapeRef> shapes;     // in kd-tree order
    std::vector<GroupDef> groups;     // two-level instancing only
    std::vector<InstanceDef> instances;
    std::vector<Bsdf> bsdfs;
    std::vector<Emitter> emitters;
    std::vector<Texture> textures;
    std::vector<float> texTexels;     // all textures' MIP levels (half-rounded RGB)
    Sensor sensor;
    Film film;
    IntegratorProps integrator;
    int sampleCount = 4;
    bool twoLevel = false;            // MTSH_INSTANCING_TWO_LEVEL
    std::string samplerType = "independent";
    mtsg_sampler sampler{MTSG_SAMPLER_INDEPENDENT, -1, 4, 0};
    uint64_t sobolScrambleProp = 0;   // sobol 'scramble' (before TEA)
    KDBuildParams kd;                 // the scene's tree (its <scene> kd* properties)
    KDBuildParams groupKd;            // shape groups' trees (defaults, shapegroup.cpp:74)

    // ---- flattened (filled by finalize()) ----
    std::vector<float> vtxPos, vtxNrm, triDpdu, emitterCdf, emitterTriCdf;
    std::vector<float> triUv, triDpdv;   // only with textures
    std::vector<mtsg_texture> textureDesc;
    mtsg_om omDesc{};                 // myPath2_OM only
    std::vector<uint32_t> omBits;
    std::vector<uint32_t> triIdx;
    std::vector<mtsg_rect> rectDesc;
    std::vector<mtsg_shape> shapeDesc;
    std::vector<mtsg_bsdf> bsdfDesc;
    std::vector<mtsg_emitter> emitterDesc;
    std::vector<mtsg_triaccel> triaccel;
    std::vector<float> envTexels, envCdfRows, envCdfCols, envRowWeights;
    std::vector<uint32_t> qmcPrimes, qmcOffsets;
    std::vector<uint16_t> qmcPerm;
    KDTree tree;
    std::vector<KDTree> groupTrees;
    std::vector<mtsg_instance> instanceDesc;
    std::vector<mtsg_group> groupDesc;
    std::vector<mtsg_kdnode> groupNodes;
    std::vector<uint32_t> groupIndices;
    mtsg_camera camera{};
    mtsg_scene_desc desc{};

    std::vector<uint8_t> triGrouped;  // triangle lives in a shape group's own tree (two-level)

    void finalize();                  // normals, tangents, CDFs, kd-tree, desc
    void primBounds(std::vector<float> &out) const;
    void setTree(const mtsg_kdnode *nodes, uint32_t nNodes, const uint32_t *indices, uint32_t nIndices, const float *aabbMin,
                 const float *aabbMax, uint32_t maxDepth);
};

extern int g_defaultKDThreads;   // 0 = hardware concurrency
extern int g_instancing;         // MTSH_INSTANCING_* of the next load

// Environment emitter tables (envmap.cpp in this directory)
void buildEnvmap(const Emitter &e, const float aabbMin[3], const float aabbMax[3], const float camPos[3],
                 std::vector<float> &texels, std::vector<float> &cdfRows, std::vector<float> &cdfCols,
                 std::vector<float> &rowWeights, mtsg_envmap &env);

// MIP pyramids (mipmap.cpp): TMIPMap over a linear float RGB level 0
// (3 floats per texel, rows top-down); levels are appended to `texels` with
// offsets relative to its start.  average / maximum: level-0 statistics
// after clamping negative values (may be null).
void buildMipmap(std::vector<float> level0, int w, int h, int filter, int wrapU, int wrapV, float maxValue,
                 float maxAnisotropy, std::vector<float> &texels, mtsg_mipmap &mip, float average[3], float maximum[3]);
float toHalfAndBack(float f);
// PNG image: samples (8- or 16-bit) per channel, palette expanded, gamma as
// Bitmap::readPNG sets it (-1 = sRGB)
struct PngImage {
    int width = 0, height = 0, channels = 0, depth = 8;
    float gamma = -1.0f;
    std::vector<uint16_t> samples;
};
bool readPNG(const std::string &path, PngImage &img, std::string &err);
// the bitmap plugin's input: linear float RGB, rows top-down
void loadTextureImage(const std::string &path, float gammaOverride, int &w, int &h, std::vector<float> &rgb);

// myPath2_OM's occupancy maps (om.cpp): fills omDesc / omBits
void buildOccupancyMaps(Scene &scene);

// Halton / Hammersley tables (qmc.cpp in this directory): the first 1024
// primes, offsets of each base's digit permutation, and the permutations
// (empty for scramble 0)
void buildQmcTables(int scramble, std::vector<uint32_t> &primes, std::vector<uint32_t> &offsets,
                    std::vector<uint16_t> &perm);

// Sobol' tables (qmc.cpp, embedded data of sobolseq.cpp) and the TEA'd scramble
uint64_t sobolScramble(uint64_t scramble);
void sobolTables(const uint32_t *&matrices, const uint64_t *&vdc, uint32_t &vdcRows, const uint64_t *&vdcInv,
                 uint32_t &vdcInvRows);

// PFM image (src/libcore/bitmap.cpp:3764-3814): RGB float, rows top-down
bool readPFM(const std::string &path, int &w, int &h, std::vector<float> &rgb, std::string &err);
// OpenEXR scanline image (Bitmap::readOpenEXR, bitmap.cpp:2780; exr.cpp):
// RGB float, rows top-down
bool readEXR(const std::string &path, int &w, int &h, std::vector<float> &rgb, std::string &err);

// A `shapegroup` being filled (src/shapes/shapegroup.cpp): flattening keeps
// its shapes in object space until an instance places a copy; the two-level
// mode sends them straight to Scene::meshes under Scene::groups[index]
struct ShapeGroup {
    std::string id;
    std::vector<Mesh> meshes;
    std::vector<Rect> rects;
    int index = -1;
};

// Plugin construction from Properties (builder.cpp), shared by the XML
// loader and the in-memory builder C-ABI (mtsh_scene_begin / _add_* /
// _finish).  Objects are created in the caller's order, which fixes the
// order of the descriptor's arrays; ids are indices into the scene's
// bsdfs / emitters / textures, and into this builder's shape groups.
// `line` (> 0) prefixes error messages with an XML line number.
class SceneBuilder {
public:
    explicit SceneBuilder(Scene &s);
    static std::unique_ptr<Scene> newScene();   // instancing mode, kd build parameters
    std::vector<std::string> dirStack;          // relative file names resolve against these, innermost last
    std::string resolve(const std::string &f) const;

    int texture(const std::string &type, const Properties &props, const std::string &id, int line = 0);
    // textures: BSDF parameter name -> texture id; nested: twosided's BSDFs
    int bsdf(const std::string &type, const Properties &props, const std::map<std::string, int> &textures,
             const std::vector<int> &nested, const std::string &id, int line = 0);
    int emitter(const std::string &type, const Properties &props, int line = 0);   // area (for a shape) or envmap
    // shapes: bsdf / emitter -1 = none; group -1 = the scene
    void shape(const std::string &type, const Properties &props, int bsdf, int emitter, int group, int line = 0);
    void mesh(Mesh &&m, const Transform *toWorld, bool flipNormals, int bsdf, int emitter, int group);
    int group(const std::string &id);
    void instance(int group, const Transform &toWorld);
    void integrator(const std::string &type, const Properties &props, int line = 0);
    void sensor(const std::string &type, const Properties &props, int line = 0);
    void film(const std::string &type, const Properties &props);
    void rfilter(const std::string &type, const Properties &props);
    void sceneProps(const Properties &props, int line = 0);   // Scene::Scene(props): kd build parameters
    void sampler(const std::string &type, const Properties &props);
    void finish(const mtsh_scene_overrides *overrides);   // validation, overrides, Scene::finalize

private:
    Scene &scene;
    std::vector<ShapeGroup> groups;
    std::set<int> claimed;   // area emitters attached to a shape
    V3 reflectance(const Properties &props, int tex, const V3 &constant, mtsg_bsdf &d, float &maxOut);
    int defaultBsdf(bool emitter);
    void checkEmitter(int emitter, bool inGroup, bool claim);
    ShapeGroup &groupAt(int group);
    void addRect(Rect r, int group);
    void addMesh(Mesh &&m, int group);
    static void buildCube(Mesh &m);
};

// XML loading (src/librender/scenehandler.cpp), `-D name=value` defines
std::unique_ptr<Scene> loadScene(const std::string &path,
                                 const std::map<std::string, std::string> &defines,
                                 const mtsh_scene_overrides *overrides = nullptr,
                                 const Properties *sceneProps = nullptr);

// Mesh loaders
void loadPLY(const std::string &path, Mesh &mesh);   // src/shapes/ply.cpp
void loadOBJ(const std::string &path, Mesh &mesh, bool flipTexCoords);  // src/shapes/obj.cpp
void loadSerialized(const std::string &path, int shapeIndex, Mesh &mesh);  // src/shapes/serialized.cpp

// TriMesh::computeNormals (src/librender/trimesh.cpp:608-681)
void computeNormals(Mesh &mesh, bool flipNormals);

// SAH kd-tree over `n` primitives with the given (clippable) geometry
struct PrimSource {
    virtual ~PrimSource() = default;
    virtual size_t count() const = 0;
    virtual AABB bounds(size_t i) const = 0;
    virtual AABB clippedBounds(size_t i, const AABB &box) const = 0;
};
void buildKDTree(const PrimSource &src, const KDBuildParams &params, KDTree &out);
AABB clipTriangle(const V3 &a, const V3 &b, const V3 &c, const AABB &box);   // build.cpp

// Conductor IOR lookup (generated from data/ior/*.spd), dielectric lookupIOR
bool lookupConductor(const std::string &name, V3 &eta, V3 &k);
float lookupIOR(const std::string &name);

// roughplastic: the material's slice of RoughTransmittance (rtrans.h),
// computed by quadrature (host/rtrans.cpp): T at cos(theta_k) = (k/(n-1))^4,
// and the diffuse (cosine-weighted hemispherical) transmittance
void roughTransmittanceSlice(int type, float alpha, float eta, int n, float *trans);
float roughDiffuseTransmittance(int type, float alpha, float eta);

// Film developing (hdrfilm.cpp:481-492, fmtconv.cpp:962-974) and PFM output
void writePFM(const std::string &path, int w, int h, const std::vector<float> &rgb);

}  // namespace mtsh
