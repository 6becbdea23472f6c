// Mitsuba 0.5/0.6 XML scene loading for the `path` hot path.
//
// Mirrors the SceneHandler semantics the configs need
// (reference src/librender/scenehandler.cpp:70-106 tag table, :461-625
// value tags, :700-780 object creation) and the shape/BSDF/emitter plugin
// constructors' parameter parsing:
//   shapes  ply (src/shapes/ply.cpp), obj (src/shapes/obj.cpp),
//           rectangle (src/shapes/rectangle.cpp), cube (src/shapes/cube.cpp),
//           shapegroup/instance (src/shapes/shapegroup.cpp, instance.cpp;
//           flattened into world-space meshes here)
//   bsdfs   diffuse (diffuse.cpp:75-84), roughconductor
//           (roughconductor.cpp:168-203, microfacet.h:99-146),
//           dielectric (dielectric.cpp:148-170)
//   emitter area (area.cpp:67-78)
//   sensor  perspective (perspective.cpp, sensor.cpp:150-262)
//   film    hdrfilm (hdrfilm.cpp:209-220), rfilter gaussian/box
//   sampler independent (independent.cpp:55-58), halton (halton.cpp:113-121),
//           hammersley (hammersley.cpp:93-101), ldsampler (ldsampler.cpp:82-95)
//   integrator path (integrator.cpp:199-234)
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <sstream>

#include <zlib.h>

#include "scene.h"

namespace mtsh {

// ---------------------------------------------------------------------------
// Properties
// ---------------------------------------------------------------------------
static std::runtime_error err(const std::string &m) { return std::runtime_error(m); }

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
// Minimal XML DOM
// ---------------------------------------------------------------------------
struct XNode {
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<XNode>> children;
    int line = 0;
    bool hasAttr(const std::string &k) const {
        for (auto &a : attrs) if (a.first == k) return true;
        return false;
    }
    std::string attr(const std::string &k, const std::string &def = "") const {
        for (auto &a : attrs) if (a.first == k) return a.second;
        return def;
    }
};

namespace {
struct XParser {
    const std::string &s;
    size_t i = 0;
    int line = 1;
    std::string file;
    explicit XParser(const std::string &src, const std::string &f) : s(src), file(f) {}
    [[noreturn]] void fail(const std::string &m) {
        throw err(file + ":" + std::to_string(line) + ": XML parse error: " + m);
    }
    void adv(size_t n = 1) {
        for (size_t k = 0; k < n && i < s.size(); ++k, ++i)
            if (s[i] == '\n') ++line;
    }
    bool starts(const char *p) const { return s.compare(i, strlen(p), p) == 0; }
    void ws() { while (i < s.size() && isspace((unsigned char)s[i])) adv(); }
    void skipMisc() {
        for (;;) {
            ws();
            if (starts("<!--")) {
                size_t e = s.find("-->", i);
                if (e == std::string::npos) fail("unterminated comment");
                adv(e + 3 - i);
            } else if (starts("<?")) {
                size_t e = s.find("?>", i);
                if (e == std::string::npos) fail("unterminated declaration");
                adv(e + 2 - i);
            } else if (starts("<!")) {
                size_t e = s.find('>', i);
                if (e == std::string::npos) fail("unterminated doctype");
                adv(e + 1 - i);
            } else {
                return;
            }
        }
    }
    static std::string unescape(const std::string &v) {
        std::string o;
        for (size_t k = 0; k < v.size(); ++k) {
            if (v[k] == '&') {
                size_t e = v.find(';', k);
                std::string ent = v.substr(k + 1, e - k - 1);
                if (ent == "lt") o += '<';
                else if (ent == "gt") o += '>';
                else if (ent == "amp") o += '&';
                else if (ent == "quot") o += '"';
                else if (ent == "apos") o += '\'';
                else o += "&" + ent + ";";
                k = e;
            } else {
                o += v[k];
            }
        }
        return o;
    }
    std::string name() {
        size_t b = i;
        while (i < s.size() && (isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == '-' || s[i] == ':' || s[i] == '.')) adv();
        if (b == i) fail("expected a name");
        return s.substr(b, i - b);
    }
    std::unique_ptr<XNode> element() {
        skipMisc();
        if (i >= s.size() || s[i] != '<') fail("expected '<'");
        adv();
        auto node = std::make_unique<XNode>();
        node->line = line;
        node->tag = name();
        for (;;) {
            ws();
            if (starts("/>")) { adv(2); return node; }
            if (starts(">")) { adv(); break; }
            std::string k = name();
            ws();
            if (i >= s.size() || s[i] != '=') fail("expected '=' after attribute " + k);
            adv(); ws();
            char q = s[i];
            if (q != '"' && q != '\'') fail("expected quoted attribute value");
            adv();
            size_t e = s.find(q, i);
            if (e == std::string::npos) fail("unterminated attribute value");
            std::string v = unescape(s.substr(i, e - i));
            adv(e + 1 - i);
            node->attrs.emplace_back(k, v);
        }
        for (;;) {
            // skip text content
            while (i < s.size() && s[i] != '<') adv();
            if (starts("<!--")) { skipMisc(); continue; }
            if (starts("</")) {
                adv(2);
                std::string n = name();
                if (n != node->tag) fail("mismatched </" + n + "> for <" + node->tag + ">");
                ws();
                if (s[i] != '>') fail("expected '>'");
                adv();
                return node;
            }
            if (i >= s.size()) fail("unexpected end of file inside <" + node->tag + ">");
            node->children.push_back(element());
        }
    }
};

std::string readFile(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw err("Unable to open \"" + path + "\"");
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

std::string dirName(const std::string &p) {
    size_t k = p.find_last_of('/');
    return k == std::string::npos ? std::string(".") : p.substr(0, k);
}

std::string lower(std::string s) {
    for (auto &c : s) c = (char)tolower((unsigned char)c);
    return s;
}

std::vector<std::string> tokenize(const std::string &s, const char *delims) {
    std::vector<std::string> out;
    std::string cur;
    for (char c : s) {
        if (strchr(delims, c)) {
            if (!cur.empty()) out.push_back(cur);
            cur.clear();
        } else {
            cur += c;
        }
    }
    if (!cur.empty()) out.push_back(cur);
    return out;
}

float parseF(const std::string &v, int line) {
    char *end = nullptr;
    std::string t = v;
    while (!t.empty() && isspace((unsigned char)t.back())) t.pop_back();
    size_t b = 0;
    while (b < t.size() && isspace((unsigned char)t[b])) ++b;
    t = t.substr(b);
    float f = strtof(t.c_str(), &end);
    if (t.empty() || *end != '\0') throw err("line " + std::to_string(line) + ": could not parse floating point value \"" + v + "\"");
    return f;
}
}  // namespace

// ---------------------------------------------------------------------------
// Mesh loaders
// ---------------------------------------------------------------------------
namespace {
struct PlyProp {
    std::string name, type, countType;
    bool list = false;
};
struct PlyElem {
    std::string name;
    size_t count = 0;
    std::vector<PlyProp> props;
};
size_t plyTypeSize(const std::string &t) {
    if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
    if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
    if (t == "int" || t == "uint" || t == "float" || t == "int32" || t == "uint32" || t == "float32") return 4;
    if (t == "double" || t == "float64") return 8;
    throw err("PLY: unknown property type " + t);
}
double plyRead(const unsigned char *p, const std::string &t, bool swap) {
    unsigned char b[8];
    size_t n = plyTypeSize(t);
    for (size_t k = 0; k < n; ++k) b[k] = swap ? p[n - 1 - k] : p[k];
    if (t == "char" || t == "int8") return (double)(int8_t)b[0];
    if (t == "uchar" || t == "uint8") return (double)b[0];
    if (t == "short" || t == "int16") { int16_t v; memcpy(&v, b, 2); return v; }
    if (t == "ushort" || t == "uint16") { uint16_t v; memcpy(&v, b, 2); return v; }
    if (t == "int" || t == "int32") { int32_t v; memcpy(&v, b, 4); return v; }
    if (t == "uint" || t == "uint32") { uint32_t v; memcpy(&v, b, 4); return v; }
    if (t == "float" || t == "float32") { float v; memcpy(&v, b, 4); return v; }
    double v; memcpy(&v, b, 8); return v;
}
}  // namespace

void loadPLY(const std::string &path, Mesh &mesh) {
    std::string data = readFile(path);
    size_t hdrEnd = data.find("end_header");
    if (data.compare(0, 3, "ply") != 0 || hdrEnd == std::string::npos)
        throw err("\"" + path + "\": not a PLY file");
    size_t bodyStart = data.find('\n', hdrEnd);
    if (bodyStart == std::string::npos) throw err("PLY: truncated header");
    ++bodyStart;
    std::istringstream hs(data.substr(0, hdrEnd));
    std::string line, format;
    std::vector<PlyElem> elems;
    while (std::getline(hs, line)) {
        auto tok = tokenize(line, " \t\r");
        if (tok.empty()) continue;
        if (tok[0] == "format") format = tok.at(1);
        else if (tok[0] == "element") { PlyElem e; e.name = tok.at(1); e.count = std::stoull(tok.at(2)); elems.push_back(e); }
        else if (tok[0] == "property") {
            if (elems.empty()) throw err("PLY: property before element");
            PlyProp p;
            if (tok.at(1) == "list") { p.list = true; p.countType = tok.at(2); p.type = tok.at(3); p.name = tok.at(4); }
            else { p.type = tok.at(1); p.name = tok.at(2); }
            elems.back().props.push_back(p);
        }
    }
    bool ascii = format == "ascii";
    bool swap = format == "binary_big_endian";
    if (!ascii && format != "binary_little_endian" && !swap) throw err("PLY: unknown format " + format);

    const unsigned char *p = (const unsigned char *)data.data() + bodyStart;
    const unsigned char *end = (const unsigned char *)data.data() + data.size();
    std::istringstream as(ascii ? data.substr(bodyStart) : std::string());

    bool hasN = false, hasUV = false;
    for (auto &e : elems) {
        if (e.name != "vertex") continue;
        for (auto &pr : e.props) {
            if (pr.name == "nx") hasN = true;
            if (pr.name == "u" || pr.name == "s" || pr.name == "texture_u" || pr.name == "texture_s") hasUV = true;
        }
    }
    auto readVal = [&](const std::string &t) -> double {
        if (ascii) { double v; if (!(as >> v)) throw err("PLY: truncated ascii body"); return v; }
        size_t n = plyTypeSize(t);
        if (p + n > end) throw err("PLY: truncated binary body");
        double v = plyRead(p, t, swap);
        p += n;
        return v;
    };
    for (auto &e : elems) {
        if (e.name == "vertex") {
            mesh.p.resize(e.count);
            if (hasN) mesh.n.resize(e.count);
            if (hasUV) mesh.uv.resize(2 * e.count);
            for (size_t v = 0; v < e.count; ++v) {
                for (auto &pr : e.props) {
                    if (pr.list) { size_t c = (size_t)readVal(pr.countType); for (size_t k = 0; k < c; ++k) readVal(pr.type); continue; }
                    double x = readVal(pr.type);
                    const std::string &nm = pr.name;
                    if (nm == "x") mesh.p[v].x = (float)x;
                    else if (nm == "y") mesh.p[v].y = (float)x;
                    else if (nm == "z") mesh.p[v].z = (float)x;
                    else if (nm == "nx") mesh.n[v].x = (float)x;
                    else if (nm == "ny") mesh.n[v].y = (float)x;
                    else if (nm == "nz") mesh.n[v].z = (float)x;
                    else if (nm == "u" || nm == "s" || nm == "texture_u" || nm == "texture_s") mesh.uv[2 * v] = (float)x;
                    else if (nm == "v" || nm == "t" || nm == "texture_v" || nm == "texture_t") mesh.uv[2 * v + 1] = (float)x;
                }
            }
        } else if (e.name == "face") {
            mesh.idx.reserve(e.count * 3);
            for (size_t f = 0; f < e.count; ++f) {
                for (auto &pr : e.props) {
                    if (!pr.list) { readVal(pr.type); continue; }
                    size_t c = (size_t)readVal(pr.countType);
                    uint32_t ids[4];
                    if (pr.name != "vertex_indices" && pr.name != "vertex_index") { for (size_t k = 0; k < c; ++k) readVal(pr.type); continue; }
                    if (c != 3 && c != 4) throw err("Encountered a face with " + std::to_string(c) + " vertices! Only triangle and quad-based PLY meshes are supported for now.");
                    for (size_t k = 0; k < c; ++k) {
                        double id = readVal(pr.type);
                        if (id < 0 || (size_t)id >= mesh.p.size()) throw err("PLY: vertex index out of range");
                        ids[k] = (uint32_t)id;
                    }
                    // ply.cpp:276-289 (quad -> (0,1,2), (3,0,2))
                    mesh.idx.insert(mesh.idx.end(), {ids[0], ids[1], ids[2]});
                    if (c == 4) mesh.idx.insert(mesh.idx.end(), {ids[3], ids[0], ids[2]});
                }
            }
        } else {
            for (size_t r = 0; r < e.count; ++r)
                for (auto &pr : e.props) {
                    if (pr.list) { size_t c = (size_t)readVal(pr.countType); for (size_t k = 0; k < c; ++k) readVal(pr.type); }
                    else readVal(pr.type);
                }
        }
    }
}

void loadOBJ(const std::string &path, Mesh &mesh, bool flipTexCoords) {
    // Simplified obj.cpp: all groups collapsed into one mesh, polygon fans
    // (obj.cpp:309-322), vertices deduplicated by (p, n, uv) (obj.cpp:577-660)
    std::ifstream f(path);
    if (!f) throw err("Unable to open \"" + path + "\"");
    std::vector<V3> P, N;
    std::vector<std::pair<float, float>> T;
    struct Key { int p, n, t; bool operator<(const Key &o) const { return std::tie(p, n, t) < std::tie(o.p, o.n, o.t); } };
    std::map<Key, uint32_t> vmap;
    std::vector<Key> verts;
    std::vector<uint32_t> idx;
    bool anyN = false, anyT = false;
    std::string line;
    auto parseIdx = [&](const std::string &tok) {
        Key k{0, 0, 0};
        auto parts = std::vector<std::string>();
        std::string cur;
        for (char c : tok) { if (c == '/') { parts.push_back(cur); cur.clear(); } else cur += c; }
        parts.push_back(cur);
        auto conv = [](const std::string &s, size_t n) -> int {
            if (s.empty()) return 0;
            int v = std::stoi(s);
            return v < 0 ? (int)n + v + 1 : v;
        };
        k.p = conv(parts[0], P.size());
        if (parts.size() > 1) k.t = conv(parts[1], T.size());
        if (parts.size() > 2) k.n = conv(parts[2], N.size());
        if (k.n) anyN = true;
        if (k.t) anyT = true;
        auto it = vmap.find(k);
        if (it != vmap.end()) return it->second;
        uint32_t id = (uint32_t)verts.size();
        vmap[k] = id;
        verts.push_back(k);
        return id;
    };
    while (std::getline(f, line)) {
        std::istringstream iss(line);
        std::string t;
        if (!(iss >> t)) continue;
        if (t == "v") { V3 v; iss >> v.x >> v.y >> v.z; P.push_back(v); }
        else if (t == "vn") { V3 v; iss >> v.x >> v.y >> v.z; N.push_back(v); }
        else if (t == "vt") { float u = 0, v = 0; iss >> u >> v; if (flipTexCoords) v = 1 - v; T.emplace_back(u, v); }
        else if (t == "f") {
            std::vector<std::string> toks;
            std::string s;
            while (iss >> s) toks.push_back(s);
            if (toks.size() < 3) continue;
            uint32_t a = parseIdx(toks[0]), b = parseIdx(toks[1]), c = parseIdx(toks[2]);
            idx.insert(idx.end(), {a, b, c});
            for (size_t k = 3; k < toks.size(); ++k) {
                b = c;
                c = parseIdx(toks[k]);
                idx.insert(idx.end(), {a, b, c});
            }
        }
    }
    mesh.p.resize(verts.size());
    if (anyN) mesh.n.resize(verts.size());
    if (anyT) mesh.uv.resize(2 * verts.size());
    for (size_t i = 0; i < verts.size(); ++i) {
        const Key &k = verts[i];
        if (k.p <= 0 || (size_t)k.p > P.size()) throw err("OBJ: vertex index out of range");
        mesh.p[i] = P[k.p - 1];
        if (anyN) mesh.n[i] = (k.n > 0 && (size_t)k.n <= N.size()) ? N[k.n - 1] : V3(0.0f);
        if (anyT && k.t > 0 && (size_t)k.t <= T.size()) { mesh.uv[2 * i] = T[k.t - 1].first; mesh.uv[2 * i + 1] = T[k.t - 1].second; }
    }
    mesh.idx = std::move(idx);
}

// Mitsuba's `serialized` mesh container (src/shapes/serialized.cpp:64-145,
// TriMesh::loadCompressed / readHeader / readOffset in
// src/librender/trimesh.cpp:175-300): per mesh an uncompressed header
// (uint16 0x041C, uint16 version 3 or 4) followed by a zlib (DEFLATE) stream
// holding uint32 flags, [v4: a null-terminated name], uint64 vertex and
// triangle counts, positions, optional normals / texcoords / colors (float32,
// or float64 with flag 0x2000), and uint32 triangle indices.  The file ends
// with a dictionary of the meshes' start offsets (v4: uint64, v3: uint32) and
// a uint32 mesh count.  Vertex colors are read and dropped (no texture
// plugins in this build).
namespace {
enum { kSerHasNormals = 0x0001, kSerHasTexcoords = 0x0002, kSerHasColors = 0x0008, kSerDouble = 0x2000 };

class Inflater {
public:
    Inflater(const std::string &data, size_t offset, const std::string &path) : path_(path) {
        memset(&z_, 0, sizeof(z_));
        if (inflateInit(&z_) != Z_OK) throw err("\"" + path + "\": inflateInit failed");
        z_.next_in = (Bytef *)data.data() + offset;
        z_.avail_in = (uInt)(data.size() - offset);
    }
    ~Inflater() { inflateEnd(&z_); }
    void read(void *dst, size_t n) {
        z_.next_out = (Bytef *)dst;
        z_.avail_out = (uInt)n;
        while (z_.avail_out > 0) {
            int rc = inflate(&z_, Z_SYNC_FLUSH);
            if (rc == Z_STREAM_END && z_.avail_out > 0)
                throw err("\"" + path_ + "\": unexpected end of the compressed mesh stream");
            if (rc != Z_OK && rc != Z_STREAM_END)
                throw err("\"" + path_ + "\": corrupt compressed mesh stream (zlib error " + std::to_string(rc) + ")");
        }
    }
    template <class T> T get() { T v; read(&v, sizeof(T)); return v; }
    std::string cstring() {
        std::string s;
        for (char c; (c = get<char>()) != 0;) s += c;
        return s;
    }
    // readHelper (trimesh.cpp:150-172): single or double precision to float
    void floats(std::vector<float> &out, size_t n, bool dbl) {
        out.resize(n);
        if (!dbl) { read(out.data(), n * sizeof(float)); return; }
        std::vector<double> tmp(n);
        read(tmp.data(), n * sizeof(double));
        for (size_t i = 0; i < n; ++i) out[i] = (float)tmp[i];
    }
private:
    z_stream z_;
    std::string path_;
};

template <class T> T leAt(const std::string &d, size_t off) { T v; memcpy(&v, d.data() + off, sizeof(T)); return v; }
}  // namespace

void loadSerialized(const std::string &path, int shapeIndex, Mesh &mesh) {
    const std::string data = readFile(path);
    auto header = [&](size_t off) -> int {
        if (off + 4 > data.size()) throw err("\"" + path + "\": truncated file");
        const uint16_t format = leAt<uint16_t>(data, off), version = leAt<uint16_t>(data, off + 2);
        if (format == 0x1C04)
            throw err("Encountered a geometry file generated by an old version of Mitsuba. Please re-import the scene to update this file to the current format.");
        if (format != 0x041C) throw err("\"" + path + "\": Encountered an invalid file format!");
        if (version != 3 && version != 4) throw err("\"" + path + "\": Encountered an incompatible file version!");
        return version;
    };
    if (shapeIndex < 0) throw err("Shape index must be nonnegative!");
    const int version = header(0);
    size_t offset = 0;
    if (shapeIndex != 0) {
        // readOffset (trimesh.cpp:272-291); the dictionary sits at the end
        if (data.size() < 8) throw err("\"" + path + "\": truncated file");
        const uint32_t count = leAt<uint32_t>(data, data.size() - 4);
        if (shapeIndex >= (int)count)
            throw err("Unable to unserialize mesh, shape index is out of range! (requested " + std::to_string(shapeIndex) +
                      " out of 0.." + std::to_string((int)count - 1) + ")");
        if (version == 4) {
            const size_t at = data.size() - 8 * (size_t)(count - shapeIndex) - 4;
            if (at > data.size()) throw err("\"" + path + "\": corrupt offset dictionary");
            offset = (size_t)leAt<uint64_t>(data, at);
        } else {
            const size_t at = data.size() - 4 * (size_t)(count - shapeIndex + 1);
            if (at > data.size()) throw err("\"" + path + "\": corrupt offset dictionary");
            offset = leAt<uint32_t>(data, at);
        }
        if (offset + 4 > data.size()) throw err("\"" + path + "\": corrupt offset dictionary");
        header(offset);
    }
    Inflater z(data, offset + 4, path);
    const uint32_t flags = z.get<uint32_t>();
    if (version == 4) mesh.name = z.cstring();
    const uint64_t nv = z.get<uint64_t>(), nt = z.get<uint64_t>();
    if (nv > 0xFFFFFFFFull || nt > 0x7FFFFFFFull) throw err("\"" + path + "\": mesh too large for 32-bit indices");
    const bool dbl = (flags & kSerDouble) != 0;
    std::vector<float> buf;
    z.floats(buf, 3 * nv, dbl);
    mesh.p.resize(nv);
    for (size_t i = 0; i < nv; ++i) mesh.p[i] = V3(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]);
    mesh.n.clear();
    if (flags & kSerHasNormals) {
        z.floats(buf, 3 * nv, dbl);
        mesh.n.resize(nv);
        for (size_t i = 0; i < nv; ++i) mesh.n[i] = V3(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]);
    }
    mesh.uv.clear();
    if (flags & kSerHasTexcoords) z.floats(mesh.uv, 2 * nv, dbl);
    if (flags & kSerHasColors) z.floats(buf, 3 * nv, dbl);
    mesh.idx.resize(3 * nt);
    z.read(mesh.idx.data(), mesh.idx.size() * sizeof(uint32_t));
    for (uint32_t i : mesh.idx)
        if (i >= nv) throw err("\"" + path + "\": triangle index out of range");
}

// trimesh.cpp:608-681
static float unitAngle(const V3 &u, const V3 &v) {
    if (dot(u, v) < 0) return (float)M_PI - 2.0f * std::asin(0.5f * length(v + u));
    return 2.0f * std::asin(0.5f * length(v - u));
}

void computeNormals(Mesh &mesh, bool flipNormals) {
    if (mesh.faceNormals) {
        mesh.n.clear();
        if (flipNormals)
            for (size_t i = 0; i < mesh.idx.size(); i += 3) std::swap(mesh.idx[i], mesh.idx[i + 1]);
        return;
    }
    if (!mesh.n.empty()) {
        if (flipNormals) for (auto &n : mesh.n) n = -n;
        return;
    }
    mesh.n.assign(mesh.p.size(), V3(0.0f));
    for (size_t t = 0; t < mesh.idx.size(); t += 3) {
        V3 n(0.0f);
        for (int i = 0; i < 3; ++i) {
            const V3 &v0 = mesh.p[mesh.idx[t + i]];
            const V3 &v1 = mesh.p[mesh.idx[t + (i + 1) % 3]];
            const V3 &v2 = mesh.p[mesh.idx[t + (i + 2) % 3]];
            V3 sideA = v1 - v0, sideB = v2 - v0;
            if (i == 0) {
                n = cross(sideA, sideB);
                float len = length(n);
                if (len == 0) break;
                n /= len;
            }
            float angle = unitAngle(normalize(sideA), normalize(sideB));
            mesh.n[mesh.idx[t + i]] += n * angle;
        }
    }
    for (auto &n : mesh.n) {
        float len = length(n);
        if (flipNormals) len *= -1;
        if (len != 0) n /= len;
        else n = V3(1, 0, 0);
    }
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

void writePFM(const std::string &path, int w, int h, const std::vector<float> &rgb) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) throw err("cannot write " + path);
    fprintf(f, "PF\n%d %d\n-1\n", w, h);
    // PFM stores rows bottom-to-top (bitmap.cpp:347-398)
    for (int y = h - 1; y >= 0; --y) fwrite(&rgb[(size_t)y * w * 3], sizeof(float), (size_t)w * 3, f);
    fclose(f);
}

// ---------------------------------------------------------------------------
// Scene handler
// ---------------------------------------------------------------------------
namespace {

struct ShapeGroup {
    std::vector<Mesh> meshes;   // object space (flattening)
    std::vector<Rect> rects;
    int index = -1;             // two-level: Scene::groups entry
};

struct Loader {
    Scene &scene;
    std::map<std::string, std::string> defines;
    std::map<std::string, int> bsdfIds;
    std::map<std::string, int> textureIds;
    std::map<std::string, ShapeGroup> groups;
    std::map<std::string, int> namedEmitters;
    std::vector<std::string> dirStack;

    explicit Loader(Scene &s) : scene(s) {}

    std::string subst(const std::string &v) {
        // $name substitution from -D / <default> (scenehandler.cpp:211)
        std::string o;
        for (size_t k = 0; k < v.size(); ++k) {
            if (v[k] == '$') {
                size_t e = k + 1;
                while (e < v.size() && (isalnum((unsigned char)v[e]) || v[e] == '_')) ++e;
                std::string key = v.substr(k + 1, e - k - 1);
                auto it = defines.find(key);
                if (it == defines.end()) throw err("Unresolved parameter \"$" + key + "\"");
                o += it->second;
                k = e - 1;
            } else {
                o += v[k];
            }
        }
        return o;
    }

    void substAll(XNode &n) {
        for (auto &a : n.attrs) a.second = subst(a.second);
    }

    std::string resolve(const std::string &f) {
        if (!f.empty() && f[0] == '/') return f;
        for (auto it = dirStack.rbegin(); it != dirStack.rend(); ++it) {
            std::string p = *it + "/" + f;
            std::ifstream t(p);
            if (t.good()) return p;
        }
        return dirStack.back() + "/" + f;
    }

    Transform parseTransform(XNode &n) {
        Transform t;
        for (auto &cp : n.children) {
            XNode &c = *cp;
            substAll(c);
            const std::string &tag = c.tag;
            if (tag == "translate") {
                t = Transform::translate(V3(parseF(c.attr("x", "0"), c.line), parseF(c.attr("y", "0"), c.line), parseF(c.attr("z", "0"), c.line))) * t;
            } else if (tag == "rotate") {
                V3 ax(parseF(c.attr("x", "0"), c.line), parseF(c.attr("y", "0"), c.line), parseF(c.attr("z", "0"), c.line));
                t = Transform::rotate(ax, parseF(c.attr("angle"), c.line)) * t;
            } else if (tag == "scale") {
                bool hasXYZ = c.hasAttr("x") || c.hasAttr("y") || c.hasAttr("z");
                V3 s;
                if (hasXYZ && c.hasAttr("value")) throw err("<scale>: provided both xyz and value arguments!");
                if (hasXYZ) s = V3(parseF(c.attr("x", "1"), c.line), parseF(c.attr("y", "1"), c.line), parseF(c.attr("z", "1"), c.line));
                else if (c.hasAttr("value")) s = V3(parseF(c.attr("value"), c.line));
                else throw err("<scale>: provided neither xyz nor value arguments!");
                t = Transform::scale(s) * t;
            } else if (tag == "lookat" || tag == "lookAt") {
                auto o = tokenize(c.attr("origin"), ", "), tg = tokenize(c.attr("target"), ", "), up = tokenize(c.attr("up"), ", ");
                if (o.size() != 3) throw err("<lookat>: invalid 'origin' argument");
                if (tg.size() != 3) throw err("<lookat>: invalid 'target' argument");
                V3 O(parseF(o[0], c.line), parseF(o[1], c.line), parseF(o[2], c.line));
                V3 T(parseF(tg[0], c.line), parseF(tg[1], c.line), parseF(tg[2], c.line));
                V3 U(0.0f);
                if (up.size() == 3) U = V3(parseF(up[0], c.line), parseF(up[1], c.line), parseF(up[2], c.line));
                else if (!up.empty()) throw err("<lookat>: invalid 'up' argument");
                if (dot(U, U) == 0) { V3 unused; coordinateSystem(normalize(T - O), U, unused); }
                t = Transform::lookAt(O, T, U) * t;
            } else if (tag == "matrix") {
                auto tok = tokenize(c.attr("value"), ", ");
                if (tok.size() != 16) throw err("Invalid matrix specified");
                double m[4][4];
                for (int k = 0; k < 16; ++k) m[k / 4][k % 4] = parseF(tok[k], c.line);
                t = Transform::fromMatrix(m) * t;
            } else {
                throw err("line " + std::to_string(c.line) + ": unsupported transform element <" + tag + ">");
            }
        }
        return t;
    }

    V3 parseRGB(const std::string &v, int line) {
        auto tok = tokenize(v, ", ");
        if (tok.size() == 1 && tok[0].size() == 7 && tok[0][0] == '#') {
            int enc = (int)strtol(tok[0].c_str() + 1, nullptr, 16);
            return V3(((enc & 0xFF0000) >> 16) / 255.0f, ((enc & 0x00FF00) >> 8) / 255.0f, (enc & 0xFF) / 255.0f);
        }
        if (tok.size() == 1) return V3(parseF(tok[0], line));
        if (tok.size() == 3) return V3(parseF(tok[0], line), parseF(tok[1], line), parseF(tok[2], line));
        throw err("Invalid RGB value specified");
    }

    static float srgbToLinear(float v) {
        if (v <= 0.04045f) return v * (1.0f / 12.92f);
        return std::pow((v + 0.055f) * (1.0f / 1.055f), 2.4f);
    }

    // Parse value children of a plugin element into props; returns nested
    // plugin elements for the caller.
    void parseProps(XNode &n, Properties &props, std::vector<XNode *> &nested) {
        for (auto &cp : n.children) {
            XNode &c = *cp;
            substAll(c);
            const std::string name = c.attr("name");
            const std::string &tag = c.tag;
            if (tag == "float") props.floats[name] = parseF(c.attr("value"), c.line);
            else if (tag == "integer") {
                long long v = std::stoll(c.attr("value"));
                props.ints[name] = v;
            } else if (tag == "boolean") {
                std::string v = lower(c.attr("value"));
                if (v != "true" && v != "false") throw err("line " + std::to_string(c.line) + ": could not parse boolean \"" + v + "\"");
                props.bools[name] = v == "true";
            } else if (tag == "string") props.strings[name] = c.attr("value");
            else if (tag == "rgb") props.spectra[name] = parseRGB(c.attr("value"), c.line);
            else if (tag == "srgb") { V3 v = parseRGB(c.attr("value"), c.line); props.spectra[name] = V3(srgbToLinear(v.x), srgbToLinear(v.y), srgbToLinear(v.z)); }
            else if (tag == "spectrum") {
                if (c.hasAttr("filename")) throw err("<spectrum filename=...> is not supported in RGB mode by this loader");
                auto tok = tokenize(c.attr("value"), ", ");
                if (tok.size() == 1 && tok[0].find(':') == std::string::npos) {
                    // RGB mode: reflectance -> constant, illuminant -> D65 * v = v (spectrum.cpp:164)
                    props.spectra[name] = V3(parseF(tok[0], c.line));
                } else if (tok.size() == 3 && tok[0].find(':') == std::string::npos) {
                    props.spectra[name] = V3(parseF(tok[0], c.line), parseF(tok[1], c.line), parseF(tok[2], c.line));
                } else {
                    throw err("line " + std::to_string(c.line) + ": wavelength:value spectra are not supported by this loader");
                }
            } else if (tag == "point" || tag == "vector") {
                props.points[name] = V3(parseF(c.attr("x", "0"), c.line), parseF(c.attr("y", "0"), c.line), parseF(c.attr("z", "0"), c.line));
            } else if (tag == "transform") {
                props.transforms[name] = parseTransform(c);
            } else {
                nested.push_back(&c);
            }
        }
    }

    // util.cpp:651-681 (double precision, for the quadrature below)
    static double fresnelDielectricD(double cosThetaI, double eta) {
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
    static double simpson(double eta, double a, double b, double fa, double fm, double fb, double whole, int depth) {
        const double m = 0.5 * (a + b), lm = 0.5 * (a + m), rm = 0.5 * (m + b);
        const double flm = fresnelDielectricD(std::sqrt(lm), eta), frm = fresnelDielectricD(std::sqrt(rm), eta);
        const double left = (m - a) / 6 * (fa + 4 * flm + fm), right = (b - m) / 6 * (fm + 4 * frm + fb);
        if (depth <= 0 || std::abs(left + right - whole) <= 1e-10) return left + right + (left + right - whole) / 15;
        return simpson(eta, a, m, fa, flm, fm, left, depth - 1) + simpson(eta, m, b, fm, frm, fb, right, depth - 1);
    }
    static float fresnelDiffuseReflectance(float eta) {
        const double fa = fresnelDielectricD(0.0, eta), fm = fresnelDielectricD(std::sqrt(0.5), eta), fb = fresnelDielectricD(1.0, eta);
        return (float)simpson(eta, 0.0, 1.0, fa, fm, fb, (fa + 4 * fm + fb) / 6, 40);
    }
    // BSDF::ensureEnergyConservation(texture, name, 1) (bsdf.cpp:88-113): a
    // constant whose largest component exceeds 1 is scaled by 0.99 / max
    static V3 energyConserving(Properties &props, V3 v) {
        if (!props.getBool("ensureEnergyConservation", true)) return v;
        float mx = std::max(v.x, std::max(v.y, v.z));
        return mx > 1.0f ? v * (0.99f * (1.0f / mx)) : v;
    }
    static float luminance(V3 v) { return v.x * 0.212671f + v.y * 0.715160f + v.z * 0.072169f; }   // spectrum.h:638-640
    // conductor material: the data/ior/<name>.{eta,k}.spd lookup (RGB), eta/k overrides, / extEta
    void conductorIOR(Properties &props, mtsg_bsdf &d, const char *who) {
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
    void microfacetProps(Properties &props, mtsg_bsdf &d) {
        int distr = MTSG_MF_BECKMANN;
        if (props.strings.count("distribution")) {
            std::string dn = lower(props.strings["distribution"]);
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

    // `bitmap` texture (src/textures/bitmap.cpp:179-302, Texture2D(props),
    // src/librender/texture.cpp:84-98); returns its index in scene.textures
    int parseTexture(XNode &n) {
        substAll(n);
        Properties props;
        std::vector<XNode *> nested;
        parseProps(n, props, nested);
        const std::string type = lower(n.attr("type"));
        if (type != "bitmap")
            throw err("line " + std::to_string(n.line) + ": texture plugin \"" + type + "\" is outside this build's scope (only 'bitmap')");
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
        t.id = n.attr("id");
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
        const int idx = (int)scene.textures.size() - 1;
        if (!t.id.empty()) textureIds[t.id] = idx;
        return idx;
    }

    // A BSDF's spectrum parameter given as a nested texture or a reference
    // to one: the texture index, or -1 (constant).  Only the parameters the
    // device evaluates per hit may be textured.
    int textureParam(std::vector<XNode *> &nested, const std::vector<std::string> &names, const std::string &bsdfType) {
        int found = -1;
        for (XNode *c : nested) {
            substAll(*c);
            const std::string name = c->attr("name");
            if (c->tag == "texture" || (c->tag == "ref" && textureIds.count(c->attr("id")))) {
                bool ok = false;
                for (auto &nm : names) ok |= nm == name;
                if (!ok)
                    throw err("line " + std::to_string(c->line) + ": " + bsdfType + ": a texture for parameter \"" + name +
                              "\" is outside this build's scope");
                found = c->tag == "texture" ? parseTexture(*c) : textureIds[c->attr("id")];
            } else if (c->tag != "bsdf" && c->tag != "ref") {
                throw err("line " + std::to_string(c->line) + ": unsupported element <" + c->tag + "> inside a BSDF");
            }
        }
        return found;
    }
    // Constant or textured reflectance of diffuse / plastic / roughplastic:
    // ensureEnergyConservation scales a texture by 0.99 / max through a
    // ScaleTexture (bsdf.cpp:88-113); returns the value used for
    // getAverage() (the texture's average x scale) and sets d.texture
    V3 reflectanceParam(Properties &props, std::vector<XNode *> &nested, const std::vector<std::string> &names,
                        const V3 &constant, const std::string &bsdfType, mtsg_bsdf &d, float &maxOut) {
        const int tex = textureParam(nested, names, bsdfType);
        if (tex < 0) {
            const V3 r = energyConserving(props, constant);
            maxOut = std::max(r.x, std::max(r.y, r.z));
            d.texture = 0;
            return r;
        }
        mtsg_texture &t = scene.textures[tex].d;
        float mx = std::max(t.maximum[0], std::max(t.maximum[1], t.maximum[2]));
        if (props.getBool("ensureEnergyConservation", true) && mx * t.scale > 1.0f) {
            // a second BSDF sharing the texture by reference gets its own scaled copy
            Texture copy = scene.textures[tex];
            copy.id.clear();
            copy.d.scale = t.scale * (0.99f * (1.0f / (mx * t.scale)));
            scene.textures.push_back(copy);
            return reflectanceTex((int)scene.textures.size() - 1, d, maxOut);
        }
        return reflectanceTex(tex, d, maxOut);
    }
    V3 reflectanceTex(int tex, mtsg_bsdf &d, float &maxOut) {
        const mtsg_texture &t = scene.textures[tex].d;
        d.texture = tex + 1;
        maxOut = std::max(t.maximum[0], std::max(t.maximum[1], t.maximum[2])) * t.scale;
        return V3(t.average[0], t.average[1], t.average[2]) * t.scale;
    }

    int parseBsdf(XNode &n) {
        substAll(n);
        Properties props;
        std::vector<XNode *> nested;
        parseProps(n, props, nested);
        std::string type = lower(n.attr("type"));
        Bsdf b;
        b.id = n.attr("id");
        mtsg_bsdf &d = b.d;
        if (type == "diffuse") {
            // diffuse.cpp:77-84, configure() keeps the component iff max > 0
            float mx;
            V3 r = reflectanceParam(props, nested, {"reflectance", "diffuseReflectance"},
                                    props.getSpectrum(props.has("reflectance") ? "reflectance" : "diffuseReflectance", V3(0.5f)),
                                    "diffuse", d, mx);
            d.type = MTSG_BSDF_DIFFUSE;
            d.reflectance[0] = r.x; d.reflectance[1] = r.y; d.reflectance[2] = r.z;
            d.smooth = mx > 0;
            d.ref_n_zero = 0;
        } else if (type == "roughconductor") {
            // roughconductor.cpp:168-203
            textureParam(nested, {}, type);
            V3 spec = energyConserving(props, props.getSpectrum("specularReflectance", V3(1.0f)));
            conductorIOR(props, d, "roughconductor");
            microfacetProps(props, d);
            d.type = MTSG_BSDF_ROUGHCONDUCTOR;
            for (int i = 0; i < 3; ++i) d.spec_refl[i] = spec[i];
            d.smooth = 1;
            d.ref_n_zero = 0;
        } else if (type == "dielectric") {
            // dielectric.cpp:148-170
            textureParam(nested, {}, type);
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
            textureParam(nested, {}, type);
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
            textureParam(nested, {}, type);
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
            V3 dr = reflectanceParam(props, nested, {"diffuseReflectance"}, props.getSpectrum("diffuseReflectance", V3(0.5f)),
                                     "plastic", d, dmx);
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
            V3 dr = reflectanceParam(props, nested, {"diffuseReflectance"}, props.getSpectrum("diffuseReflectance", V3(0.5f)),
                                     "roughplastic", d, dmx);
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
            std::vector<int> kids;
            for (XNode *c : nested) {
                substAll(*c);
                if (c->tag == "bsdf") kids.push_back(parseBsdf(*c));
                else if (c->tag == "ref") {
                    std::string id = c->attr("id");
                    if (!bsdfIds.count(id)) throw err("Referenced object '" + id + "' not found!");
                    kids.push_back(bsdfIds[id]);
                } else {
                    throw err("line " + std::to_string(c->line) + ": unsupported element <" + c->tag + "> inside twosided");
                }
            }
            if (kids.empty()) throw err("A nested one-sided material is required!");
            if (kids.size() > 2) throw err("No more than two nested BRDFs can be added!");
            for (int k : kids) {
                const mtsg_bsdf &kd = scene.bsdfs[k].d;
                if (kd.type == MTSG_BSDF_DIELECTRIC || kd.type == MTSG_BSDF_ROUGHDIELECTRIC)
                    throw err("Only materials without a transmission component can be nested!");
                if (kd.twosided) throw err("twosided: a nested twosided material is not supported by this build");
            }
            const int backIdx = kids.size() == 2 ? kids[1] : kids[0];
            d = scene.bsdfs[kids[0]].d;
            d.twosided = 1;
            d.back = backIdx;
            d.smooth = scene.bsdfs[kids[0]].d.smooth || scene.bsdfs[backIdx].d.smooth;
            d.ref_n_zero = 1;    // EBackSide component (records.inl:160-164)
        } else {
            throw err("line " + std::to_string(n.line) + ": BSDF plugin \"" + type + "\" is outside this build's scope");
        }
        scene.bsdfs.push_back(b);
        int id = (int)scene.bsdfs.size() - 1;
        if (!b.id.empty()) bsdfIds[b.id] = id;
        return id;
    }

    int defaultBsdf(bool emitter) {
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

    int parseEmitter(XNode &n) {
        substAll(n);
        Properties props;
        std::vector<XNode *> nested;
        parseProps(n, props, nested);
        std::string type = lower(n.attr("type"));
        if (type != "area") throw err("line " + std::to_string(n.line) + ": emitter plugin \"" + type + "\" is outside this build's scope");
        if (props.transforms.count("toWorld")) throw err("Found a 'toWorld' transformation -- this is not allowed -- the area light inherits this transformation from its parent shape");
        Emitter e;
        e.radiance = props.getSpectrum("radiance", V3(1.0f));   // D65 == 1 in RGB mode
        e.samplingWeight = props.getFloat("samplingWeight", 1.0f);
        scene.emitters.push_back(e);
        return (int)scene.emitters.size() - 1;
    }

    // Scene-level emitter: only `envmap` (envmap.cpp:105-185); area lights
    // must be nested in a shape
    void parseSceneEmitter(XNode &n) {
        substAll(n);
        Properties props;
        std::vector<XNode *> nested;
        parseProps(n, props, nested);
        std::string type = lower(n.attr("type"));
        if (type != "envmap")
            throw err("line " + std::to_string(n.line) + ": emitter \"" + type + "\" outside a shape is outside this build's scope");
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
    }

    // Returns meshes/rects in object->world space given the toWorld transform
    void parseShape(XNode &n, std::vector<Mesh> &meshes, std::vector<Rect> &rects, bool inGroup) {
        substAll(n);
        std::string type = lower(n.attr("type"));
        if (type == "shapegroup") {
            if (inGroup) throw err("Nested instancing is not permitted");
            ShapeGroup g;
            for (auto &cp : n.children) {
                substAll(*cp);
                if (cp->tag != "shape") throw err("shapegroup may only contain shapes");
                parseShape(*cp, g.meshes, g.rects, true);
            }
            std::string id = n.attr("id");
            if (id.empty()) throw err("shapegroup needs an id");
            if (scene.twoLevel) {
                // ShapeGroup::addChild / configure (shapegroup.cpp:94-138): the
                // group's shapes get their own kd-tree in group space
                if (!g.rects.empty())
                    throw err("shapegroup \"" + id + "\": rectangles inside shape groups are outside the two-level "
                              "variant of this build (use the flattening mode)");
                GroupDef gd;
                gd.id = id;
                g.index = (int)scene.groups.size();
                for (auto &m : g.meshes) {
                    m.group = g.index;
                    scene.meshes.push_back(std::move(m));
                    gd.shapes.push_back((int)scene.shapes.size());
                    scene.shapes.push_back({MTSG_SHAPE_MESH, (int)scene.meshes.size() - 1});
                }
                g.meshes.clear();
                scene.groups.push_back(std::move(gd));
            }
            groups[id] = std::move(g);
            return;
        }
        Properties props;
        std::vector<XNode *> nested;
        parseProps(n, props, nested);
        int bsdf = -1, emitter = -1;
        std::string instRef;
        for (XNode *c : nested) {
            substAll(*c);
            if (c->tag == "bsdf") bsdf = parseBsdf(*c);
            else if (c->tag == "emitter") {
                if (inGroup) throw err("emitters inside shapegroups are not supported");
                emitter = parseEmitter(*c);
            } else if (c->tag == "ref") {
                std::string id = c->attr("id");
                if (bsdfIds.count(id)) bsdf = bsdfIds[id];
                else if (groups.count(id)) instRef = id;
                else throw err("Referenced object '" + id + "' not found!");
            } else {
                throw err("line " + std::to_string(c->line) + ": unsupported element <" + c->tag + "> inside <shape>");
            }
        }
        Transform toWorld = props.getTransform("toWorld", Transform());
        bool flip = props.getBool("flipNormals", false);
        if (type == "instance") {
            if (instRef.empty()) throw err("A reference to a 'shapegroup' must be specified!");
            if (inGroup) throw err("Nested instancing is not permitted");
            const ShapeGroup &g = groups[instRef];
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
            for (const Mesh &m0 : g.meshes) {
                Mesh m = m0;
                m.instanced = true;   // an Instance in the reference: not one of Scene::getMeshes()
                for (auto &p : m.p) p = toWorld.point(p);
                for (auto &nn : m.n) nn = normalize(toWorld.normal(nn));
                meshes.push_back(std::move(m));
            }
            for (const Rect &r0 : g.rects) {
                Rect r = r0;
                r.toWorld = toWorld * r0.toWorld;
                rects.push_back(r);
            }
            return;
        }
        if (bsdf < 0) bsdf = defaultBsdf(emitter >= 0);
        if (type == "rectangle") {
            Rect r;
            r.toWorld = toWorld;
            if (flip) r.toWorld = r.toWorld * Transform::scale(V3(1, 1, -1));
            r.bsdf = bsdf;
            r.emitter = emitter;
            rects.push_back(r);
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
            loadSerialized(resolve(props.getString("filename", "")), props.getInt("shapeIndex", 0), m);
            const auto &M = toWorld.m;
            const double det = (double)M[0][0] * ((double)M[1][1] * M[2][2] - (double)M[1][2] * M[2][1]) -
                               (double)M[0][1] * ((double)M[1][0] * M[2][2] - (double)M[1][2] * M[2][0]) +
                               (double)M[0][2] * ((double)M[1][0] * M[2][1] - (double)M[1][1] * M[2][0]);
            if (det < 0)
                for (size_t t = 0; t + 2 < m.idx.size(); t += 3) std::swap(m.idx[t], m.idx[t + 1]);
        } else {
            throw err("line " + std::to_string(n.line) + ": shape plugin \"" + type + "\" is outside this build's scope");
        }
        m.faceNormals = props.getBool("faceNormals", false);
        for (auto &p : m.p) p = toWorld.point(p);
        for (auto &nn : m.n) nn = normalize(toWorld.normal(nn));
        computeNormals(m, flip);
        m.bsdf = bsdf;
        m.emitter = emitter;
        meshes.push_back(std::move(m));
    }

    static void buildCube(Mesh &m) {
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

    void parseScene(XNode &root) {
        for (auto &cp : root.children) {
            XNode &c = *cp;
            substAll(c);
            const std::string &tag = c.tag;
            if (tag == "default") {
                std::string name = c.attr("name");
                if (!defines.count(name)) defines[name] = c.attr("value");
            } else if (tag == "include") {
                std::string path = resolve(c.attr("filename"));
                std::string src = readFile(path);
                XParser p(src, path);
                p.skipMisc();
                auto sub = p.element();
                dirStack.push_back(dirName(path));
                parseScene(*sub);
                dirStack.pop_back();
            } else if (tag == "integrator") {
                Properties props;
                std::vector<XNode *> nested;
                parseProps(c, props, nested);
                std::string type = c.attr("type");
                IntegratorProps &ip = scene.integrator;
                if (type == "myPath2_OM") {
                    // myPath2OMIntegrator(props) (myPath2_OM.cpp:61-85)
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
                    continue;
                }
                type = lower(type);
                if (type != "path") throw err("line " + std::to_string(c.line) + ": integrator \"" + type + "\" is outside this build's scope (only 'path' and 'myPath2_OM')");
                ip.type = type;
                ip.rrDepth = (int)props.getInt("rrDepth", 5);
                ip.maxDepth = (int)props.getInt("maxDepth", -1);
                ip.strictNormals = props.getBool("strictNormals", false);
                ip.hideEmitters = props.getBool("hideEmitters", false);
                if (ip.rrDepth <= 0) throw err("'rrDepth' must be set to a value greater than zero!");
                if (ip.maxDepth <= 0 && ip.maxDepth != -1) throw err("'maxDepth' must be set to -1 (infinite) or a value greater than zero!");
            } else if (tag == "sensor" || tag == "camera") {
                parseSensor(c);
            } else if (tag == "bsdf") {
                parseBsdf(c);
            } else if (tag == "texture") {
                parseTexture(c);
            } else if (tag == "shape") {
                std::vector<Mesh> meshes;
                std::vector<Rect> rects;
                parseShape(c, meshes, rects, false);
                addShapes(meshes, rects);
            } else if (tag == "emitter") {
                parseSceneEmitter(c);
            } else if (tag == "ref") {
                // scene-level refs are ignored
            } else {
                throw err("line " + std::to_string(c.line) + ": unsupported element <" + tag + ">");
            }
        }
    }

    void addShapes(std::vector<Mesh> &meshes, std::vector<Rect> &rects) {
        for (auto &m : meshes) {
            scene.meshes.push_back(std::move(m));
            int si = (int)scene.shapes.size();
            scene.shapes.push_back({MTSG_SHAPE_MESH, (int)scene.meshes.size() - 1});
            if (scene.meshes.back().emitter >= 0) scene.emitters[scene.meshes.back().emitter].shape = si;
        }
        for (auto &r : rects) {
            scene.rects.push_back(r);
            int si = (int)scene.shapes.size();
            scene.shapes.push_back({MTSG_SHAPE_RECT, (int)scene.rects.size() - 1});
            if (r.emitter >= 0) scene.emitters[r.emitter].shape = si;
        }
    }

    void parseSensor(XNode &c) {
        Properties props;
        std::vector<XNode *> nested;
        parseProps(c, props, nested);
        std::string type = lower(c.attr("type"));
        if (type != "perspective") throw err("line " + std::to_string(c.line) + ": sensor \"" + type + "\" is outside this build's scope");
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
        for (XNode *n : nested) {
            substAll(*n);
            if (n->tag == "film") parseFilm(*n);
            else if (n->tag == "sampler") {
                Properties sp;
                std::vector<XNode *> sn;
                parseProps(*n, sp, sn);
                std::string st = lower(n->attr("type"));
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
            } else {
                throw err("unsupported element <" + n->tag + "> inside <sensor>");
            }
        }
    }

    void parseFilm(XNode &c) {
        Properties props;
        std::vector<XNode *> nested;
        parseProps(c, props, nested);
        std::string type = lower(c.attr("type"));
        if (type != "hdrfilm") throw err("film \"" + type + "\" is outside this build's scope (only 'hdrfilm')");
        Film &f = scene.film;
        f.width = (int)props.getInt("width", 768);
        f.height = (int)props.getInt("height", 576);
        f.cropX = (int)props.getInt("cropOffsetX", 0);
        f.cropY = (int)props.getInt("cropOffsetY", 0);
        f.cropW = (int)props.getInt("cropWidth", f.width);
        f.cropH = (int)props.getInt("cropHeight", f.height);
        f.pixelFormat = lower(props.getString("pixelFormat", "rgb"));
        f.hasAlpha = f.pixelFormat.find('a') != std::string::npos;
        for (XNode *n : nested) {
            substAll(*n);
            if (n->tag != "rfilter") throw err("unsupported element <" + n->tag + "> inside <film>");
            Properties fp;
            std::vector<XNode *> fn;
            parseProps(*n, fp, fn);
            std::string ft = lower(n->attr("type"));
            if (ft == "gaussian") { f.filter = ft; f.stddev = fp.getFloat("stddev", 0.5f); }
            else if (ft == "box") { f.filter = ft; f.boxRadius = fp.getFloat("radius", 0.5f); }
            else throw err("rfilter \"" + ft + "\" is outside this build's scope");
        }
    }
};
}  // namespace

bool readPFM(const std::string &path, int &w, int &h, std::vector<float> &rgb, std::string &err) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) { err = "cannot open " + path; return false; }
    auto token = [&](std::string &out) {
        out.clear();
        int c;
        while ((c = fgetc(f)) != EOF && isspace(c)) {}
        while (c != EOF && !isspace(c)) { out.push_back((char)c); c = fgetc(f); }
        return !out.empty();
    };
    std::string magic, ws, hs, ss;
    bool ok = token(magic) && token(ws) && token(hs) && token(ss);
    if (!ok || (magic != "PF" && magic != "Pf")) { fclose(f); err = "invalid PFM header"; return false; }
    const bool color = magic == "PF";
    w = atoi(ws.c_str()); h = atoi(hs.c_str());
    const float scaleAndOrder = (float)strtod(ss.c_str(), nullptr);
    if (w <= 0 || h <= 0) { fclose(f); err = "invalid PFM size"; return false; }
    const size_t ch = color ? 3 : 1, n = (size_t)w * h * ch;
    std::vector<float> data(n);
    if (fread(data.data(), sizeof(float), n, f) != n) { fclose(f); err = "truncated PFM"; return false; }
    fclose(f);
    if (scaleAndOrder > 0) {   // big endian
        for (auto &v : data) {
            uint32_t u;
            memcpy(&u, &v, 4);
            u = __builtin_bswap32(u);
            memcpy(&v, &u, 4);
        }
    }
    const float scale = std::fabs(scaleAndOrder);
    if (scale != 1) for (auto &v : data) v *= scale;
    rgb.assign((size_t)w * h * 3, 0.0f);
    for (int y = 0; y < h; ++y)   // flipVertically(): PFM rows are bottom-up
        for (int x = 0; x < w; ++x)
            for (int k = 0; k < 3; ++k)
                rgb[((size_t)y * w + x) * 3 + k] = data[((size_t)(h - 1 - y) * w + x) * ch + (color ? k : 0)];
    return true;
}

int g_defaultKDThreads = 0;
int g_instancing = 0;

std::unique_ptr<Scene> loadScene(const std::string &path, const std::map<std::string, std::string> &defines,
                                 const mtsh_scene_overrides *ov) {
    auto scene = std::make_unique<Scene>();
    scene->kd.threads = g_defaultKDThreads;
    scene->twoLevel = g_instancing == 1;
    // build-parameter overrides (tree-quality experiments; defaults follow gkdtree.h:734-744)
    if (const char *v = getenv("MTSH_KD_TRAVERSAL")) scene->kd.traversalCost = (float)atof(v);
    if (const char *v = getenv("MTSH_KD_QUERY")) scene->kd.queryCost = (float)atof(v);
    if (const char *v = getenv("MTSH_KD_EMPTY_BONUS")) scene->kd.emptySpaceBonus = (float)atof(v);
    if (const char *v = getenv("MTSH_KD_STOP_PRIMS")) scene->kd.stopPrims = atoi(v);
    if (const char *v = getenv("MTSH_KD_EXACT_LIMIT")) scene->kd.exactSweepLimit = atoi(v);
    if (const char *v = getenv("MTSH_KD_MAX_DEPTH")) scene->kd.maxDepth = atoi(v);
    if (const char *v = getenv("MTSH_KD_RETRACT")) scene->kd.retract = atoi(v) != 0;
    Loader L(*scene);
    L.defines = defines;
    L.dirStack.push_back(dirName(path));
    std::string src = readFile(path);
    XParser p(src, path);
    p.skipMisc();
    auto root = p.element();
    if (root->tag != "scene") throw err("root element must be <scene>");
    L.parseScene(*root);
    if (!scene->sensor.present) throw err("scene has no <sensor>");
    for (auto &e : scene->emitters)
        if (e.type == MTSG_EMITTER_AREA && e.shape < 0) throw err("area emitter without a parent shape");
    if (ov) {
        // the in-memory values of a Mitsuba plugin (mtsh.h mtsh_scene_overrides)
        if (ov->mask & (MTSH_OVERRIDE_FILM_SIZE | MTSH_OVERRIDE_FILM_CROP)) {
            Film &f = scene->film;
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
            scene->sampleCount = ov->sample_count;
            if (scene->sampler.type == MTSG_SAMPLER_LDSAMPLER) {   // ldsampler.cpp:82-95
                uint32_t r = 1;
                while (r < (uint32_t)ov->sample_count) r <<= 1;
                scene->sampleCount = (int)r;
            }
        }
        if (ov->mask & MTSH_OVERRIDE_INTEGRATOR) {
            IntegratorProps &ip = scene->integrator;
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
    scene->finalize();
    return scene;
}

}  // namespace mtsh
