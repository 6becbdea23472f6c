// OpenEXR input for the environment emitter: Bitmap::readOpenEXR
// (src/libcore/bitmap.cpp:2780-3100) reads `envmap` images through the
// OpenEXR library, which this image does not have.  This is a restatement of
// the parts of the published OpenEXR 2.x file format that scanline images
// need: the header attributes, the line offset table, and the NO / RLE / ZIPS /
// ZIP / PIZ compressors (PIZ: range compression of the 16-bit values,
// canonical Huffman with run-length codes, 2-D Haar wavelet -- the layout of
// ImfPizCompressor / ImfHuf / ImfWav).  HALF and FLOAT channels; channel
// selection as Bitmap::readOpenEXR does it (R/G/B by name, luminance Y
// otherwise); the result is RGB float, rows top-down.
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "scene.h"

namespace mtsh {
namespace {

struct Channel {
    std::string name;
    int type = 1;                   // 0 UINT, 1 HALF, 2 FLOAT
    int xs = 1, ys = 1;
};

uint32_t rdU32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
uint16_t rdU16(const uint8_t *p) { return (uint16_t)(p[0] | p[1] << 8); }

float halfToFloat(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1F, m = h & 0x3FF;
    uint32_t f;
    if (e == 0) {
        if (m == 0) f = s;
        else {   // subnormal half -> normal float
            int ee = -1;
            uint32_t mm = m;
            do { ++ee; mm <<= 1; } while (!(mm & 0x400));
            f = s | (uint32_t)(127 - 15 - ee) << 23 | (mm & 0x3FF) << 13;
        }
    } else if (e == 31) {
        f = s | 0x7F800000u | m << 13;
    } else {
        f = s | (e + 127 - 15) << 23 | m << 13;
    }
    float r;
    memcpy(&r, &f, 4);
    return r;
}

// ---- PIZ: canonical Huffman (ImfHuf.cpp layout) ---------------------------
constexpr int HUF_ENCSIZE = (1 << 16) + 1;
constexpr int SHORT_ZEROCODE_RUN = 59, LONG_ZEROCODE_RUN = 63;
constexpr int SHORTEST_LONG_RUN = 2 + LONG_ZEROCODE_RUN - SHORT_ZEROCODE_RUN;

struct BitReader {
    const uint8_t *p, *end;
    uint64_t c = 0;
    int lc = 0;
    bool ok = true;
    uint64_t get(int n) {   // MSB first
        while (lc < n) {
            if (p >= end) { ok = false; return 0; }
            c = (c << 8) | *p++;
            lc += 8;
        }
        lc -= n;
        return (c >> lc) & ((1ull << n) - 1);
    }
};

bool hufUncompress(const uint8_t *in, size_t nIn, uint16_t *out, size_t nOut, std::string &err) {
    if (nIn == 0) { if (nOut) { err = "PIZ: empty Huffman block"; return false; } return true; }
    if (nIn < 20) { err = "PIZ: truncated Huffman header"; return false; }
    const uint32_t im = rdU32(in), iM = rdU32(in + 4), nBits = rdU32(in + 12);
    if (im >= (uint32_t)HUF_ENCSIZE || iM >= (uint32_t)HUF_ENCSIZE || im > iM) { err = "PIZ: bad Huffman table range"; return false; }
    // code lengths, 6 bits each, with zero runs (hufUnpackEncTable)
    std::vector<uint64_t> hcode(HUF_ENCSIZE, 0);
    BitReader br{in + 20, in + nIn};
    for (uint32_t i = im; i <= iM; ++i) {
        const uint64_t l = br.get(6);
        if (!br.ok) { err = "PIZ: truncated Huffman table"; return false; }
        if (l == (uint64_t)LONG_ZEROCODE_RUN) {
            uint32_t run = (uint32_t)br.get(8) + SHORTEST_LONG_RUN;
            if (i + run > iM + 1) { err = "PIZ: bad zero run"; return false; }
            while (run--) hcode[i++] = 0;
            --i;
        } else if (l >= (uint64_t)SHORT_ZEROCODE_RUN) {
            uint32_t run = (uint32_t)(l - SHORT_ZEROCODE_RUN + 2);
            if (i + run > iM + 1) { err = "PIZ: bad zero run"; return false; }
            while (run--) hcode[i++] = 0;
            --i;
        } else {
            hcode[i] = l;
        }
    }
    const uint8_t *data = br.p;   // the bit stream starts at the next byte
    // canonical code assignment (hufCanonicalCodeTable): for each length,
    // the first code value, then consecutive codes in symbol order
    uint64_t n[59] = {0};
    for (int i = 0; i < HUF_ENCSIZE; ++i) n[hcode[i]]++;
    uint64_t first[59], cstart = 0;
    for (int l = 58; l > 0; --l) {
        const uint64_t nc = (cstart + n[l]) >> 1;
        first[l] = cstart;
        cstart = nc;
    }
    std::vector<std::vector<uint32_t>> syms(59);   // symbols per length, code order
    for (int i = 0; i < HUF_ENCSIZE; ++i)
        if (hcode[i]) syms[hcode[i]].push_back((uint32_t)i);
    if ((uint64_t)nBits > 8ull * (uint64_t)(in + nIn - data)) { err = "PIZ: bit count exceeds the block"; return false; }
    // decode bit by bit: canonical codes are prefix-free, the first
    // (length, value) that names a code is the symbol; the run-length symbol
    // iM repeats the previous value by the following 8-bit count (getCode)
    size_t o = 0;
    uint64_t code = 0;
    int len = 0;
    uint64_t pos = 0;
    auto bit = [&](uint64_t k) { return (data[k >> 3] >> (7 - (k & 7))) & 1u; };
    while (pos < nBits) {
        code = (code << 1) | bit(pos++);
        if (++len > 58) { err = "PIZ: invalid Huffman code"; return false; }
        const std::vector<uint32_t> &sl = syms[len];
        if (sl.empty() || code < first[len] || code - first[len] >= sl.size()) continue;
        const uint32_t s = sl[code - first[len]];
        code = 0;
        len = 0;
        if (s == iM) {
            if (pos + 8 > nBits) { err = "PIZ: truncated run length"; return false; }
            uint32_t cs = 0;
            for (int k = 0; k < 8; ++k) cs = (cs << 1) | bit(pos++);
            if (o == 0 || o + cs > nOut) { err = "PIZ: bad run length"; return false; }
            const uint16_t v = out[o - 1];
            while (cs--) out[o++] = v;
        } else {
            if (o >= nOut) { err = "PIZ: too much data"; return false; }
            out[o++] = (uint16_t)s;
        }
    }
    if (o != nOut) { err = "PIZ: not enough data"; return false; }
    return true;
}

// ---- PIZ: 2-D Haar wavelet (ImfWav.cpp layout) ------------------------------
inline void wdec14(uint16_t l, uint16_t h, uint16_t &a, uint16_t &b) {
    const int16_t ls = (int16_t)l, hs = (int16_t)h;
    const int hi = hs;
    const int ai = ls + (hi & 1) + (hi >> 1);
    a = (uint16_t)(int16_t)ai;
    b = (uint16_t)(int16_t)(ai - hi);
}
inline void wdec16(uint16_t l, uint16_t h, uint16_t &a, uint16_t &b) {
    const int m = l, d = h;
    const int bb = (m - (d >> 1)) & 0xFFFF;
    const int aa = (d + bb - (1 << 15)) & 0xFFFF;
    b = (uint16_t)bb;
    a = (uint16_t)aa;
}
void wav2Decode(uint16_t *in, int nx, int ox, int ny, int oy, uint16_t mx) {
    const bool w14 = mx < (1 << 14);
    const int n = nx > ny ? ny : nx;
    int p = 1;
    while (p <= n) p <<= 1;
    p >>= 1;
    int p2 = p;
    p >>= 1;
    auto dec = [&](uint16_t l, uint16_t h, uint16_t &a, uint16_t &b) { if (w14) wdec14(l, h, a, b); else wdec16(l, h, a, b); };
    while (p >= 1) {
        uint16_t *py = in;
        uint16_t *ey = in + oy * (ny - p2);
        const int oy1 = oy * p, oy2 = oy * p2, ox1 = ox * p, ox2 = ox * p2;
        uint16_t i00, i01, i10, i11;
        for (; py <= ey; py += oy2) {
            uint16_t *px = py;
            uint16_t *ex = py + ox * (nx - p2);
            for (; px <= ex; px += ox2) {
                uint16_t *p01 = px + ox1, *p10 = px + oy1, *p11 = p10 + ox1;
                dec(*px, *p10, i00, i10);
                dec(*p01, *p11, i01, i11);
                dec(i00, i01, *px, *p01);
                dec(i10, i11, *p10, *p11);
            }
            if (nx & p) {   // odd column
                uint16_t *p10 = px + oy1;
                dec(*px, *p10, i00, *p10);
                *px = i00;
            }
        }
        if (ny & p) {   // odd line
            uint16_t *px = py;
            uint16_t *ex = py + ox * (nx - p2);
            for (; px <= ex; px += ox2) {
                uint16_t *p01 = px + ox1;
                dec(*px, *p01, i00, *p01);
                *px = i00;
            }
        }
        p2 = p;
        p >>= 1;
    }
}

// PIZ block -> the uncompressed scanline layout (line by line, channel by
// channel, little-endian values)
bool pizUncompress(const uint8_t *in, size_t nIn, const std::vector<Channel> &ch, int width, int lines,
                   std::vector<uint8_t> &out, std::string &err) {
    struct CD { size_t start; int nx, ny, size; };
    std::vector<CD> cd(ch.size());
    size_t total = 0;
    for (size_t i = 0; i < ch.size(); ++i) {
        cd[i].start = total;
        cd[i].nx = width;
        cd[i].ny = lines;
        cd[i].size = ch[i].type == 1 ? 1 : 2;
        total += (size_t)cd[i].nx * cd[i].ny * cd[i].size;
    }
    if (nIn < 4) { err = "PIZ: truncated block"; return false; }
    const uint16_t minNZ = rdU16(in), maxNZ = rdU16(in + 2);
    size_t p = 4;
    std::vector<uint8_t> bitmap(8192, 0);
    if (maxNZ >= 8192) { err = "PIZ: bad bitmap range"; return false; }
    if (minNZ <= maxNZ) {
        const size_t nb = (size_t)maxNZ - minNZ + 1;
        if (p + nb > nIn) { err = "PIZ: truncated bitmap"; return false; }
        memcpy(&bitmap[minNZ], in + p, nb);
        p += nb;
    }
    // reverseLutFromBitmap
    std::vector<uint16_t> lut(65536, 0);
    int k = 0;
    for (int i = 0; i < 65536; ++i)
        if (i == 0 || (bitmap[i >> 3] & (1 << (i & 7)))) lut[k++] = (uint16_t)i;
    const uint16_t maxValue = (uint16_t)(k - 1);
    if (p + 4 > nIn) { err = "PIZ: truncated block"; return false; }
    const uint32_t length = rdU32(in + p);
    p += 4;
    if (p + length > nIn) { err = "PIZ: Huffman block exceeds the chunk"; return false; }
    std::vector<uint16_t> tmp(total);
    if (!hufUncompress(in + p, length, tmp.data(), total, err)) return false;
    for (size_t i = 0; i < ch.size(); ++i)
        for (int j = 0; j < cd[i].size; ++j)
            wav2Decode(tmp.data() + cd[i].start + j, cd[i].nx, cd[i].size, cd[i].ny, cd[i].nx * cd[i].size, maxValue);
    for (auto &v : tmp) v = lut[v];   // applyLut
    out.resize(total * 2);
    size_t o = 0;
    std::vector<size_t> cur(ch.size());
    for (size_t i = 0; i < ch.size(); ++i) cur[i] = cd[i].start;
    for (int y = 0; y < lines; ++y)
        for (size_t i = 0; i < ch.size(); ++i)
            for (int x = 0; x < cd[i].nx * cd[i].size; ++x) {
                const uint16_t v = tmp[cur[i]++];
                out[o++] = (uint8_t)(v & 0xFF);
                out[o++] = (uint8_t)(v >> 8);
            }
    return true;
}

// ZIP / ZIPS: zlib, then the predictor and the two-half interleave
bool zipUncompress(const uint8_t *in, size_t nIn, size_t nOut, std::vector<uint8_t> &out, std::string &err) {
    std::vector<uint8_t> t(nOut);
    uLongf dl = (uLongf)nOut;
    if (uncompress(t.data(), &dl, in, (uLong)nIn) != Z_OK || dl != nOut) { err = "ZIP: zlib error"; return false; }
    for (size_t i = 1; i < nOut; ++i) t[i] = (uint8_t)(t[i - 1] + t[i] - 128);
    out.resize(nOut);
    const size_t half = (nOut + 1) / 2;
    for (size_t i = 0, a = 0, b = half; i < nOut; ++i) out[i] = (i & 1) ? t[b++] : t[a++];
    return true;
}

bool rleUncompress(const uint8_t *in, size_t nIn, size_t nOut, std::vector<uint8_t> &out, std::string &err) {
    std::vector<uint8_t> t;
    t.reserve(nOut);
    size_t p = 0;
    while (p < nIn) {
        const int8_t c = (int8_t)in[p++];
        if (c < 0) {
            const size_t n = (size_t)(-c);
            if (p + n > nIn) { err = "RLE: truncated"; return false; }
            t.insert(t.end(), in + p, in + p + n);
            p += n;
        } else {
            if (p >= nIn) { err = "RLE: truncated"; return false; }
            t.insert(t.end(), (size_t)c + 1, in[p++]);
        }
    }
    if (t.size() != nOut) { err = "RLE: size mismatch"; return false; }
    for (size_t i = 1; i < nOut; ++i) t[i] = (uint8_t)(t[i - 1] + t[i] - 128);
    out.resize(nOut);
    const size_t half = (nOut + 1) / 2;
    for (size_t i = 0, a = 0, b = half; i < nOut; ++i) out[i] = (i & 1) ? t[b++] : t[a++];
    return true;
}

}  // namespace

bool readEXR(const std::string &path, int &w, int &h, std::vector<float> &rgb, std::string &err) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) { err = "cannot open " + path; return false; }
    std::vector<uint8_t> d;
    uint8_t buf[65536];
    size_t r;
    while ((r = fread(buf, 1, sizeof(buf), f)) > 0) d.insert(d.end(), buf, buf + r);
    fclose(f);
    if (d.size() < 8 || rdU32(d.data()) != 20000630u) { err = "not an OpenEXR file"; return false; }
    const uint32_t version = rdU32(d.data() + 4);
    if ((version & 0xFF) != 2 || (version & 0x200) || (version & 0x1000) || (version & 0x800)) {
        err = "OpenEXR: only single-part scanline files are supported";
        return false;
    }
    size_t p = 8;
    auto cstr = [&](std::string &s) {
        s.clear();
        while (p < d.size() && d[p]) s.push_back((char)d[p++]);
        if (p >= d.size()) return false;
        ++p;
        return true;
    };
    std::vector<Channel> ch;
    int compression = -1, xmin = 0, ymin = 0, xmax = -1, ymax = -1, lineOrder = 0;
    for (;;) {
        std::string name, type;
        if (!cstr(name)) { err = "OpenEXR: truncated header"; return false; }
        if (name.empty()) break;
        if (!cstr(type) || p + 4 > d.size()) { err = "OpenEXR: truncated header"; return false; }
        const uint32_t size = rdU32(&d[p]);
        p += 4;
        if (p + size > d.size()) { err = "OpenEXR: truncated header"; return false; }
        const uint8_t *v = &d[p];
        if (name == "channels") {
            size_t q = 0;
            while (q < size && v[q]) {
                Channel c;
                while (q < size && v[q]) c.name.push_back((char)v[q++]);
                ++q;
                if (q + 16 > size) { err = "OpenEXR: bad channel list"; return false; }
                c.type = (int)rdU32(v + q);
                c.xs = (int)rdU32(v + q + 8);
                c.ys = (int)rdU32(v + q + 12);
                q += 16;
                ch.push_back(c);
            }
        } else if (name == "compression") {
            if (size < 1) { err = "OpenEXR: bad compression attribute"; return false; }
            compression = v[0];
        } else if (name == "dataWindow") {
            if (size < 16) { err = "OpenEXR: bad dataWindow attribute"; return false; }
            xmin = (int)rdU32(v); ymin = (int)rdU32(v + 4); xmax = (int)rdU32(v + 8); ymax = (int)rdU32(v + 12);
        } else if (name == "lineOrder") {
            if (size < 1) { err = "OpenEXR: bad lineOrder attribute"; return false; }
            lineOrder = v[0];
        }
        p += size;
    }
    if (ch.empty() || xmax < xmin || ymax < ymin) { err = "OpenEXR: missing channels or data window"; return false; }
    for (auto &c : ch)
        if (c.xs != 1 || c.ys != 1 || (c.type != 1 && c.type != 2)) { err = "OpenEXR: only full-resolution HALF/FLOAT channels are supported"; return false; }
    (void)lineOrder;   // chunks carry their own y
    // the window in 64 bits: a hostile one must not overflow w, h or w * h * 3
    const int64_t w64 = (int64_t)xmax - xmin + 1, h64 = (int64_t)ymax - ymin + 1;
    if (w64 > (1 << 20) || h64 > (1 << 20) || w64 * h64 > (int64_t)1 << 30) {
        err = "OpenEXR: data window of " + std::to_string(w64) + " x " + std::to_string(h64) + " pixels is too large";
        return false;
    }
    w = (int)w64;
    h = (int)h64;
    int linesPerChunk;
    switch (compression) {
        case 0: case 1: case 2: linesPerChunk = 1; break;
        case 3: linesPerChunk = 16; break;
        case 4: linesPerChunk = 32; break;
        default: err = "OpenEXR: compression " + std::to_string(compression) + " is not supported (NO, RLE, ZIPS, ZIP, PIZ)"; return false;
    }
    // channels are stored sorted by name (R, G, B picked as Bitmap::readOpenEXR does)
    std::vector<int> order(ch.size());
    for (size_t i = 0; i < ch.size(); ++i) order[i] = (int)i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return ch[a].name < ch[b].name; });
    std::vector<Channel> sorted;
    for (int i : order) sorted.push_back(ch[i]);
    ch = sorted;
    auto lower = [](std::string s) { for (auto &c : s) c = (char)tolower((unsigned char)c); return s; };
    auto match = [&](const char *a, const char *b) {
        for (size_t i = 0; i < ch.size(); ++i) {
            const std::string n = lower(ch[i].name);
            if (n == a || n == b || (n.size() > 2 && (n.substr(n.size() - 2) == std::string(".") + a)) ||
                (n.size() > strlen(b) + 1 && n.substr(n.size() - strlen(b) - 1) == std::string(".") + b))
                return (int)i;
        }
        return -1;
    };
    int cr = match("r", "red"), cg = match("g", "green"), cb = match("b", "blue"), cy = match("y", "luminance");
    if (!(cr >= 0 && cg >= 0 && cb >= 0) && cy < 0) {
        err = "readOpenEXR(): Don't know how to deal with this file! There was no known pattern of color/luminance/chroma channels.";
        return false;
    }
    const int nChunks = (h + linesPerChunk - 1) / linesPerChunk;
    if (p + 8ull * nChunks > d.size()) { err = "OpenEXR: truncated offset table"; return false; }
    std::vector<uint64_t> offs(nChunks);
    for (int i = 0; i < nChunks; ++i) offs[i] = (uint64_t)rdU32(&d[p + 8 * i]) | (uint64_t)rdU32(&d[p + 8 * i + 4]) << 32;
    size_t pixelBytes = 0;
    for (auto &c : ch) pixelBytes += c.type == 1 ? 2 : 4;
    rgb.assign((size_t)w * h * 3, 0.0f);
    std::vector<uint8_t> lineData;
    for (int ci = 0; ci < nChunks; ++ci) {
        const uint64_t o = offs[ci];
        if (o + 8 > d.size()) { err = "OpenEXR: bad chunk offset"; return false; }
        const int y0 = (int)rdU32(&d[o]) - ymin;
        const uint32_t packed = rdU32(&d[o + 4]);
        if (o + 8 + packed > d.size() || y0 < 0 || y0 >= h) { err = "OpenEXR: bad chunk"; return false; }
        const int lines = std::min(linesPerChunk, h - y0);
        const size_t raw = pixelBytes * w * lines;
        const uint8_t *src = &d[o + 8];
        bool ok = true;
        if (packed >= raw) lineData.assign(src, src + raw);   // stored uncompressed
        else if (compression == 4) ok = pizUncompress(src, packed, ch, w, lines, lineData, err);
        else if (compression == 2 || compression == 3) ok = zipUncompress(src, packed, raw, lineData, err);
        else if (compression == 1) ok = rleUncompress(src, packed, raw, lineData, err);
        else { err = "OpenEXR: compressed chunk without a compressor"; ok = false; }
        if (!ok) return false;
        // scanline layout: per line, per channel (sorted), w values
        size_t q = 0;
        for (int ly = 0; ly < lines; ++ly) {
            float *row = &rgb[(size_t)(y0 + ly) * w * 3];
            for (size_t c = 0; c < ch.size(); ++c) {
                const int dst = (int)c == cr ? 0 : (int)c == cg ? 1 : (int)c == cb ? 2 : ((int)c == cy && cr < 0) ? 3 : -1;
                for (int x = 0; x < w; ++x) {
                    float v;
                    if (ch[c].type == 1) { v = halfToFloat(rdU16(&lineData[q])); q += 2; }
                    else { uint32_t u = rdU32(&lineData[q]); memcpy(&v, &u, 4); q += 4; }
                    if (dst >= 0 && dst < 3) row[3 * x + dst] = v;
                    else if (dst == 3) row[3 * x] = row[3 * x + 1] = row[3 * x + 2] = v;   // luminance image
                }
            }
        }
    }
    return true;
}

}  // namespace mtsh
