// MIP pyramids (host side) shared by the environment emitter and the
// `bitmap` texture, plus the PNG reader and the texel conversion of the
// bitmap plugin.
//
//   TMIPMap constructor   include/mitsuba/render/mipmap.h:155-302: level
//                         count from (w + 1) / 2 halving, level k+1 =
//                         Bitmap::resample of the float level k with a
//                         2-lobe Lanczos filter and the u / v boundary
//                         conditions, clamped to [0, maxValue]
//                         (src/libcore/bitmap.cpp:2230-2330 driving
//                         Resampler, include/mitsuba/core/rfilter.h:107-460);
//                         levels are stored in half precision; nearest and
//                         bilinear pyramids keep level 0 only
//   BitmapTexture         src/textures/bitmap.cpp:179-302: load, convert to
//                         linear float RGB (fmtconv.cpp:1093-1160), MIP map
//   readPNG               src/libcore/bitmap.cpp:2460-2560 (libpng with
//                         palette / low-bit gray expansion; gamma from the
//                         sRGB / gAMA chunks, sRGB by default)
#include <zlib.h>

#include <cmath>
#include <cstring>
#include <fstream>
#include <limits>
#include <stdexcept>

#include "scene.h"

namespace mtsh {

// IEEE binary16 round trip, round-to-nearest-even (OpenEXR's half(float)).
float toHalfAndBack(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = x & 0x80000000u;
    const uint32_t ax = x & 0x7FFFFFFFu;
    uint16_t h;
    if (ax >= 0x7F800000u) {                       // inf / nan
        h = (uint16_t)(ax > 0x7F800000u ? 0x7E00 : 0x7C00);
    } else if (ax >= 0x477FF000u) {                // rounds to >= 65520 -> inf
        h = 0x7C00;
    } else if (ax < 0x38800000u) {                 // half subnormal / zero
        if (ax < 0x33000000u) {
            h = 0;
        } else {
            const uint32_t e = ax >> 23, m = (ax & 0x7FFFFFu) | 0x800000u;
            const uint32_t shift = 126 - e;        // 14 - (e - 112)
            uint32_t hm = m >> shift;
            const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
            if (rem > half || (rem == half && (hm & 1u))) ++hm;
            h = (uint16_t)hm;
        }
    } else {
        uint32_t v = ax - 0x38000000u;             // rebias exponent 127 -> 15
        const uint32_t rem = v & 0x1FFFu;
        v >>= 13;
        if (rem > 0x1000u || (rem == 0x1000u && (v & 1u))) ++v;
        h = (uint16_t)v;
    }
    // back to float
    const uint32_t he = (h >> 10) & 0x1Fu, hm = h & 0x3FFu;
    uint32_t out;
    if (he == 0) {
        if (hm == 0) {
            out = 0;
        } else {                                   // subnormal
            int e = -1;
            uint32_t m = hm;
            do { ++e; m <<= 1; } while (!(m & 0x400u));
            out = ((uint32_t)(127 - 15 - e) << 23) | ((m & 0x3FFu) << 13);
        }
    } else if (he == 31) {
        out = 0x7F800000u | (hm << 13);
    } else {
        out = ((he + 112) << 23) | (hm << 13);
    }
    out |= sign;
    float r;
    memcpy(&r, &out, 4);
    return r;
}

namespace {

// LanczosSincFilter::eval (src/rfilters/lanczos.cpp:44-56), lobes = 2
float lanczos2(float x) {
    const float radius = 2.0f;
    x = std::fabs(x);
    if (x < 1e-4f) return 1.0f;        // Epsilon
    if (x > radius) return 0.0f;
    const float x1 = (float)(M_PI * x);
    const float x2 = x1 / radius;
    return (std::sin(x1) * std::sin(x2)) / (x1 * x2);
}

int modulo(int a, int b) { int r = a % b; return r < 0 ? r + b : r; }   // math::modulo

// Resampler<float> in resampling mode + resampleAndClamp(min 0, max)
struct Resampler1D {
    int src, dst, taps, bc;
    std::vector<int> start;
    std::vector<float> w;
    Resampler1D(int sourceRes, int targetRes, int bc_) : src(sourceRes), dst(targetRes), bc(bc_) {
        float filterRadius = 2.0f, scale = 1.0f, invScale = 1.0f;
        if (targetRes < sourceRes) {
            scale = (float)sourceRes / (float)targetRes;
            invScale = 1 / scale;
            filterRadius *= scale;
        }
        taps = (int)std::ceil(filterRadius * 2);
        start.resize(targetRes);
        w.resize((size_t)taps * targetRes);
        for (int i = 0; i < targetRes; ++i) {
            const float center = (i + 0.5f) / targetRes * sourceRes;
            start[i] = (int)std::floor(center - filterRadius + 0.5f);
            float sum = 0;
            for (int j = 0; j < taps; ++j) {
                const float pos = start[i] + j + 0.5f - center;
                const float weight = lanczos2(pos * invScale);
                w[(size_t)i * taps + j] = weight;
                sum += weight;
            }
            const float normalization = 1.0f / sum;
            for (int j = 0; j < taps; ++j) w[(size_t)i * taps + j] = w[(size_t)i * taps + j] * normalization;
        }
    }
    // Resampler::lookup (rfilter.h:436-458)
    float lookup(const float *source, int pos, size_t stride, int ch) const {
        if (pos < 0 || pos >= src) {
            switch (bc) {
                case MTSG_WRAP_CLAMP: pos = std::min(std::max(pos, 0), src - 1); break;
                case MTSG_WRAP_REPEAT: pos = modulo(pos, src); break;
                case MTSG_WRAP_MIRROR:
                    pos = modulo(pos, 2 * src);
                    if (pos >= src) pos = 2 * src - pos - 1;
                    break;
                case MTSG_WRAP_ZERO: return 0.0f;
                default: return 1.0f;   // EOne
            }
        }
        return source[stride * pos + ch];
    }
    // source/target: element i at base + stride * i, 3 channels each
    void run(const float *source, size_t srcStride, float *target, size_t dstStride, float maxValue) const {
        for (int i = 0; i < dst; ++i)
            for (int ch = 0; ch < 3; ++ch) {
                float result = 0;
                for (int j = 0; j < taps; ++j) result += lookup(source, start[i] + j, srcStride, ch) * w[(size_t)i * taps + j];
                target[dstStride * i + ch] = std::min(maxValue, std::max(0.0f, result));
            }
    }
};

// Bitmap::resample(lanczos2, bcu, bcv, size, 0, maxValue): x pass, then y
std::vector<float> resample(const std::vector<float> &src, int sw, int sh, int tw, int th, int bcu, int bcv, float maxValue) {
    std::vector<float> tmp;
    const std::vector<float> *cur = &src;
    int cw = sw;
    if (sw != tw) {
        Resampler1D r(sw, tw, bcu);
        tmp.assign((size_t)tw * sh * 3, 0.0f);
        for (int y = 0; y < sh; ++y) r.run(src.data() + (size_t)y * sw * 3, 3, tmp.data() + (size_t)y * tw * 3, 3, maxValue);
        cur = &tmp;
        cw = tw;
    }
    if (sh == th) return *cur;
    Resampler1D r(sh, th, bcv);
    std::vector<float> out((size_t)cw * th * 3, 0.0f);
    for (int x = 0; x < cw; ++x)
        r.run(cur->data() + (size_t)x * 3, (size_t)cw * 3, out.data() + (size_t)x * 3, (size_t)cw * 3, maxValue);
    return out;
}

}  // namespace

void buildMipmap(std::vector<float> level, int W, int H, int filter, int wrapU, int wrapV, float maxValue,
                 float maxAnisotropy, std::vector<float> &texels, mtsg_mipmap &mip, float average[3], float maximum[3]) {
    memset(&mip, 0, sizeof(mip));
    if (W <= 0 || H <= 0 || level.size() != (size_t)W * H * 3) throw std::runtime_error("MIP map: bad level-0 image");
    // level 0: component-wise min / max / average of the float image
    // (BlockedArray::init, barray.h:103-126); negative values are clamped
    // and the statistics recomputed (mipmap.h:232-240)
    auto stats = [&]() {
        float mn[3], mx[3], avg[3];
        for (int c = 0; c < 3; ++c) { mn[c] = std::numeric_limits<float>::infinity(); mx[c] = -mn[c]; avg[c] = 0; }
        for (size_t i = 0; i < (size_t)W * H; ++i)
            for (int c = 0; c < 3; ++c) {
                const float v = level[3 * i + c];
                mn[c] = std::min(mn[c], v);
                mx[c] = std::max(mx[c], v);
                avg[c] += v;
            }
        for (int c = 0; c < 3; ++c) {
            if (average) average[c] = avg[c] / (float)((size_t)W * H);
            if (maximum) maximum[c] = mx[c];
        }
        return std::min(mn[0], std::min(mn[1], mn[2]));
    };
    if (stats() < 0) {
        for (auto &v : level) if (v < 0) v = 0;   // Spectrum::clampNegative
        stats();
    }
    const bool pyramid = filter != MTSG_MIP_NEAREST && filter != MTSG_MIP_BILINEAR;
    int levels = 1;
    if (pyramid) {
        int w = W, h = H;
        while (w > 1 || h > 1) { w = std::max(1, (w + 1) / 2); h = std::max(1, (h + 1) / 2); ++levels; }
    }
    if (levels > MTSG_MIPMAP_MAX_LEVELS) throw std::runtime_error("MIP map: too many levels");
    mip.levels = levels;
    mip.filter = filter;
    mip.wrap_u = wrapU;
    mip.wrap_v = wrapV;
    mip.max_anisotropy = filter == MTSG_MIP_EWA ? maxAnisotropy : 1.0f;
    int w = W, h = H;
    for (int l = 0; l < levels; ++l) {
        if (l > 0) {
            const int nw = std::max(1, (w + 1) / 2), nh = std::max(1, (h + 1) / 2);
            level = resample(level, w, h, nw, nh, wrapU, wrapV, maxValue);
            w = nw; h = nh;
        }
        mip.level_w[l] = w;
        mip.level_h[l] = h;
        mip.level_offset[l] = (uint32_t)texels.size();
        mip.size_ratio_x[l] = (float)w / (float)W;
        mip.size_ratio_y[l] = (float)h / (float)H;
        for (float v : level) texels.push_back(toHalfAndBack(v));   // SpectrumHalf storage
    }
    // EWA weights: math::fastexp(-2 r^2) - fastexp(-2) (mipmap.h:296-301)
    for (int i = 0; i < MTSG_MIPMAP_LUT_SIZE; ++i) {
        const float r2 = (float)i / (float)(MTSG_MIPMAP_LUT_SIZE - 1);
        mip.weight_lut[i] = (float)std::exp((double)(-2.0f * r2)) - (float)std::exp(-2.0);
    }
}

// ---------------------------------------------------------------------------
// PNG (RFC 2083): chunk walk, zlib inflate of the IDAT stream, scanline
// unfiltering, libpng's expansions as the reference requests them
// ---------------------------------------------------------------------------
namespace {
uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}
}  // namespace

bool readPNG(const std::string &path, PngImage &img, std::string &err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { err = "cannot open"; return false; }
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (buf.size() < 8 || memcmp(buf.data(), sig, 8) != 0) { err = "not a PNG file"; return false; }
    uint32_t W = 0, H = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, palette;
    bool srgb = false, hasGama = false;
    uint32_t gama = 0;
    size_t pos = 8;
    while (pos + 12 <= buf.size()) {
        const uint32_t len = be32(&buf[pos]);
        if (pos + 12 + (size_t)len > buf.size()) { err = "truncated chunk"; return false; }
        const std::string type((const char *)&buf[pos + 4], 4);
        const uint8_t *data = &buf[pos + 8];
        if (type == "IHDR") {
            if (len < 13) { err = "bad IHDR"; return false; }
            W = be32(data); H = be32(data + 4);
            depth = data[8]; ctype = data[9]; interlace = data[12];
            if (data[10] != 0 || data[11] != 0) { err = "unknown compression / filter method"; return false; }
        } else if (type == "PLTE") {
            palette.assign(data, data + len);
        } else if (type == "IDAT") {
            idat.insert(idat.end(), data, data + len);
        } else if (type == "sRGB") {
            srgb = true;
        } else if (type == "gAMA" && len >= 4) {
            hasGama = true;
            gama = be32(data);
        } else if (type == "IEND") {
            break;
        }
        pos += 12 + len;
    }
    if (W == 0 || H == 0 || ctype < 0) { err = "missing IHDR"; return false; }
    if (interlace != 0) { err = "interlaced (Adam7) PNG files are not supported by this build"; return false; }
    int channels;
    switch (ctype) {
        case 0: channels = 1; break;
        case 2: channels = 3; break;
        case 3: channels = 1; break;
        case 4: channels = 2; break;
        case 6: channels = 4; break;
        default: err = "unknown color type " + std::to_string(ctype); return false;
    }
    if (ctype == 0 && depth == 1) { err = "1-bit (bitmask) PNG files are not supported by this build"; return false; }
    if ((ctype != 0 && ctype != 3 && depth < 8) || (depth != 1 && depth != 2 && depth != 4 && depth != 8 && depth != 16) ||
        (ctype == 3 && depth > 8)) {
        err = "unsupported bit depth " + std::to_string(depth);
        return false;
    }
    if (ctype == 3 && palette.empty()) { err = "palette image without PLTE"; return false; }
    const size_t bitsPerPixel = (size_t)channels * depth;
    const size_t rowBytes = (W * bitsPerPixel + 7) / 8, bpp = std::max<size_t>(1, bitsPerPixel / 8);
    std::vector<uint8_t> raw((rowBytes + 1) * H);
    uLongf rawLen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawLen, idat.data(), (uLong)idat.size()) != Z_OK || rawLen != raw.size()) {
        err = "corrupt image data";
        return false;
    }
    std::vector<uint8_t> prev(rowBytes, 0), cur(rowBytes);
    // output: 8-bit or 16-bit samples, palette expanded to RGB, 2/4-bit gray to 8 bits
    const int outCh = ctype == 3 ? 3 : channels;
    const int outDepth = depth == 16 ? 16 : 8;
    img.width = (int)W;
    img.height = (int)H;
    img.channels = outCh;
    img.depth = outDepth;
    img.samples.assign((size_t)W * H * outCh, 0);
    for (uint32_t y = 0; y < H; ++y) {
        const uint8_t *line = &raw[y * (rowBytes + 1)];
        const int ft = line[0];
        for (size_t i = 0; i < rowBytes; ++i) {
            const int x = line[1 + i], a = i >= bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
            int v;
            switch (ft) {
                case 0: v = x; break;
                case 1: v = x + a; break;
                case 2: v = x + b; break;
                case 3: v = x + ((a + b) >> 1); break;
                case 4: v = x + paeth(a, b, c); break;
                default: err = "bad filter type"; return false;
            }
            cur[i] = (uint8_t)v;
        }
        uint16_t *out = &img.samples[(size_t)y * W * outCh];
        for (uint32_t x = 0; x < W; ++x) {
            if (depth == 16) {
                for (int c = 0; c < channels; ++c) out[x * outCh + c] = (uint16_t)(cur[2 * (x * channels + c)] << 8 | cur[2 * (x * channels + c) + 1]);
            } else if (depth == 8) {
                if (ctype == 3) {
                    const size_t idx = cur[x];
                    if (3 * idx + 2 >= palette.size()) { err = "palette index out of range"; return false; }
                    for (int c = 0; c < 3; ++c) out[x * 3 + c] = palette[3 * idx + c];
                } else {
                    for (int c = 0; c < channels; ++c) out[x * outCh + c] = cur[x * channels + c];
                }
            } else {   // 1/2/4-bit palette indices or 2/4-bit gray
                const size_t bit = (size_t)x * depth;
                const int v = (cur[bit / 8] >> (8 - depth - (int)(bit % 8))) & ((1 << depth) - 1);
                if (ctype == 3) {
                    if (3 * (size_t)v + 2 >= palette.size()) { err = "palette index out of range"; return false; }
                    for (int c = 0; c < 3; ++c) out[x * 3 + c] = palette[3 * v + c];
                } else {
                    out[x] = (uint16_t)(v * (255 / ((1 << depth) - 1)));   // png_set_expand_gray_1_2_4_to_8
                }
            }
        }
        std::swap(prev, cur);
    }
    // Bitmap::readPNG gamma (bitmap.cpp:2534-2541)
    if (srgb) img.gamma = -1.0f;
    else if (hasGama && gama != 0) img.gamma = (float)1 / (float)((double)gama / 100000.0);
    else img.gamma = -1.0f;
    return true;
}

namespace {
// FormatConverterImpl::undoGamma (src/libcore/fmtconv.cpp:1093-1102)
float undoGamma(float value, float gamma) {
    if (gamma == -1) {
        if (value <= (float)0.04045) return value * (float)(1.0 / 12.92);
        return std::pow((float)((value + (float)0.055) * (float)(1.0 / 1.055)), (float)2.4);
    }
    return std::pow(value, gamma);
}
bool endsWith(const std::string &s, const std::string &e) {
    if (s.size() < e.size()) return false;
    for (size_t i = 0; i < e.size(); ++i)
        if (std::tolower((unsigned char)s[s.size() - e.size() + i]) != e[i]) return false;
    return true;
}
}  // namespace

// Bitmap(EAuto) + expand()->convert(ERGB / ELuminance, EFloat, gamma 1)
// (bitmap.cpp:179-302, fmtconv.cpp:109-160, 1137-1160): linear float RGB,
// one channel broadcast (MIPMap1 and MIPMap3 give the same values), alpha
// dropped.  gammaOverride != 0 replaces the file's gamma (Bitmap::setGamma).
void loadTextureImage(const std::string &path, float gammaOverride, int &w, int &h, std::vector<float> &rgb) {
    std::string e;
    if (endsWith(path, ".png")) {
        PngImage img;
        if (!readPNG(path, img, e)) throw std::runtime_error("texture \"" + path + "\": " + e);
        const float gamma = gammaOverride != 0 ? gammaOverride : img.gamma;
        const int maxv = img.depth == 16 ? 65535 : 255;
        // convertScalar with the precomputed table of the compact formats:
        // value * (1 / max), then undoGamma (fmtconv.cpp:154-157, 1142-1148)
        std::vector<float> table((size_t)maxv + 1);
        for (int i = 0; i <= maxv; ++i) {
            float v = (float)i * (float)(1.0f / (float)maxv);
            if (gamma != 1) v = undoGamma(v, gamma);
            table[i] = v;
        }
        w = img.width;
        h = img.height;
        rgb.assign((size_t)w * h * 3, 0.0f);
        const int ch = img.channels;
        for (size_t i = 0; i < (size_t)w * h; ++i) {
            const uint16_t *s = &img.samples[i * ch];
            if (ch >= 3) for (int c = 0; c < 3; ++c) rgb[3 * i + c] = table[s[c]];
            else for (int c = 0; c < 3; ++c) rgb[3 * i + c] = table[s[0]];
        }
        return;
    }
    bool ok;
    if (endsWith(path, ".pfm")) ok = readPFM(path, w, h, rgb, e);
    else if (endsWith(path, ".exr")) ok = readEXR(path, w, h, rgb, e);
    else throw std::runtime_error("texture \"" + path + "\": only PNG, OpenEXR and PFM images are supported by this build");
    if (!ok) throw std::runtime_error("texture \"" + path + "\": " + e);
    if (gammaOverride != 0 && gammaOverride != 1)
        for (auto &v : rgb) v = undoGamma(v, gammaOverride);
}

}  // namespace mtsh
