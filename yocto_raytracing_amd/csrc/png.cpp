// png.cpp -- PNG decode/encode over zlib, replacing the reference's stb_image /
// stb_image_write use (src/image.cpp:25-47).
//
// Decode reproduces stbi_load(path, &w, &h, &n, 4) for non-interlaced PNGs:
// grey / grey+alpha / RGB / RGBA / palette at 1-8 bits, and 16-bit samples
// reduced to their high byte (stb's 16->8 conversion). Missing alpha becomes 255,
// palette alpha comes from tRNS. Gamma chunks are ignored, as stb does.
// Encode writes 8-bit RGBA with filter 0 (any valid PNG is acceptable: the
// reference's stbi_write_png bytes are not part of the parity contract, only pixels).
#include <zlib.h>

#include <cstring>
#include <string>
#include <vector>

#include "yrt_scene.h"

namespace yrt {
namespace {

uint32_t be32(const unsigned char* p) {
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

int paeth(int a, int b, int c) {
    int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p,
        pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return a;
    if (pb <= pc) return b;
    return c;
}

}  // namespace

bool png_decode_rgba8(const std::vector<unsigned char>& f, int& w, int& h,
                      std::vector<unsigned char>& rgba, std::string& err) {
    static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (f.size() < 8 || memcmp(f.data(), sig, 8) != 0) {
        err = "not a png";
        return false;
    }
    size_t pos = 8;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<unsigned char> idat, plte, trns;
    while (pos + 12 <= f.size()) {
        uint32_t len = be32(&f[pos]);
        if (pos + 12 + (size_t)len > f.size()) break;
        const unsigned char* type = &f[pos + 4];
        const unsigned char* data = &f[pos + 8];
        if (!memcmp(type, "IHDR", 4) && len >= 13) {
            w = (int)be32(data);
            h = (int)be32(data + 4);
            depth = data[8];
            ctype = data[9];
            interlace = data[12];
        } else if (!memcmp(type, "PLTE", 4)) {
            plte.assign(data, data + len);
        } else if (!memcmp(type, "tRNS", 4)) {
            trns.assign(data, data + len);
        } else if (!memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), data, data + len);
        } else if (!memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + len;
    }
    if (ctype < 0 || w <= 0 || h <= 0) {
        err = "bad png header";
        return false;
    }
    if (interlace) {
        err = "interlaced png not supported";
        return false;
    }
    int chans = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    if (!chans || !(depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)) {
        err = "unsupported png format";
        return false;
    }
    size_t bits_pp = (size_t)chans * depth;
    size_t stride = ((size_t)w * bits_pp + 7) / 8;
    size_t bpp = (bits_pp + 7) / 8;  // filter byte distance
    std::vector<unsigned char> raw((stride + 1) * h);
    uLongf rawlen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawlen, idat.data(), (uLong)idat.size()) != Z_OK ||
        rawlen != raw.size()) {
        err = "png inflate failed";
        return false;
    }
    std::vector<unsigned char> img(stride * h), zero(stride, 0);
    for (int y = 0; y < h; y++) {
        const unsigned char* in = &raw[y * (stride + 1)];
        int ft = in[0];
        in++;
        unsigned char* out = &img[y * stride];
        const unsigned char* prev = y ? &img[(y - 1) * stride] : zero.data();
        for (size_t x = 0; x < stride; x++) {
            int a = x >= bpp ? out[x - bpp] : 0, b = prev[x], c = x >= bpp ? prev[x - bpp] : 0;
            int v = in[x];
            switch (ft) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: v += paeth(a, b, c); break;
                default: err = "bad png filter"; return false;
            }
            out[x] = (unsigned char)v;
        }
    }
    rgba.assign((size_t)w * h * 4, 0);
    auto sample = [&](const unsigned char* row, int x, int c) -> int {
        if (depth == 8) return row[x * chans + c];
        if (depth == 16) return row[(x * chans + c) * 2];  // high byte
        int idx = x * chans + c;
        int per = 8 / depth;
        int byte = row[idx / per];
        int shift = 8 - depth * (idx % per + 1);
        return (byte >> shift) & ((1 << depth) - 1);
    };
    // stb scales sub-8-bit grey up to 8 bits; palette indices stay indices
    int scale = depth == 1 ? 0xff : depth == 2 ? 0x55 : depth == 4 ? 0x11 : 1;
    for (int y = 0; y < h; y++) {
        const unsigned char* row = &img[y * stride];
        for (int x = 0; x < w; x++) {
            unsigned char* o = &rgba[((size_t)y * w + x) * 4];
            if (ctype == 3) {
                int i = sample(row, x, 0);
                o[0] = 3 * i + 2 < (int)plte.size() ? plte[3 * i] : 0;
                o[1] = 3 * i + 2 < (int)plte.size() ? plte[3 * i + 1] : 0;
                o[2] = 3 * i + 2 < (int)plte.size() ? plte[3 * i + 2] : 0;
                o[3] = i < (int)trns.size() ? trns[i] : 255;
            } else if (ctype == 0 || ctype == 4) {
                int g = sample(row, x, 0) * (depth < 8 ? scale : 1);
                o[0] = o[1] = o[2] = (unsigned char)g;
                o[3] = ctype == 4 ? (unsigned char)sample(row, x, 1) : 255;
            } else {
                o[0] = (unsigned char)sample(row, x, 0);
                o[1] = (unsigned char)sample(row, x, 1);
                o[2] = (unsigned char)sample(row, x, 2);
                o[3] = ctype == 6 ? (unsigned char)sample(row, x, 3) : 255;
            }
        }
    }
    return true;
}

bool png_encode_rgba8(const unsigned char* rgba, int w, int h, std::vector<unsigned char>& out) {
    std::vector<unsigned char> raw((size_t)(w * 4 + 1) * h);
    for (int y = 0; y < h; y++) {
        raw[(size_t)y * (w * 4 + 1)] = 0;
        memcpy(&raw[(size_t)y * (w * 4 + 1) + 1], rgba + (size_t)y * w * 4, (size_t)w * 4);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<unsigned char> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return false;
    z.resize(zlen);
    out.clear();
    static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    out.insert(out.end(), sig, sig + 8);
    auto chunk = [&](const char* type, const unsigned char* d, size_t n) {
        unsigned char hdr[8] = {(unsigned char)(n >> 24), (unsigned char)(n >> 16),
                                (unsigned char)(n >> 8), (unsigned char)n,
                                (unsigned char)type[0], (unsigned char)type[1],
                                (unsigned char)type[2], (unsigned char)type[3]};
        out.insert(out.end(), hdr, hdr + 8);
        out.insert(out.end(), d, d + n);
        uLong crc = crc32(0, (const Bytef*)type, 4);
        crc = crc32(crc, d, (uInt)n);
        unsigned char c[4] = {(unsigned char)(crc >> 24), (unsigned char)(crc >> 16),
                              (unsigned char)(crc >> 8), (unsigned char)crc};
        out.insert(out.end(), c, c + 4);
    };
    unsigned char ihdr[13] = {(unsigned char)(w >> 24), (unsigned char)(w >> 16),
                              (unsigned char)(w >> 8),  (unsigned char)w,
                              (unsigned char)(h >> 24), (unsigned char)(h >> 16),
                              (unsigned char)(h >> 8),  (unsigned char)h,
                              8, 6, 0, 0, 0};
    chunk("IHDR", ihdr, 13);
    chunk("IDAT", z.data(), z.size());
    chunk("IEND", nullptr, 0);
    return true;
}

}  // namespace yrt
