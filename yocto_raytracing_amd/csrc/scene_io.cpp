// scene_io.cpp -- .yrtscene / .yrtbvh interchange formats and image output.
//
// .yrtscene (gzip, little-endian; spec DESIGN.md §3) carries exactly the arrays
// raytrace() reads from a loaded reference scene (src/scene.h:26-155): cameras,
// 8-bit textures, materials (ke kd ks kr rs kd_txt ks_txt), shapes (pos norm
// texcoord radius points lines triangles) and instances (frame shape material).
// The reference harness (oracle/ref_harness.cpp) writes the same format from the
// reference's own loader, so product and reference scenes compare byte-for-byte.
//
// Image output restates tonemap + save_hdr_or_ldr (src/image.cpp:55-88).
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "rgbe.h"
#include "yrt_scene.h"

namespace yrt {
namespace {

struct gz_writer {
    gzFile f;
    explicit gz_writer(const std::string& p) : f(gzopen(p.c_str(), "wb6")) {
        if (!f) throw std::runtime_error("cannot write " + p);
    }
    ~gz_writer() { gzclose(f); }
    void raw(const void* p, size_t n) {
        if (n && gzwrite(f, p, (unsigned)n) != (int)n) throw std::runtime_error("gzwrite failed");
    }
    void u32(uint32_t v) { raw(&v, 4); }
    void i32(int32_t v) { raw(&v, 4); }
    template <class T>
    void vec(const std::vector<T>& v) {
        u32((uint32_t)v.size());
        raw(v.data(), v.size() * sizeof(T));
    }
};

struct gz_reader {
    gzFile f;
    std::string path;
    explicit gz_reader(const std::string& p) : f(gzopen(p.c_str(), "rb")), path(p) {
        if (!f) throw std::runtime_error("cannot open filename " + p);
    }
    ~gz_reader() { gzclose(f); }
    void raw(void* p, size_t n) {
        if (n && gzread(f, p, (unsigned)n) != (int)n)
            throw std::runtime_error("truncated scene file " + path);
    }
    uint32_t u32() {
        uint32_t v;
        raw(&v, 4);
        return v;
    }
    int32_t i32() {
        int32_t v;
        raw(&v, 4);
        return v;
    }
    template <class T>
    void vec(std::vector<T>& v, uint32_t limit = 1u << 28) {
        uint32_t n = u32();
        if (n > limit) throw std::runtime_error("corrupt scene file " + path);
        v.resize(n);
        raw(v.data(), (size_t)n * sizeof(T));
    }
};

}  // namespace

void save_yrtscene(const std::string& filename, const scene& scn) {
    gz_writer o(filename);
    o.raw("YRTSCN1", 8);
    o.u32((uint32_t)scn.cameras.size());
    for (auto& c : scn.cameras) {
        o.raw(&c.frame, 48);
        o.raw(&c.fovy, 4);
        o.raw(&c.aspect, 4);
        o.raw(&c.aperture, 4);
        o.raw(&c.focus, 4);
    }
    o.u32((uint32_t)scn.textures.size());
    for (auto& t : scn.textures) {
        o.i32(t.width);
        o.i32(t.height);
        o.raw(t.pixels.data(), t.pixels.size() * 4);
    }
    o.u32((uint32_t)scn.materials.size());
    for (auto& m : scn.materials) {
        o.raw(&m.ke, 12);
        o.raw(&m.kd, 12);
        o.raw(&m.ks, 12);
        o.raw(&m.kr, 12);
        o.raw(&m.rs, 4);
        o.i32(m.kd_txt);
        o.i32(m.ks_txt);
    }
    o.u32((uint32_t)scn.shapes.size());
    for (auto& s : scn.shapes) {
        o.vec(s.pos);
        o.vec(s.norm);
        o.vec(s.texcoord);
        o.vec(s.radius);
        o.vec(s.points);
        o.vec(s.lines);
        o.vec(s.triangles);
    }
    o.u32((uint32_t)scn.instances.size());
    for (auto& i : scn.instances) {
        o.raw(&i.frame, 48);
        o.i32(i.shp);
        o.i32(i.mat);
    }
}

void load_yrtscene(const std::string& filename, scene& scn) {
    gz_reader in(filename);
    char magic[8];
    in.raw(magic, 8);
    if (memcmp(magic, "YRTSCN1", 8) != 0) throw std::runtime_error("not a .yrtscene file: " + filename);
    scn = scene();
    scn.cameras.resize(in.u32());
    for (auto& c : scn.cameras) {
        in.raw(&c.frame, 48);
        in.raw(&c.fovy, 4);
        in.raw(&c.aspect, 4);
        in.raw(&c.aperture, 4);
        in.raw(&c.focus, 4);
    }
    scn.textures.resize(in.u32());
    for (auto& t : scn.textures) {
        t.width = in.i32();
        t.height = in.i32();
        if (t.width < 0 || t.height < 0 || (size_t)t.width * t.height > (1u << 28))
            throw std::runtime_error("corrupt texture in " + filename);
        t.pixels.resize((size_t)t.width * t.height);
        in.raw(t.pixels.data(), t.pixels.size() * 4);
    }
    scn.materials.resize(in.u32());
    for (auto& m : scn.materials) {
        in.raw(&m.ke, 12);
        in.raw(&m.kd, 12);
        in.raw(&m.ks, 12);
        in.raw(&m.kr, 12);
        in.raw(&m.rs, 4);
        m.kd_txt = in.i32();
        m.ks_txt = in.i32();
    }
    scn.shapes.resize(in.u32());
    for (auto& s : scn.shapes) {
        in.vec(s.pos);
        in.vec(s.norm);
        in.vec(s.texcoord);
        in.vec(s.radius);
        in.vec(s.points);
        in.vec(s.lines);
        in.vec(s.triangles);
    }
    scn.instances.resize(in.u32());
    for (auto& i : scn.instances) {
        in.raw(&i.frame, 48);
        i.shp = in.i32();
        i.mat = in.i32();
        if (i.shp < 0 || i.shp >= (int)scn.shapes.size())
            throw std::runtime_error("instance with invalid shape in " + filename);
    }
}

void load_scene_any(const std::string& filename, scene& scn) {
    auto dot = filename.rfind('.');
    std::string ext = dot == std::string::npos ? "" : filename.substr(dot);
    if (ext == ".obj" || ext == ".OBJ")
        load_obj_scene(filename, scn);
    else
        load_yrtscene(filename, scn);
}

void save_yrtbvh(const std::string& filename, const scene& scn) {
    gz_writer o(filename);
    o.raw("YRTBVH1", 8);
    o.u32((uint32_t)scn.shapes.size());
    for (auto& s : scn.shapes) {
        o.vec(s.bvh.nodes);
        o.vec(s.bvh.leaf_prims);
    }
    o.vec(scn.bvh.nodes);
    o.vec(scn.bvh.leaf_prims);
}

// image.cpp:55-77 with exposure 0 (pow(2,0) == 1 exactly), no filmic, srgb on
void tonemap_rgba8(const float* px, int w, int h, unsigned char* out) {
    for (size_t k = 0; k < (size_t)w * h; k++) {
        float r = std::pow(px[k * 4 + 0], 1 / 2.2f);
        float g = std::pow(px[k * 4 + 1], 1 / 2.2f);
        float b = std::pow(px[k * 4 + 2], 1 / 2.2f);
        float a = px[k * 4 + 3];
        out[k * 4 + 0] = (unsigned char)(sclamp(r, 0.0f, 1.0f) * 255);
        out[k * 4 + 1] = (unsigned char)(sclamp(g, 0.0f, 1.0f) * 255);
        out[k * 4 + 2] = (unsigned char)(sclamp(b, 0.0f, 1.0f) * 255);
        out[k * 4 + 3] = (unsigned char)(sclamp(a, 0.0f, 1.0f) * 255);
    }
}

// The 8-bit value of one color channel, (uchar)(clamp(pow(x, 1/2.2), 0, 1) * 255), is a
// non-decreasing step function of x with this host's powf: it is fully described by
// the smallest float reaching each level k = 1..255 (found by bisection over the
// positive float bit patterns, whose integer order is their float order). The device
// tonemap compares against these and so reproduces the host's libm powf bit for bit,
// where a device pow could differ by an ulp at a truncation boundary.
static unsigned char tonemap_channel(float x) {
    return (unsigned char)(sclamp(std::pow(x, 1 / 2.2f), 0.0f, 1.0f) * 255);
}

int tonemap_neg_inf_level() { return tonemap_channel(-HUGE_VALF); }

void tonemap_thresholds(float thr[256]) {
    thr[0] = 0.0f;
    for (int k = 1; k < 256; k++) {
        uint32_t lo = 0, hi = 0x7f800000u;  // f(+0) = 0 < k <= 255 = f(+inf)
        while (hi - lo > 1) {
            const uint32_t mid = lo + (hi - lo) / 2;
            float x;
            memcpy(&x, &mid, 4);
            if (tonemap_channel(x) >= k) hi = mid;
            else lo = mid;
        }
        memcpy(&thr[k], &hi, 4);
        float below;
        memcpy(&below, &lo, 4);
        if (tonemap_channel(thr[k]) < k || tonemap_channel(below) >= k || (k > 1 && thr[k] < thr[k - 1]))
            throw std::runtime_error("tonemap: host powf is not monotone at level " + std::to_string(k));
    }
}

// RGBE bytes of a frame in the layout the scanline writer consumes: for run-length
// encoded widths each row as four planes (all R bytes, all G, all B, all E: the
// per-component runs of stbiw__write_hdr_scanline), otherwise interleaved quadruples.
// The device encoder (render.hip launch_rgbe) produces the same bytes.
void rgbe_encode(const float* px, int w, int h, unsigned char* out) {
    const bool planar = rgbe_rle_width(w);
    for (int j = 0; j < h; j++)
        for (int i = 0; i < w; i++) {
            const float* p = px + ((size_t)j * w + i) * 4;
            unsigned char e[4];
            linear_to_rgbe(p[0], p[1], p[2], e);
            for (int c = 0; c < 4; c++)
                out[planar ? ((size_t)j * 4 + c) * w + i : ((size_t)j * w + i) * 4 + c] = e[c];
        }
}

namespace {
// one component plane of a scanline, run-length encoded as the reference's writer does
// (stb_image_write.h:562-612): literal stretches in records of <= 128 bytes (a count
// byte, then the bytes) up to the next run of >= 3 equal bytes, that run in records of
// <= 127 (128 + count, then the byte), repeated to the end of the plane
void rle_plane(const unsigned char* v, int w, std::vector<unsigned char>& out) {
    int x = 0;
    while (x < w) {
        int run = x;  // first position of a run of three, if one starts before w - 2
        while (run + 2 < w && !(v[run] == v[run + 1] && v[run] == v[run + 2])) run++;
        const bool has_run = run + 2 < w;
        const int lit_end = has_run ? run : w;
        while (x < lit_end) {
            const int n = std::min(lit_end - x, 128);
            out.push_back((unsigned char)n);
            out.insert(out.end(), v + x, v + x + n);
            x += n;
        }
        if (has_run) {
            int end = run;
            while (end < w && v[end] == v[run]) end++;
            while (x < end) {
                const int n = std::min(end - x, 127);
                out.push_back((unsigned char)(128 + n));
                out.push_back(v[x]);
                x += n;
            }
        }
    }
}
}  // namespace

// stbi_write_hdr (stb_image_write.h:617-637): its header lines, then per row either the
// flat quadruples or {2, 2, w >> 8, w & 255} and the four run-length encoded planes
void save_hdr_rgbe(const std::string& filename, const unsigned char* rgbe, int w, int h) {
    std::vector<unsigned char> buf;
    const std::string head = "#?RADIANCE\n# Written by stb_image_write.h\nFORMAT=32-bit_rle_rgbe\n"
                             "EXPOSURE=          1.0000000000000\n\n-Y " +
                             std::to_string(h) + " +X " + std::to_string(w) + "\n";
    buf.insert(buf.end(), head.begin(), head.end());
    const size_t row = (size_t)w * 4;
    if (!rgbe_rle_width(w)) {
        buf.insert(buf.end(), rgbe, rgbe + row * h);
    } else {
        for (int j = 0; j < h; j++) {
            const unsigned char hdr[4] = {2, 2, (unsigned char)((w & 0xff00) >> 8), (unsigned char)(w & 0xff)};
            buf.insert(buf.end(), hdr, hdr + 4);
            for (int c = 0; c < 4; c++) rle_plane(rgbe + (size_t)j * row + (size_t)c * w, w, buf);
        }
    }
    FILE* f = fopen(filename.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + filename);
    const size_t wrote = fwrite(buf.data(), 1, buf.size(), f);
    const int closed = fclose(f);
    if (wrote != buf.size() || closed != 0) throw std::runtime_error("cannot write " + filename);
}

void save_hdr_or_ldr(const std::string& filename, const float* px, int w, int h) {
    const bool hdr = filename.size() >= 4 && filename.substr(filename.size() - 4) == ".hdr";
    if (hdr) {
        std::vector<unsigned char> rgbe((size_t)w * h * 4);
        rgbe_encode(px, w, h, rgbe.data());
        save_hdr_rgbe(filename, rgbe.data(), w, h);
    } else {
        std::vector<unsigned char> ldr((size_t)w * h * 4);
        tonemap_rgba8(px, w, h, ldr.data());
        save_ldr_png(filename, ldr.data(), w, h);
    }
}

void save_ldr_png(const std::string& filename, const unsigned char* rgba8, int w, int h) {
    std::vector<unsigned char> png;
    png_encode_rgba8(rgba8, w, h, png);
    FILE* f = fopen(filename.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + filename);
    const size_t wrote = fwrite(png.data(), 1, png.size(), f);
    fclose(f);
    if (wrote != png.size()) throw std::runtime_error("cannot write " + filename);
}

}  // namespace yrt
