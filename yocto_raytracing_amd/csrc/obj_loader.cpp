// obj_loader.cpp -- host loader for the Yocto-OBJ dialect used by in/*.
//
// The reference loads scenes through three layers; this file restates the
// semantics of all three that change the arrays raytrace() consumes:
//   yobj::load_obj / load_mtl   src/ext/yocto_obj.cpp:212-332, 362-530
//       line tokens v vn vt vc vr f l p o usemtl g s mtllib c i; atof-then-float
//       parsing (:44-61); 1-based/negative index triplets (:86-110); `vt` v flipped to
//       1-v (:410-411, obj_flip_texcoord default true, yocto_scn.h:424); groups split on
//       o/usemtl/g/s (:446-471); empty groups/objects dropped (:501-509)
//   yscn::obj_to_scene          src/ext/yocto_scn.cpp:151-481
//       first-seen vertex de-duplication per group (:299-307); polylines to segments
//       (:333-339); fan triangulation (:349-361); arrays sized by the group's first
//       vertex (:367-388); rs = pow(2/(Ns+2), 1/4) (:253); `i` lines -> one instance
//       per shape of the named object (:469-477)
//   yscn::add_elements          src/ext/yocto_scn.cpp:1533-1665 with the options of
//       src/scene.cpp:124-129 (point/line radius 0.001, shape instances, default camera)
//   load_scene                  src/scene.cpp:113-225
//       8-bit RGBA textures (stbi_load, req_comp 4), per-instance material = the
//       shape's material, smooth normals when a shape has none (scene.cpp:11-31)
// The result is compared byte-for-byte with the reference loader's output
// (tests/test_library.py::test_obj_loader_matches_reference_loader, via the .yrtscene serialisation).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <unordered_map>
#include <unordered_set>

#include "yrt_scene.h"

namespace yrt {
namespace {

struct obj_vert {
    int pos, texcoord, norm, color, radius;  // yocto_obj.h:142-152 order
    bool operator==(const obj_vert& o) const {
        return pos == o.pos && texcoord == o.texcoord && norm == o.norm && color == o.color &&
               radius == o.radius;
    }
};
struct obj_vert_hash {
    size_t operator()(const obj_vert& v) const {
        size_t h = 0;
        const int* p = &v.pos;
        for (int i = 0; i < 5; i++) h ^= std::hash<int>()(p[i]) + 0x9e3779b9 + (h << 6) + (h >> 2);
        return h;
    }
};

enum class elem_kind { point, line, face, tetra };
struct obj_elem {
    uint32_t start;
    elem_kind kind;
    uint16_t size;
};
struct obj_group {
    std::string matname, groupname;
    bool smoothing = true;
    std::vector<obj_vert> verts;
    std::vector<obj_elem> elems;
};
struct obj_object {
    std::string name;
    std::vector<obj_group> groups;
};
struct obj_camera {
    std::string name;
    int ortho = 0;
    float yfov = 2, aspect = 16.0f / 9.0f, aperture = 0, focus = 1;
    frame3f frame = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
};
struct obj_instance {
    std::string name, objname;
    frame3f frame;
};
struct mtl_material {
    std::string name;
    vec3f ke = {0, 0, 0}, kd = {0, 0, 0}, ks = {0, 0, 0}, kr = {0, 0, 0};
    float ns = 1;
    std::string kd_txt, ks_txt;
};
struct obj_file {
    std::vector<vec3f> pos, norm;
    std::vector<vec2f> texcoord;
    std::vector<float> radius;
    std::vector<obj_object> objects;
    std::vector<obj_camera> cameras;
    std::vector<obj_instance> instances;
    std::vector<mtl_material> materials;
    std::vector<std::string> textures;
};

// whitespace tokenizer over a mutable line (yocto_obj.cpp:31-45 semantics)
int split_ws(char* s, char** toks, int maxt) {
    int n = 0;
    bool prev_space = true;
    for (; *s && n < maxt; s++) {
        if (isspace((unsigned char)*s)) {
            *s = 0;
            prev_space = true;
        } else {
            if (prev_space) toks[n++] = s;
            prev_space = false;
        }
    }
    toks[n] = nullptr;
    return n;
}

float tof(const char* t) { return t ? (float)atof(t) : 0.0f; }
int toi(const char* t) { return t ? atoi(t) : 0; }
vec3f tof3(char** t) { return {tof(t[0]), tof(t[1]), tof(t[2])}; }
frame3f tof12(char** t) {
    frame3f f;
    float* m = &f.x.x;
    for (int i = 0; i < 12; i++) m[i] = tof(t[i]);
    return f;
}

std::string dir_of(const std::string& f) {
    auto p = f.rfind('/');
    if (p == std::string::npos) p = f.rfind('\\');
    return p == std::string::npos ? std::string() : f.substr(0, p + 1);
}

std::vector<obj_vert> parse_verts(char** toks, int n, const obj_vert& counts) {
    std::vector<obj_vert> out;
    for (int i = 0; i < n; i++) {
        const char* parts[5] = {toks[i], nullptr, nullptr, nullptr, nullptr};
        int np = 1;
        for (char* c = toks[i]; *c; c++) {
            if (*c == '/') {
                *c = 0;
                if (np < 5) parts[np++] = c + 1;
            }
        }
        obj_vert v;
        int* vp = &v.pos;
        const int* cp = &counts.pos;
        for (int k = 0; k < 5; k++) {
            if (!parts[k]) {
                vp[k] = -1;
                continue;
            }
            int x = atoi(parts[k]);
            vp[k] = x < 0 ? cp[k] + x : x - 1;
        }
        out.push_back(v);
    }
    return out;
}

void add_texture_name(const std::string& p, std::vector<std::string>& list,
                      std::unordered_set<std::string>& seen) {
    if (!p.empty() && !seen.count(p)) {
        list.push_back(p);
        seen.insert(p);
    }
}

// texture statement: options start with '-', the path is the last token
std::string texture_path(char** toks, int n) {
    if (n <= 0) return "";
    std::string p = toks[n - 1];
    for (auto& c : p)
        if (c == '\\') c = '/';
    return p;
}

void load_mtl_file(const std::string& filename, std::vector<mtl_material>& mats,
                   std::vector<std::string>& textures) {
    FILE* f = fopen(filename.c_str(), "rt");
    if (!f) throw std::runtime_error("cannot open filename " + filename);
    std::unordered_set<std::string> seen;
    std::vector<mtl_material> out(1);  // preemptive fake material, dropped below
    char line[4096];
    char* toks[1024];
    while (fgets(line, sizeof line, f)) {
        int n = split_ws(line, toks, 1023);
        if (!n || toks[0][0] == '#') continue;
        std::string k = toks[0];
        char** t = toks + 1;
        int nt = n - 1;
        auto& m = out.back();
        if (k == "newmtl") {
            out.emplace_back();
            out.back().name = nt ? t[0] : "";
        } else if (k == "Ke") {
            m.ke = tof3(t);
        } else if (k == "Kd") {
            m.kd = tof3(t);
        } else if (k == "Ks") {
            m.ks = tof3(t);
        } else if (k == "Kr") {
            m.kr = tof3(t);
        } else if (k == "Ns") {
            m.ns = tof(t[0]);
        } else if (k == "map_Kd") {
            m.kd_txt = texture_path(t, nt);
            add_texture_name(m.kd_txt, textures, seen);
        } else if (k == "map_Ks") {
            m.ks_txt = texture_path(t, nt);
            add_texture_name(m.ks_txt, textures, seen);
        } else if (k == "map_Ke" || k == "map_Ka" || k == "map_Kr" || k == "map_Tr" ||
                   k == "map_Ns" || k == "map_d" || k == "map_Ni" || k == "map_bump" ||
                   k == "bump" || k == "map_disp" || k == "disp" || k == "map_norm" ||
                   k == "norm") {
            // not read by raytrace(), but registered: texture indices depend on them
            add_texture_name(texture_path(t, nt), textures, seen);
        }
    }
    fclose(f);
    out.erase(out.begin());
    mats.insert(mats.end(), out.begin(), out.end());
}

void parse_obj(const std::string& filename, obj_file& obj) {
    FILE* f = fopen(filename.c_str(), "rt");
    if (!f) throw std::runtime_error("cannot open filename " + filename);
    obj.objects.push_back({});
    obj.objects.back().groups.push_back({});
    obj_vert counts = {0, 0, 0, 0, 0};
    std::string cur_mat;
    std::vector<std::string> mtllibs;
    char line[4096];
    char* toks[1024];
    while (fgets(line, sizeof line, f)) {
        int n = split_ws(line, toks, 1023);
        if (!n || toks[0][0] == '#') continue;
        std::string k = toks[0];
        char** t = toks + 1;
        int nt = n - 1;
        if (k == "v") {
            counts.pos++;
            obj.pos.push_back(tof3(t));
        } else if (k == "vn") {
            counts.norm++;
            obj.norm.push_back(tof3(t));
        } else if (k == "vt") {
            counts.texcoord++;
            vec2f uv = {tof(t[0]), tof(t[1])};
            uv.y = 1 - uv.y;  // obj_flip_texcoord
            obj.texcoord.push_back(uv);
        } else if (k == "vc") {
            counts.color++;
        } else if (k == "vr") {
            counts.radius++;
            obj.radius.push_back(tof(t[0]));
        } else if (k == "f" || k == "l" || k == "p" || k == "t") {
            auto vs = parse_verts(t, nt, counts);
            auto& g = obj.objects.back().groups.back();
            elem_kind kind = k == "f"   ? elem_kind::face
                             : k == "l" ? elem_kind::line
                             : k == "p" ? elem_kind::point
                                        : elem_kind::tetra;
            g.elems.push_back({(uint32_t)g.verts.size(), kind, (uint16_t)vs.size()});
            g.verts.insert(g.verts.end(), vs.begin(), vs.end());
        } else if (k == "o") {
            obj.objects.push_back({nt ? t[0] : "", {}});
            obj_group g;
            g.matname = cur_mat;
            obj.objects.back().groups.push_back(g);
        } else if (k == "usemtl") {
            cur_mat = nt ? t[0] : "";
            obj_group g;
            g.matname = cur_mat;
            obj.objects.back().groups.push_back(g);
        } else if (k == "g") {
            obj_group g;
            g.matname = cur_mat;
            g.groupname = nt ? t[0] : "";
            obj.objects.back().groups.push_back(g);
        } else if (k == "s") {
            std::string name = nt ? t[0] : "";
            bool smoothing = name == "on";
            if (obj.objects.back().groups.back().smoothing != smoothing) {
                obj_group g;
                g.matname = cur_mat;
                g.groupname = name;
                g.smoothing = smoothing;
                obj.objects.back().groups.push_back(g);
            }
        } else if (k == "mtllib") {
            std::string name = nt ? t[0] : "";
            if (!name.empty()) {
                bool found = false;
                for (auto& l : mtllibs) found = found || l == name;
                if (!found) mtllibs.push_back(name);
            }
        } else if (k == "c") {
            obj_camera c;
            c.name = nt ? t[0] : "";
            c.ortho = toi(t[1]);
            c.yfov = tof(t[2]);
            c.aspect = tof(t[3]);
            c.aperture = tof(t[4]);
            c.focus = tof(t[5]);
            c.frame = tof12(t + 6);
            obj.cameras.push_back(c);
        } else if (k == "i") {
            obj_instance ist;
            ist.name = nt ? t[0] : "<unnamed>";
            ist.objname = (nt - 1) ? t[1] : "<unnamed_mesh>";
            ist.frame = tof12(t + 2);
            obj.instances.push_back(ist);
        }
    }
    fclose(f);
    for (auto& o : obj.objects) {
        std::vector<obj_group> kept;
        for (auto& g : o.groups)
            if (!g.verts.empty()) kept.push_back(std::move(g));
        o.groups = std::move(kept);
    }
    std::vector<obj_object> kept;
    for (auto& o : obj.objects)
        if (!o.groups.empty()) kept.push_back(std::move(o));
    obj.objects = std::move(kept);

    auto dir = dir_of(filename);
    std::unordered_set<std::string> tseen;
    for (auto& lib : mtllibs) {
        std::vector<std::string> txts;
        load_mtl_file(dir + lib, obj.materials, txts);
        for (auto& tx : txts) add_texture_name(tx, obj.textures, tseen);
    }
}

std::vector<unsigned char> read_file(const std::string& path, bool& ok) {
    std::vector<unsigned char> data;
    FILE* f = fopen(path.c_str(), "rb");
    ok = f != nullptr;
    if (!f) return data;
    unsigned char buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) data.insert(data.end(), buf, buf + n);
    fclose(f);
    return data;
}

// scene.cpp:11-31
void compute_smooth_normals(shape& s) {
    s.norm.assign(s.pos.size(), vec3f{0, 0, 0});
    for (auto l : s.lines) {
        vec3f d = s.pos[l.y] - s.pos[l.x];
        vec3f n = normalize(d);
        float w = length(d);
        s.norm[l.x] = s.norm[l.x] + n * w;
        s.norm[l.y] = s.norm[l.y] + n * w;
    }
    for (auto t : s.triangles) {
        vec3f c = cross(s.pos[t.y] - s.pos[t.x], s.pos[t.z] - s.pos[t.x]);
        vec3f n = normalize(c);
        float w = length(c) / 2;
        s.norm[t.x] = s.norm[t.x] + n * w;
        s.norm[t.y] = s.norm[t.y] + n * w;
        s.norm[t.z] = s.norm[t.z] + n * w;
    }
    for (auto& n : s.norm) n = normalize(n);
}

// yocto dot/normalize start the sum from 0 (yocto_math.h:889-957)
float ydot(vec3f a, vec3f b) {
    float c = 0;
    c += a.x * b.x;
    c += a.y * b.y;
    c += a.z * b.z;
    return c;
}
vec3f ynormalize(vec3f a) {
    float l = std::sqrt(ydot(a, a));
    if (l == 0) return a;
    return a * (1 / l);
}

// add_elements default camera (yocto_scn.cpp:1644-1664); parity unpinned by in/*
// (every shipped scene has a `c` line), pinned by a synthetic test against the reference.
camera default_camera(const scene& scn) {
    auto bounds_of = [](const shape& s) {
        bbox3f b = invalid_bbox3f;
        for (auto p : s.pos) b = expand_bbox(b, p);
        return b;
    };
    bbox3f bbox = invalid_bbox3f;
    if (!scn.instances.empty()) {
        for (auto& ist : scn.instances) {
            bbox3f sb = bounds_of(scn.shapes[ist.shp]);
            bbox3f wb = invalid_bbox3f;
            const vec3f c[8] = {{sb.min.x, sb.min.y, sb.min.z}, {sb.min.x, sb.min.y, sb.max.z},
                                {sb.min.x, sb.max.y, sb.min.z}, {sb.min.x, sb.max.y, sb.max.z},
                                {sb.max.x, sb.min.y, sb.min.z}, {sb.max.x, sb.min.y, sb.max.z},
                                {sb.max.x, sb.max.y, sb.min.z}, {sb.max.x, sb.max.y, sb.max.z}};
            for (int k = 0; k < 8; k++) wb = expand_bbox(wb, transform_point(ist.frame, c[k]));
            bbox = expand_bbox(bbox, wb);
        }
    } else {
        for (auto& s : scn.shapes) bbox = expand_bbox(bbox, bounds_of(s));
    }
    vec3f center = (bbox.min + bbox.max) / 2;
    vec3f size = bbox.max - bbox.min;
    float msize = smax(size.x, smax(size.y, size.z));
    camera cam;
    cam.name = "default_camera";
    vec3f from = vec3f{1, 0.4f, 1} * msize + center;
    vec3f to = center;
    vec3f up = {0, 1, 0};
    vec3f w = ynormalize(from - to);
    vec3f u = ynormalize(cross(up, w));
    vec3f v = ynormalize(cross(w, u));
    cam.frame = {u, v, w, from};
    cam.aspect = 16.0f / 9.0f;
    cam.fovy = 2 * atanf(0.5f);
    cam.aperture = 0;
    vec3f d = to - from;
    cam.focus = std::sqrt(ydot(d, d));
    return cam;
}

}  // namespace

void load_obj_scene(const std::string& filename, scene& scn) {
    obj_file obj;
    parse_obj(filename, obj);
    scn = scene();
    auto dir = dir_of(filename);

    // textures, in MTL first-appearance order (yocto_scn.cpp:168-221, scene.cpp:149-160)
    std::map<std::string, int> tmap;
    for (auto& p : obj.textures) {
        texture t;
        t.path = p;
        if (p.size() >= 4 && p.substr(p.size() - 4) == ".hdr")
            throw unsupported_error("hdr textures are not supported: " + p);
        bool ok = false;
        auto data = read_file(dir + p, ok);
        std::vector<unsigned char> rgba;
        std::string err;
        if (ok && png_decode_rgba8(data, t.width, t.height, rgba, err)) {
            t.pixels.resize((size_t)t.width * t.height);
            memcpy(t.pixels.data(), rgba.data(), rgba.size());
        } else {
            t.width = t.height = 0;  // stbi_load failure leaves an empty image
        }
        tmap[p] = (int)scn.textures.size();
        scn.textures.push_back(std::move(t));
    }

    // materials (yocto_scn.cpp:244-297)
    std::unordered_map<std::string, int> mmap = {{"", -1}};
    for (auto& om : obj.materials) {
        material m;
        m.name = om.name;
        m.ke = om.ke;
        m.kd = om.kd;
        m.ks = om.ks;
        m.kr = om.kr;
        m.rs = std::pow(2 / (om.ns + 2), 1 / 4.0f);
        m.kd_txt = om.kd_txt.empty() ? -1 : tmap.at(om.kd_txt);
        m.ks_txt = om.ks_txt.empty() ? -1 : tmap.at(om.ks_txt);
        mmap[m.name] = (int)scn.materials.size();
        scn.materials.push_back(m);
    }

    // shapes (yocto_scn.cpp:300-449)
    std::unordered_map<std::string, std::vector<int>> omap = {{"", {}}};
    std::vector<int> shape_mat;
    for (auto& o : obj.objects) {
        omap[o.name] = {};
        for (auto& g : o.groups) {
            if (g.verts.empty() || g.elems.empty()) continue;
            shape s;
            s.name = o.name + g.groupname;
            auto mit = mmap.find(g.matname);
            int mat = mit == mmap.end() ? -1 : mit->second;
            if (mit == mmap.end()) mmap[g.matname] = -1;
            std::unordered_map<obj_vert, int, obj_vert_hash> vmap;
            std::vector<int> ids;
            std::vector<obj_vert> uniq;
            for (auto& v : g.verts) {
                auto it = vmap.find(v);
                if (it == vmap.end()) {
                    int id = (int)vmap.size();
                    vmap.emplace(v, id);
                    uniq.push_back(v);
                    ids.push_back(id);
                } else {
                    ids.push_back(it->second);
                }
            }
            for (auto& e : g.elems) {
                if (e.kind == elem_kind::point) {
                    for (uint32_t i = e.start; i < e.start + e.size; i++) s.points.push_back(ids[i]);
                } else if (e.kind == elem_kind::line) {
                    for (int i = (int)e.start; i < (int)e.start + (int)e.size - 1; i++)
                        s.lines.push_back({ids[i], ids[i + 1]});
                } else if (e.kind == elem_kind::face) {
                    if (e.size == 3) {
                        s.triangles.push_back({ids[e.start], ids[e.start + 1], ids[e.start + 2]});
                    } else {
                        for (uint32_t i = e.start + 2; i < e.start + e.size; i++)
                            s.triangles.push_back({ids[e.start], ids[i - 1], ids[i]});
                    }
                }
            }
            const obj_vert& v0 = g.verts[0];
            size_t nv = uniq.size();
            if (v0.pos >= 0) s.pos.assign(nv, vec3f{0, 0, 0});
            if (v0.texcoord >= 0) s.texcoord.assign(nv, vec2f{0, 0});
            if (v0.norm >= 0) s.norm.assign(nv, vec3f{0, 0, 0});
            if (v0.radius >= 0) s.radius.assign(nv, 0.0f);
            for (size_t i = 0; i < nv; i++) {
                const obj_vert& v = uniq[i];
                if (v0.pos >= 0 && v.pos >= 0) s.pos[i] = obj.pos.at(v.pos);
                if (v0.texcoord >= 0 && v.texcoord >= 0) s.texcoord[i] = obj.texcoord.at(v.texcoord);
                if (v0.norm >= 0 && v.norm >= 0) s.norm[i] = obj.norm.at(v.norm);
                if (v0.radius >= 0 && v.radius >= 0) s.radius[i] = obj.radius.at(v.radius);
            }
            omap[o.name].push_back((int)scn.shapes.size());
            shape_mat.push_back(mat);
            scn.shapes.push_back(std::move(s));
        }
    }

    // cameras (yocto_scn.cpp:452-463, scene.cpp:134-143)
    for (auto& oc : obj.cameras) {
        camera c;
        c.name = oc.name;
        c.frame = oc.frame;
        c.fovy = oc.yfov;
        c.aspect = oc.aspect;
        c.focus = oc.focus;
        c.aperture = oc.aperture;
        scn.cameras.push_back(c);
    }

    // instances (yocto_scn.cpp:469-477); material is the shape's (scene.cpp:202)
    for (auto& oi : obj.instances) {
        for (int si : omap[oi.objname]) {
            instance ist;
            ist.name = oi.name;
            ist.frame = oi.frame;
            ist.shp = si;
            ist.mat = shape_mat[si];
            scn.instances.push_back(ist);
        }
    }

    // add_elements with scene.cpp:124-129 options
    for (auto& s : scn.shapes) {
        if ((s.points.empty() && s.lines.empty()) || !s.radius.empty()) continue;
        s.radius.assign(s.pos.size(), 0.001f);
    }
    if (scn.instances.empty()) {
        for (int si = 0; si < (int)scn.shapes.size(); si++) {
            instance ist;
            ist.name = scn.shapes[si].name;
            ist.shp = si;
            ist.mat = shape_mat[si];
            scn.instances.push_back(ist);
        }
    }
    if (scn.cameras.empty()) scn.cameras.push_back(default_camera(scn));

    // smooth normals where missing, in instance order (scene.cpp:217-222)
    for (auto& ist : scn.instances) {
        auto& s = scn.shapes[ist.shp];
        if (s.norm.empty()) compute_smooth_normals(s);
    }
}

}  // namespace yrt
