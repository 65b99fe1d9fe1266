// yrt_scene.h -- host scene model (C++), the product-side counterpart of the
// reference's scene.h. Index-based instead of pointer-based, but field for field
// the data raytrace() reads:
//   bvh_node/bvh_tree   scene.h:9-22  (same 32-byte node, same meaning)
//   shape               scene.h:26-50 (pos/norm/texcoord/radius, points/lines/triangles)
//   texture             scene.h:54-58 (8-bit RGBA, `ldr`)
//   material            scene.h:62-86 (ke/kd/ks/kr, rs, kd_txt/ks_txt)
//   instance            scene.h:99-111 (frame, material, shape)
//   camera              scene.h:115-123
//   scene               scene.h:136-155
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "yrt_math.h"

namespace yrt {

// Typed failures; the C-ABI (capi.cpp guarded()) maps each type to its status code:
//   unsupported_error -> YRT_ERR_UNSUPPORTED  (input the kernels do not handle)
//   device_error      -> YRT_ERR_HIP          (a HIP runtime call failed)
//   device_oom        -> YRT_ERR_OOM          (hipMalloc / hipErrorOutOfMemory)
//   std::invalid_argument -> YRT_ERR_INVALID_ARG, any other runtime_error -> YRT_ERR_IO
struct unsupported_error : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct device_error : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct device_oom : device_error {
    using device_error::device_error;
};
// the message yrt_last_error() reports on this thread (capi.cpp)
void set_last_error(const std::string& msg);

struct bvh_node {
    bbox3f bbox;     // bounding box
    uint32_t start;  // first child node (inner) or first leaf_prims slot (leaf)
    uint16_t count;  // children (always 2) or primitives
    uint8_t isleaf;
    uint8_t axis;
};
static_assert(sizeof(bvh_node) == 32, "bvh_node must stay 32 bytes (scene.h:9-15)");

struct bvh_tree {
    std::vector<bvh_node> nodes;
    std::vector<int> leaf_prims;
};

struct texture {
    std::string path;
    int width = 0, height = 0;
    std::vector<vec4b> pixels;  // row-major, pixels[j*width+i] (image.h:28)
};

struct material {
    std::string name;
    vec3f ke = {0, 0, 0};
    vec3f kd = {0, 0, 0};
    vec3f ks = {0, 0, 0};
    vec3f kr = {0, 0, 0};
    float rs = 0;
    int kd_txt = -1;
    int ks_txt = -1;
};

struct shape {
    std::string name;
    std::vector<vec3f> pos;
    std::vector<vec3f> norm;
    std::vector<vec2f> texcoord;
    std::vector<float> radius;
    std::vector<int> points;
    std::vector<vec2i> lines;
    std::vector<vec3i> triangles;
    bvh_tree bvh;
};

struct instance {
    std::string name;
    frame3f frame = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
    int mat = -1;
    int shp = -1;
};

struct camera {
    std::string name;
    frame3f frame = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
    float fovy = 1;
    float aspect = 16.0f / 9.0f;
    float aperture = 0;
    float focus = 1;
};

struct scene {
    std::vector<camera> cameras;
    std::vector<texture> textures;
    std::vector<material> materials;
    std::vector<shape> shapes;
    std::vector<instance> instances;
    bvh_tree bvh;  // instance level
    bool has_bvh = false;
};

// ---- loaders / IO (scene_io.cpp, obj_loader.cpp, png.cpp) ----
// All throw std::runtime_error with a message on failure; the C-ABI converts.

// Yocto-OBJ dialect loader reproducing load_scene (src/scene.cpp:113-225) with
// yscn::load_scene / add_elements semantics (see obj_loader.cpp for citations).
void load_obj_scene(const std::string& filename, scene& scn);
// .yrtscene interchange format: the shading-relevant arrays only.
void load_yrtscene(const std::string& filename, scene& scn);
void save_yrtscene(const std::string& filename, const scene& scn);
// load by extension: .obj -> OBJ loader, otherwise .yrtscene
void load_scene_any(const std::string& filename, scene& scn);
// BVH dump (.yrtbvh), byte-compatible with the reference's bvh_node arrays.
void save_yrtbvh(const std::string& filename, const scene& scn);

// ---- BVH (bvh_build.cpp): restates build_bvh (src/scene.cpp:509-658) ----
void build_bvh(scene& scn, bool equal_num);
// the same nodes, byte for byte, with the tree construction on GPU `device`
// (bvh_gpu.hip); kernel_ms (optional): device time of the level passes
void build_bvh_gpu(scene& scn, bool equal_num, int device, float* kernel_ms);
int bvh_max_depth(const bvh_tree& bvh);

// ---- PNG (png.cpp) ----
// decode to 8-bit RGBA (stbi_load(..., 4) semantics for 8/16-bit, non-interlaced)
bool png_decode_rgba8(const std::vector<unsigned char>& file, int& w, int& h,
                      std::vector<unsigned char>& rgba, std::string& err);
bool png_encode_rgba8(const unsigned char* rgba, int w, int h, std::vector<unsigned char>& out);

// ---- image helpers (image.cpp) ----
// tonemap (image.cpp:55-77 with exposure 0, no filmic, srgb): RGBA f32 -> RGBA8
void tonemap_rgba8(const float* rgba, int w, int h, unsigned char* out);
// thr[k] (k = 1..255): the smallest float whose tonemapped channel is >= k with this
// host's powf (thr[0] = 0); the device tonemap's table (scene_io.cpp)
void tonemap_thresholds(float thr[256]);
int tonemap_neg_inf_level();  // the level of -inf (pow(-inf, 1/2.2) = +inf)
// save_hdr_or_ldr (image.cpp:81-88): .hdr -> Radiance RGBE, otherwise PNG of tonemap
void save_hdr_or_ldr(const std::string& filename, const float* rgba, int w, int h);
// PNG of an already tonemapped RGBA8 image (the device-tonemap path of yrt_save_image_mem)
void save_ldr_png(const std::string& filename, const unsigned char* rgba8, int w, int h);
// the .hdr writer in two halves: RGBE bytes of a frame (rows as four component planes when
// the width is run-length encoded, else interleaved; rgbe.h), then the reference's file
// (stbi_write_hdr's header and scanlines). The device path encodes on the GPU.
void rgbe_encode(const float* rgba, int w, int h, unsigned char* out);
void save_hdr_rgbe(const std::string& filename, const unsigned char* rgbe, int w, int h);

}  // namespace yrt
