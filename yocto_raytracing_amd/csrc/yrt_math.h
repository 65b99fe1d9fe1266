// yrt_math.h -- fp32 vector/frame/ray/bbox math shared by the host BVH builder and
// the gfx950 kernels.
//
// Every function reproduces the reference's operation order exactly
// (src/vmath.h), because the product is held to bit-exact parity with it:
//   * dot is (a.x*b.x + a.y*b.y) + a.z*b.z               vmath.h:112-114
//   * normalize returns its input when the length is 0   vmath.h:118-122
//   * min/max are ?: selects, NOT fminf/fmaxf, so NaN propagation is
//     argument-order dependent as in the reference       vmath.h:215-216
//   * transform_direction(_inverse) renormalises          vmath.h:169-175
// Translation units that include this header are compiled with
// -ffp-contract=off so that no a*b+c is fused (the reference's x86-64 build has
// no FMA), and HIP's default correctly rounded fp32 division and sqrt.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define YRT_HD __host__ __device__ __forceinline__
#else
#define YRT_HD inline
#endif

namespace yrt {

struct vec2f {
    float x, y;
};
struct vec3f {
    float x, y, z;
};
struct vec4f {
    float x, y, z, w;
};
struct vec2i {
    int x, y;
};
struct vec3i {
    int x, y, z;
};
struct vec4b {
    unsigned char x, y, z, w;
};
struct frame3f {
    vec3f x, y, z, o;
};
struct bbox3f {
    vec3f min, max;
};

constexpr float flt_max = 3.402823466e+38f;
constexpr float ray_eps = 1e-4f;  // vmath.h:264

YRT_HD vec2f operator+(vec2f a, vec2f b) { return {a.x + b.x, a.y + b.y}; }
YRT_HD vec2f operator*(vec2f a, float b) { return {a.x * b, a.y * b}; }
YRT_HD vec3f operator+(vec3f a, vec3f b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
YRT_HD vec3f operator-(vec3f a, vec3f b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
YRT_HD vec3f operator*(vec3f a, vec3f b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
YRT_HD vec3f operator*(vec3f a, float b) { return {a.x * b, a.y * b, a.z * b}; }
YRT_HD vec3f operator/(vec3f a, float b) { return {a.x / b, a.y / b, a.z / b}; }
YRT_HD bool operator==(vec3f a, vec3f b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

YRT_HD float dot(vec3f a, vec3f b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
YRT_HD vec3f cross(vec3f a, vec3f b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
YRT_HD float length(vec3f a) { return __builtin_sqrtf(dot(a, a)); }
YRT_HD vec3f normalize(vec3f a) {
    float l = length(a);
    if (l == 0) return a;
    return a * (1 / l);
}

// ?: selects (vmath.h:215-217) -- deliberately not fminf/fmaxf
YRT_HD float smin(float x, float y) { return (x < y) ? x : y; }
YRT_HD float smax(float x, float y) { return (x > y) ? x : y; }
YRT_HD float sclamp(float x, float a, float b) { return smin(smax(x, a), b); }

// frames (vmath.h:152-175)
YRT_HD vec3f transform_point(const frame3f& a, vec3f b) {
    return a.x * b.x + a.y * b.y + a.z * b.z + a.o;
}
YRT_HD vec3f transform_vector(const frame3f& a, vec3f b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
YRT_HD vec3f transform_direction(const frame3f& a, vec3f b) { return normalize(transform_vector(a, b)); }
YRT_HD vec3f transform_point_inverse(const frame3f& a, vec3f b) {
    vec3f bo = b - a.o;
    return {dot(a.x, bo), dot(a.y, bo), dot(a.z, bo)};
}
YRT_HD vec3f transform_direction_inverse(const frame3f& a, vec3f b) {
    return normalize(vec3f{dot(a.x, b), dot(a.y, b), dot(a.z, b)});
}

// bboxes (vmath.h:284-326)
constexpr bbox3f invalid_bbox3f = {{flt_max, flt_max, flt_max}, {-flt_max, -flt_max, -flt_max}};
YRT_HD bbox3f expand_bbox(const bbox3f& a, vec3f b) {
    return {{smin(a.min.x, b.x), smin(a.min.y, b.y), smin(a.min.z, b.z)},
            {smax(a.max.x, b.x), smax(a.max.y, b.y), smax(a.max.z, b.z)}};
}
YRT_HD bbox3f expand_bbox(const bbox3f& a, const bbox3f& b) {
    return {{smin(a.min.x, b.min.x), smin(a.min.y, b.min.y), smin(a.min.z, b.min.z)},
            {smax(a.max.x, b.max.x), smax(a.max.y, b.max.y), smax(a.max.z, b.max.z)}};
}
YRT_HD bbox3f bbox_to_world(const frame3f& a, const bbox3f& b) {
    const vec3f c[8] = {
        {b.min.x, b.min.y, b.min.z}, {b.min.x, b.min.y, b.max.z}, {b.min.x, b.max.y, b.min.z},
        {b.min.x, b.max.y, b.max.z}, {b.max.x, b.min.y, b.min.z}, {b.max.x, b.min.y, b.max.z},
        {b.max.x, b.max.y, b.min.z}, {b.max.x, b.max.y, b.max.z},
    };
    bbox3f r = invalid_bbox3f;
    for (int i = 0; i < 8; i++) r = expand_bbox(r, transform_point(a, c[i]));
    return r;
}

}  // namespace yrt
