// rgbe.h -- the float -> Radiance RGBE conversion of the reference's .hdr writer
// (save_hdr_or_ldr, src/image.cpp:39-42,81-84 -> stbi_write_hdr,
// src/ext/stb_image_write.h:493-510), shared by the host writer (scene_io.cpp) and the
// device encoder (render.hip), so both give the reference's bytes:
//
//  * maxcomp = max(r, max(g, b)) with stbiw__max, i.e. `a > b ? a : b` (a NaN operand
//    loses to the left operand only when it is on the right: the x86 build's maxss);
//  * maxcomp < 1e-32f (false for NaN) -> four zero bytes;
//  * otherwise normalize = frexp(maxcomp) * 256 / maxcomp, each colour byte the
//    truncation of c * normalize, the exponent byte exponent + 128 -- with the values
//    the reference's x86-64 build produces where C leaves them open:
//      - (unsigned char)(float) is cvttss2si to a 32-bit int, then its low byte
//        (a negative -3.5 -> -3 -> 0xfd; NaN or |x| >= 2^31 -> 0x80000000 -> 0x00);
//      - glibc's frexpf stores exponent 0 for +-inf and NaN (its value is returned as is,
//        so normalize is NaN there and the colour bytes are 0, the exponent byte 128).
#pragma once

#include <stdint.h>

#ifdef __HIPCC__
#define YRT_HD __host__ __device__ __forceinline__
#else
#define YRT_HD inline
#endif

namespace yrt {

// (unsigned char)(float) as compiled for x86-64 (cvttss2si r32 + low byte)
YRT_HD unsigned char rgbe_trunc_u8(float v) {
    const int32_t i = (v >= -2147483648.0f && v < 2147483648.0f) ? (int32_t)v : INT32_MIN;
    return (unsigned char)((uint32_t)i & 0xffu);
}

YRT_HD float rgbe_frexp(float x, int* e) {
    // +-inf / NaN: glibc stores 0 and returns x; every finite x: the exact mantissa in
    // [0.5, 1) and exponent (0 for 0, never reached here: maxcomp >= 1e-32)
    if (!(x - x == 0.0f)) {
        *e = 0;
        return x;
    }
    return __builtin_frexpf(x, e);
}

// stbiw__linear_to_rgbe on one pixel's r, g, b
YRT_HD void linear_to_rgbe(float r, float g, float b, unsigned char out[4]) {
    const float m12 = g > b ? g : b;
    const float maxcomp = r > m12 ? r : m12;
    if (maxcomp < 1e-32f) {
        out[0] = out[1] = out[2] = out[3] = 0;
        return;
    }
    int e = 0;
    const float normalize = rgbe_frexp(maxcomp, &e) * 256.0f / maxcomp;
    out[0] = rgbe_trunc_u8(r * normalize);
    out[1] = rgbe_trunc_u8(g * normalize);
    out[2] = rgbe_trunc_u8(b * normalize);
    out[3] = (unsigned char)(e + 128);
}

// widths whose scanlines the writer run-length encodes (stb: 8 <= w < 32768; other
// widths are written as flat RGBE quadruples without a scanline header)
YRT_HD bool rgbe_rle_width(int w) { return w >= 8 && w < 32768; }

}  // namespace yrt
