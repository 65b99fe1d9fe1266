// fast_div.h -- the reference's IEEE divisions (x86-64 divss: correctly rounded) in fewer
// instructions where the operands are in range, for the instance entry of the walks.
//
// hipcc's a / b is a ten-instruction sequence (v_div_scale x2, v_rcp, four fma,
// v_div_fmas, v_div_fixup) that also covers denormals, overflow and the special values.
// In the normal range the same answer takes a reciprocal and Newton steps on fma:
//   rcp_nr(x)      = y1 = y0 + y0 (1 - x y0),  y0 = v_rcp_f32(x)        (3 instructions)
//   div_nr(a,b,y)  = q1 = q0 + y (a - b q0),   q0 = a y, y = rcp_nr(b) (3 instructions)
//   sqrt_nr(x)     = v_sqrt_f32 and its one-ulp correction, without the range scaling
// Both are checked bit for bit against hipcc's division by tools/check_fast_div.hip:
// rcp_nr on all 2^32 inputs that rcp_nr_ok admits, div_nr on all 2^31 positive a for a
// sweep of b (the sign is symmetric). Outside the admitted ranges the callers take the
// exact division.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace yrt {

// |x| in [2^-126, 2^126): x and 1/x normal
__device__ __forceinline__ bool rcp_nr_ok(float x) {
    const uint32_t ax = __float_as_uint(x) & 0x7fffffffu;
    return ax - 0x00800000u < 0x7e800000u - 0x00800000u;
}

__device__ __forceinline__ float rcp_nr(float x) {
    const float y0 = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}

// a zero, or |a| and |b| in [2^-60, 2^60]: a/b, a*y and the residual stay normal
__device__ __forceinline__ bool div_nr_ok(float a, float b) {
    const uint32_t aa = __float_as_uint(a) & 0x7fffffffu, ab = __float_as_uint(b) & 0x7fffffffu;
    constexpr uint32_t lo = 0x21800000u, hi = 0x5d800000u;  // 2^-60, 2^60
    return (aa == 0u || aa - lo <= hi - lo) && ab - lo <= hi - lo;
}

__device__ __forceinline__ float div_nr(float a, float b, float y) {
    const float q0 = a * y;
    const float r = __builtin_fmaf(-b, q0, a);
    return __builtin_fmaf(r, y, q0);
}

// x in [2^-96, +inf): the correctly rounded sqrt needs no scaling (no denormal residual)
__device__ __forceinline__ bool sqrt_nr_ok(float x) { return x >= 0x1p-96f && x < __builtin_inff(); }

// hipcc's correctly rounded sqrtf without its range scaling: v_sqrt_f32, then the
// candidate one ulp below or above wins when the fma residual says so (the same
// correction the compiler emits, checked on every admitted input by check_fast_div)
__device__ __forceinline__ float sqrt_nr(float x) {
    const float y = __builtin_amdgcn_sqrtf(x);
    const float ym = __uint_as_float(__float_as_uint(y) - 1u), yp = __uint_as_float(__float_as_uint(y) + 1u);
    const float rm = __builtin_fmaf(-ym, y, x), rp = __builtin_fmaf(-yp, y, x);
    float r = rm <= 0.0f ? ym : y;
    r = rp > 0.0f ? yp : r;
    return r;
}

}  // namespace yrt
