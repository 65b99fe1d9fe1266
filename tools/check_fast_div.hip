// Exhaustive / sweep check of the division shortcuts in trace_common.h against the IEEE
// division the reference performs (hipcc's correctly rounded 1.0f / x and a / b):
//   rcp_nr(x)     for every one of the 2^32 f32 inputs x;
//   sqrt_nr(x)    for every one of the 2^32 f32 inputs x (against sqrtf);
//   div_nr(a, b)  for every positive a (2^31; the sign is symmetric) and a list of b.
// Each mismatch class is counted (NaN results compare equal to NaN). Build and run:
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -I yocto_raytracing_amd/csrc \
//         tools/check_fast_div.hip -o /tmp/check_fast_div && /tmp/check_fast_div
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "fast_div.h"

__device__ unsigned long long g_bad[4];
__device__ unsigned g_first[4];

__device__ __forceinline__ bool same(float a, float b) {
    return (a != a && b != b) || __float_as_uint(a) == __float_as_uint(b);
}

// every 32-bit pattern: fast reciprocal where rcp_nr_ok says it applies
__global__ void k_rcp(unsigned long long base) {
    const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float((unsigned)i);
    const float ref = 1.0f / x;
    if (yrt::rcp_nr_ok(x)) {
        if (!same(yrt::rcp_nr(x), ref)) {
            if (atomicAdd(&g_bad[0], 1ull) == 0) g_first[0] = (unsigned)i;
        }
    } else {
        atomicAdd(&g_bad[1], 1ull);  // inputs left to the exact division
    }
}

// every 32-bit pattern: sqrt_nr where sqrt_nr_ok admits it, against sqrtf
__global__ void k_sqrt(unsigned long long base) {
    const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float((unsigned)i);
    if (yrt::sqrt_nr_ok(x)) {
        if (!same(yrt::sqrt_nr(x), __builtin_sqrtf(x))) {
            if (atomicAdd(&g_bad[2], 1ull) == 0) g_first[2] = (unsigned)i;
        }
    } else {
        atomicAdd(&g_bad[3], 1ull);
    }
}

// every positive a against one b
__global__ void k_div(unsigned base, float b) {
    const unsigned i = base + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 0x80000000u) return;
    const float a = __uint_as_float(i);
    const float ref = a / b;
    if (yrt::div_nr_ok(a, b)) {
        const float y = yrt::rcp_nr(b);
        if (!same(yrt::div_nr(a, b, y), ref)) {
            if (atomicAdd(&g_bad[2], 1ull) == 0) g_first[2] = i;
        }
    } else {
        atomicAdd(&g_bad[3], 1ull);
    }
}

static void check(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
        exit(1);
    }
}

int main() {
    unsigned long long z[4] = {};
    check(hipMemcpyToSymbol(HIP_SYMBOL(g_bad), z, sizeof z), "reset");
    const unsigned long long n = 1ull << 32;
    const unsigned blk = 256, grid = 1u << 22;  // 2^30 inputs per launch
    for (unsigned long long base = 0; base < n; base += (unsigned long long)blk * grid)
        hipLaunchKernelGGL(k_rcp, dim3(grid), dim3(blk), 0, 0, base);
    check(hipDeviceSynchronize(), "k_rcp");
    unsigned long long bad[4];
    unsigned first[4];
    check(hipMemcpyFromSymbol(bad, HIP_SYMBOL(g_bad), sizeof bad), "read");
    check(hipMemcpyFromSymbol(first, HIP_SYMBOL(g_first), sizeof first), "read");
    printf("rcp_nr: 2^32 inputs, %llu mismatches (first 0x%08x), %llu left to the division\n", bad[0], first[0],
           bad[1]);
    int fails = bad[0] != 0;

    check(hipMemcpyToSymbol(HIP_SYMBOL(g_bad), z, sizeof z), "reset");
    for (unsigned long long base = 0; base < n; base += (unsigned long long)blk * grid)
        hipLaunchKernelGGL(k_sqrt, dim3(grid), dim3(blk), 0, 0, base);
    check(hipDeviceSynchronize(), "k_sqrt");
    check(hipMemcpyFromSymbol(bad, HIP_SYMBOL(g_bad), sizeof bad), "read");
    check(hipMemcpyFromSymbol(first, HIP_SYMBOL(g_first), sizeof first), "read");
    printf("sqrt_nr: 2^32 inputs, %llu mismatches (first 0x%08x), %llu left to sqrtf\n", bad[2], first[2], bad[3]);
    fails |= bad[2] != 0;

    // b: around 1 (normalize divides by lengths of unit-ish vectors), then a spread
    float bs[64];
    int nb = 0;
    float one = 1.0f;
    for (int k = -12; k <= 12; k++) {
        unsigned u;
        memcpy(&u, &one, 4);
        u += k;
        float b;
        memcpy(&b, &u, 4);
        bs[nb++] = b;
    }
    const float spread[] = {0.5f, 0.7071068f, 0.9999f, 1.0001f, 1.4142135f, 1.9999999f, 2.0f,   3.0f,
                            7.0f, 0.1f,       1e-3f,   1e3f,    123.456f,   1e-20f,     1e20f, 3.3e-38f,
                            1.7e38f, 0.33333334f, 5.9604645e-08f, 16777215.0f};
    for (float b : spread) bs[nb++] = b;
    srand(12345);
    while (nb < 64) bs[nb++] = ldexpf((float)rand() / RAND_MAX + 0.5f, rand() % 200 - 100);
    for (int q = 0; q < nb; q++) {
        check(hipMemcpyToSymbol(HIP_SYMBOL(g_bad), z, sizeof z), "reset");
        for (unsigned base = 0; base < 0x80000000u; base += blk * (1u << 21))
            hipLaunchKernelGGL(k_div, dim3(1u << 21), dim3(blk), 0, 0, base, bs[q]);
        check(hipDeviceSynchronize(), "k_div");
        check(hipMemcpyFromSymbol(bad, HIP_SYMBOL(g_bad), sizeof bad), "read");
        check(hipMemcpyFromSymbol(first, HIP_SYMBOL(g_first), sizeof first), "read");
        printf("div_nr: b = %.9g, 2^31 a, %llu mismatches (first a = 0x%08x), %llu left to the division\n", bs[q],
               bad[2], first[2], bad[3]);
        fails |= bad[2] != 0;
    }
    printf(fails ? "FAIL\n" : "PASS\n");
    return fails;
}
