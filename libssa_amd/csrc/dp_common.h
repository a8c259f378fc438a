// dp_common.h -- device helpers shared by the DP kernels (kernels.hip,
// pair_sw.hip, pair_nw.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "kernels.h"

namespace ssa {

typedef short s2 __attribute__((ext_vector_type(2)));

#define AS_U32(x) __builtin_bit_cast(uint32_t, (x))
#define AS_S2(x) __builtin_bit_cast(s2, (uint32_t)(x))

__device__ __forceinline__ s2 adds(s2 a, s2 b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ s2 vmax(s2 a, s2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ uint32_t perm(uint32_t hi_src, uint32_t lo_src, uint32_t sel) {
    return __builtin_amdgcn_perm(hi_src, lo_src, sel);
}
__device__ __forceinline__ short sat16(int v) { return (short)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }
__device__ __forceinline__ uint32_t pack16(short lo, short hi) {
    return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16);
}

// byte selectors for v_perm_b32(a, b, sel): bytes 0-3 of b, 4-7 of a
constexpr uint32_t SEL_LO_BHI_HI_ALO = 0x05040302u;  // lo = b.hi,  hi = a.lo
constexpr uint32_t SEL_LO_BLO_HI_ALO = 0x05040100u;  // lo = b.lo,  hi = a.lo
constexpr uint32_t SEL_LO_BHI_HI_AHI = 0x07060302u;  // lo = b.hi,  hi = a.hi

template <int NP>
__device__ __forceinline__ void load_row(uint32_t (&dst)[NP], const uint32_t* row) {
#pragma unroll
    for (int i = 0; i < NP / 4; i++) {
        const uint4 v = *(const uint4*)(row + 4 * i);
        dst[4 * i + 0] = v.x;
        dst[4 * i + 1] = v.y;
        dst[4 * i + 2] = v.z;
        dst[4 * i + 3] = v.w;
    }
    if constexpr (NP % 4 == 2) {
        const uint2 v = *(const uint2*)(row + NP - 2);
        dst[NP - 2] = v.x;
        dst[NP - 1] = v.y;
    }
}

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t fmax3(uint32_t a, uint32_t b, uint32_t c) {
    const h2 m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(__builtin_bit_cast(h2, a),
                                                                            __builtin_bit_cast(h2, b)),
                                               __builtin_bit_cast(h2, c));
    return __builtin_bit_cast(uint32_t, m);
}
__device__ __forceinline__ uint32_t fmax2(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_maximum(__builtin_bit_cast(h2, a),
                                                                      __builtin_bit_cast(h2, b)));
}
__device__ __forceinline__ uint32_t psubsat16(uint32_t a, uint32_t b) {   // v_pk_sub_u16 clamp
    typedef unsigned short u2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(u2, a), __builtin_bit_cast(u2, b)));
}
__device__ __forceinline__ uint32_t padd16(uint32_t a, uint32_t b) {   // v_pk_add_u16 (wrapping)
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u2, a) + __builtin_bit_cast(u2, b));
}

// where a wave runs, for the timeline: XCC << 16 | HW_ID[15:0] (wave slot,
// SIMD, pipe, CU, shader array, SE)
__device__ inline uint32_t hw_place() {
    uint32_t id, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    return (xcc & 0xffu) << 16 | (id & 0xffffu);
}

// hipFuncSetAttribute (dynamic LDS above 64 KiB) once per kernel and device:
// the per-device search threads of a multi-GPU search launch concurrently
inline hipError_t lds_attr_once(const void* fn, std::atomic<uint64_t>& done, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

}  // namespace ssa
