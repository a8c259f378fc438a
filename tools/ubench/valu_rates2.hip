#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(256) k_v_add_u32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_add_u32_e64(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_sub_u32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_and_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_and_b32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_and_b32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_and_b32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_and_b32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_and_b32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_and_b32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_and_b32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_and_b32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_or_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_or_b32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_or_b32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_or_b32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_or_b32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_or_b32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_or_b32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_or_b32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_or_b32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_xor_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_max_i32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_max_u32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_max_u32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_max_u32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_max_u32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_max_u32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_max_u32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_max_u32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_max_u32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_max_u32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_min_i32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_min_i32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_min_i32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_min_i32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_min_i32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_min_i32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_min_i32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_min_i32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_min_i32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_max3_i32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_add3_u32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_med3_i32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_lshlrev_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_lshl_add_u32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_perm_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_bfi_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_cndmask_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_mov_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_mov_b32 %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_mov_b32 %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_mov_b32 %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_mov_b32 %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_mov_b32 %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_mov_b32 %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_mov_b32 %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_mov_b32 %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_add_u16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_add_u16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_add_u16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_add_u16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_add_u16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_add_u16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_add_u16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_add_u16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_add_u16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_max_i16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_max_i16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_max_i16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_max_i16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_max_i16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_max_i16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_max_i16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_max_i16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_max_i16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_max_u16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_max_u16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_max_u16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_max_u16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_max_u16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_max_u16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_max_u16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_max_u16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_max_u16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_add_i16_clamp(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_add_i16 %0, %0, %1 clamp" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_add_i16 %0, %0, %1 clamp" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_add_i16 %0, %0, %1 clamp" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_add_i16 %0, %0, %1 clamp" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_add_i16 %0, %0, %1 clamp" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_add_i16 %0, %0, %1 clamp" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_add_i16 %0, %0, %1 clamp" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_add_i16 %0, %0, %1 clamp" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_max3_i16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_add_i16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_add_i16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_add_i16_clamp(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_add_u16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_sub_u16_clamp(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_max_i16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_max_u16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_min_i16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_min_i16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_min_i16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_min_i16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_min_i16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_min_i16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_min_i16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_min_i16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_min_i16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_mad_i16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_mad_i16 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_mad_i16 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_mad_i16 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_mad_i16 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_mad_i16 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_mad_i16 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_mad_i16 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_mad_i16 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_add_f32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_max_f32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_max3_f32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_fma_f32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_add_f16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_max_f16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_max_f16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_max_f16 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_max_f16 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_max_f16 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_max_f16 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_max_f16 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_max_f16 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_max_f16 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_max_f16 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_pk_maximum3_f16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_maximum3_f32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_dot2_i32_i16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_sad_u16(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <typename K> void run(const char* name, K kern) {
    const int blocks = 256 * 8;
    uint32_t* out; (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    kern<<<blocks, 256>>>(out, 20, 1);
    (void)hipEventRecord(e0);
    kern<<<blocks, 256>>>(out, 2000, 3);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double wi = 2000.0 * 64 * blocks * 4;
    printf("%-22s %.3f ms  %.2f cycles/wave-instr/SIMD @2.4GHz\n", name, ms, 2.4 / (wi / 1024 / (ms * 1e6)));
    (void)hipFree(out);
}
int main() {
    run("v_add_u32", k_v_add_u32);
    run("v_add_u32_e64", k_v_add_u32_e64);
    run("v_sub_u32", k_v_sub_u32);
    run("v_and_b32", k_v_and_b32);
    run("v_or_b32", k_v_or_b32);
    run("v_xor_b32", k_v_xor_b32);
    run("v_max_i32", k_v_max_i32);
    run("v_max_u32", k_v_max_u32);
    run("v_min_i32", k_v_min_i32);
    run("v_max3_i32", k_v_max3_i32);
    run("v_add3_u32", k_v_add3_u32);
    run("v_med3_i32", k_v_med3_i32);
    run("v_lshlrev_b32", k_v_lshlrev_b32);
    run("v_lshl_add_u32", k_v_lshl_add_u32);
    run("v_perm_b32", k_v_perm_b32);
    run("v_bfi_b32", k_v_bfi_b32);
    run("v_cndmask_b32", k_v_cndmask_b32);
    run("v_mov_b32", k_v_mov_b32);
    run("v_add_u16", k_v_add_u16);
    run("v_max_i16", k_v_max_i16);
    run("v_max_u16", k_v_max_u16);
    run("v_add_i16_clamp", k_v_add_i16_clamp);
    run("v_max3_i16", k_v_max3_i16);
    run("v_pk_add_i16", k_v_pk_add_i16);
    run("v_pk_add_i16_clamp", k_v_pk_add_i16_clamp);
    run("v_pk_add_u16", k_v_pk_add_u16);
    run("v_pk_sub_u16_clamp", k_v_pk_sub_u16_clamp);
    run("v_pk_max_i16", k_v_pk_max_i16);
    run("v_pk_max_u16", k_v_pk_max_u16);
    run("v_pk_min_i16", k_v_pk_min_i16);
    run("v_pk_mad_i16", k_v_pk_mad_i16);
    run("v_add_f32", k_v_add_f32);
    run("v_max_f32", k_v_max_f32);
    run("v_max3_f32", k_v_max3_f32);
    run("v_fma_f32", k_v_fma_f32);
    run("v_pk_add_f16", k_v_pk_add_f16);
    run("v_pk_max_f16", k_v_pk_max_f16);
    run("v_max_f16", k_v_max_f16);
    run("v_pk_maximum3_f16", k_v_pk_maximum3_f16);
    run("v_maximum3_f32", k_v_maximum3_f32);
    run("v_dot2_i32_i16", k_v_dot2_i32_i16);
    run("v_sad_u16", k_v_sad_u16);
    return 0;
}
