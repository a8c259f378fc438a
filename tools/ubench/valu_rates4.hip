#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(256) k_v_mul_lo_u32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_mul_hi_u32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_mad_u32_u24(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_mul_u32_u24(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_bfe_u32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_lshrrev_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_and_or_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void __launch_bounds__(256) k_v_lshl_or_b32(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(a7) : "v"(x), "v"(y));
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
    run("v_mul_lo_u32", k_v_mul_lo_u32);
    run("v_mul_hi_u32", k_v_mul_hi_u32);
    run("v_mad_u32_u24", k_v_mad_u32_u24);
    run("v_mul_u32_u24", k_v_mul_u32_u24);
    run("v_bfe_u32", k_v_bfe_u32);
    run("v_lshrrev_b32", k_v_lshrrev_b32);
    run("v_and_or_b32", k_v_and_or_b32);
    run("v_lshl_or_b32", k_v_lshl_or_b32);
    run("v_pk_maximum3_f16", k_v_pk_maximum3_f16);
    run("v_add_u32", k_v_add_u32);
    return 0;
}
