// Microbenchmark: sustained VALU issue rate of the instructions the strip
// kernel is made of (v_pk_add_i16 clamp, v_pk_max_i16, v_bfi_b32, and 32-bit
// v_add_u32 / v_max_i32 for comparison) on MI355X.  8 independent chains per
// lane, every CU full of waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef short s2 __attribute__((ext_vector_type(2)));
#define AS_S2(x) __builtin_bit_cast(s2, (uint32_t)(x))
#define AS_U32(x) __builtin_bit_cast(uint32_t, (x))

template <int KIND, int CHAINS>
__global__ void __launch_bounds__(256) k(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a[CHAINS];
#pragma unroll
    for (int i = 0; i < CHAINS; i++) a[i] = seed * (threadIdx.x + i * 7919u);
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
#pragma unroll
            for (int i = 0; i < CHAINS; i++) {
                if (KIND == 0) asm volatile("v_pk_add_i16 %0, %0, %1 clamp" : "+v"(a[i]) : "v"(x));
                if (KIND == 1) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a[i]) : "v"(y));
                if (KIND == 2) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(x), "v"(y));
                if (KIND == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
                if (KIND == 4) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a[i]) : "v"(y));
                if (KIND == 5) asm volatile("v_pk_add_i16 %0, %0, %1 clamp\n\tv_pk_max_i16 %0, %0, %2" : "+v"(a[i]) : "v"(x), "v"(y));
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; i++) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int KIND, int CHAINS>
void run(const char* name, int waves_per_simd) {
    const int blocks = 256 * waves_per_simd;   // 256-thread blocks = 4 waves = 1 per SIMD
    uint32_t* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    const int iters = 4000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k<KIND, CHAINS><<<blocks, 256>>>(out, 10, 1);
    hipEventRecord(e0);
    k<KIND, CHAINS><<<blocks, 256>>>(out, iters, 3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double ops_per_thread = (double)iters * 8 * CHAINS * (KIND == 5 ? 2 : 1);
    const double wave_instr = ops_per_thread * blocks * 4;       // wave-level instructions
    const double per_simd_per_ns = wave_instr / 1024 / (ms * 1e6);
    printf("%-28s chains=%d waves/SIMD=%d  %.3f ms  %.3f wave-instr/SIMD/ns  (%.2f cycles/instr @2.4GHz)\n",
           name, CHAINS, waves_per_simd, ms, per_simd_per_ns, 2.4 / per_simd_per_ns);
    hipFree(out);
}

int main() {
    for (int w : {1, 2, 4, 8}) {
        run<0, 8>("v_pk_add_i16 clamp", w);
        run<1, 8>("v_pk_max_i16", w);
        run<5, 8>("pk add+max", w);
        run<2, 8>("v_bfi_b32", w);
        run<3, 8>("v_add_u32", w);
        run<4, 8>("v_max_i32", w);
    }
    run<0, 1>("v_pk_add_i16 dependent", 1);
    run<0, 1>("v_pk_add_i16 dependent", 4);
    run<0, 2>("v_pk_add_i16 2 chains", 1);
    run<0, 4>("v_pk_add_i16 4 chains", 1);
    return 0;
}
