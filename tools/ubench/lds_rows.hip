// LDS gathers of pair-table rows on gfx950 (tools/ubench): each lane reads a
// 96-byte row (24 dwords) at a pseudo-random row of a 441-row table, as the
// pair kernel does per column, with ds_read_b128 x 6, ds_read_b64 x 12 or
// ds_read_b32 x 24, at row strides of 24, 28 and 32 dwords; also every lane
// reading the same row (no conflicts).  3 workgroups of 4 waves per CU;
// reports cycles per wave per row read, per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_rows lds_rows.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int STRIDE, int WIDTH, bool UNIFORM>
__global__ void __launch_bounds__(256) k_rows(uint32_t* out, int iters) {
    extern __shared__ uint32_t tab[];
    for (int i = threadIdx.x; i < 441 * STRIDE; i += 256) tab[i] = i * 2654435761u;
    __syncthreads();
    uint32_t x = (threadIdx.x * 7919u + blockIdx.x * 104729u) | 1u, acc = 0;
    for (int it = 0; it < iters; it++) {
        x = x * 1664525u + 1013904223u;
        uint32_t row = (x >> 8) % 441u;
        if (UNIFORM) row = __builtin_amdgcn_readfirstlane(row);
        const uint32_t* p = tab + row * STRIDE;
        if (WIDTH == 16) {
#pragma unroll
            for (int q = 0; q < 6; q++) { const uint4 v = *(const uint4*)(p + 4 * q); acc ^= v.x + v.y + v.z + v.w; }
        } else if (WIDTH == 8) {
#pragma unroll
            for (int q = 0; q < 12; q++) { const uint2 v = *(const uint2*)(p + 2 * q); acc ^= v.x + v.y; }
        } else {
#pragma unroll
            for (int q = 0; q < 24; q++) acc ^= p[q];
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int STRIDE, int WIDTH, bool UNIFORM>
void run(const char* name) {
    const int blocks = 256 * 3 * 8;
    uint32_t* out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    const size_t lds = 441 * STRIDE * 4;
    (void)hipFuncSetAttribute((const void*)k_rows<STRIDE, WIDTH, UNIFORM>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k_rows<STRIDE, WIDTH, UNIFORM><<<blocks, 256, lds>>>(out, 50);
    (void)hipEventRecord(e0);
    const int iters = 2000;
    k_rows<STRIDE, WIDTH, UNIFORM><<<blocks, 256, lds>>>(out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double rows_per_cu = (double)iters * blocks * 4 / 256;   // wave-level row reads per CU
    printf("%-28s %7.3f ms  %6.2f cycles per wave row read per CU @2.4GHz\n", name, ms, 2.4e6 * ms / rows_per_cu);
    (void)hipFree(out);
}

int main() {
    run<28, 16, false>("stride28 b128 x6 random");
    run<24, 16, false>("stride24 b128 x6 random");
    run<32, 16, false>("stride32 b128 x6 random");
    run<28, 8, false>("stride28 b64 x12 random");
    run<26, 8, false>("stride26 b64 x12 random");
    run<25, 4, false>("stride25 b32 x24 random");
    run<28, 16, true>("stride28 b128 x6 uniform");
    return 0;
}
