// Issue cost of the DP's instruction mix on gfx950 (tools/ubench): groups of
// five independent instructions per lane (10 accumulators = 2 groups per
// asm), 8 waves per SIMD; reports cycles per 5-instruction group per SIMD.
//   slow5:   pk_add, max3, pk_add, max3, max3  (all packed / VOP3)
//   cur:     the SW/NW row today: pk_add, max3, add_u32, max3, max3
//   fastadd: the diagonal add as v_add_u32 too: add, max3, add, max3, max3
//   batch4:  the adds of two groups back to back: add x4, max3 x6
//   pairs:   add, add, max3 x3
//   fast5:   5 x v_add_u32
// Build: hipcc --offload-arch=gfx950 -O3 -o mix_rates mix_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define A2(op, d, s) op " " d ", " d ", " s "\n\t"
#define A3(op, d, s, t) op " " d ", " d ", " s ", " t "\n\t"

#define KERNEL(NAME, OPS)                                                                                  \
    __global__ void __launch_bounds__(256) NAME(uint32_t* out, int iters, uint32_t seed) {                 \
        uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11;       \
        uint32_t a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19, a8 = a0 ^ 23, a9 = a0 ^ 29;                     \
        const uint32_t x = seed ^ 0x12345u, y = seed + 77u;                                                \
        for (int it = 0; it < iters; it++) {                                                               \
            _Pragma("unroll") for (int u = 0; u < 8; u++) {                                                \
                asm volatile(OPS                                                                           \
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),      \
                               "+v"(a7), "+v"(a8), "+v"(a9)                                                \
                             : "v"(x), "v"(y));                                                            \
            }                                                                                              \
        }                                                                                                  \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ a8 ^ a9;      \
    }

#define PK(d) A2("v_pk_add_u16", d, "%10")
#define AD(d) A2("v_add_u32", d, "%11")
#define MX(d) A3("v_pk_maximum3_f16", d, "%10", "%11")

KERNEL(k_slow5, PK("%0") MX("%1") PK("%2") MX("%3") MX("%4") PK("%5") MX("%6") PK("%7") MX("%8") MX("%9"))
KERNEL(k_cur, PK("%0") MX("%1") AD("%2") MX("%3") MX("%4") PK("%5") MX("%6") AD("%7") MX("%8") MX("%9"))
KERNEL(k_fastadd, AD("%0") MX("%1") AD("%2") MX("%3") MX("%4") AD("%5") MX("%6") AD("%7") MX("%8") MX("%9"))
KERNEL(k_batch4, AD("%0") AD("%1") AD("%2") AD("%3") MX("%4") MX("%5") MX("%6") MX("%7") MX("%8") MX("%9"))
KERNEL(k_pairs, AD("%0") AD("%1") MX("%2") MX("%3") MX("%4") AD("%5") AD("%6") MX("%7") MX("%8") MX("%9"))
KERNEL(k_fast5, AD("%0") AD("%1") AD("%2") AD("%3") AD("%4") AD("%5") AD("%6") AD("%7") AD("%8") AD("%9"))

template <typename K>
void run(const char* name, K kern) {
    const int blocks = 256 * 8;
    uint32_t* out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<<<blocks, 256>>>(out, 20, 1);
    (void)hipEventRecord(e0);
    kern<<<blocks, 256>>>(out, 1000, 3);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double groups = 1000.0 * 8 * 2 * blocks * 4;   // wave-level 5-instruction groups
    printf("%-10s %.3f ms  %.2f cycles per 5-instruction group per SIMD @2.4GHz\n", name, ms,
           2.4e6 * ms / (groups / 1024));
    (void)hipFree(out);
}

int main() {
    run("slow5", k_slow5);
    run("cur", k_cur);
    run("fastadd", k_fastadd);
    run("batch4", k_batch4);
    run("pairs", k_pairs);
    run("fast5", k_fast5);
    return 0;
}
