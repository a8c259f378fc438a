// VGPR bank conflicts on gfx950 (tools/ubench): does a 3-source VALU
// instruction cost more when two of its sources sit in the same VGPR bank
// (register number mod 4)?  16 independent v_pk_maximum3_f16 per asm block on
// fixed physical registers, 8 waves per SIMD; cycles per instruction per SIMD.
//   banks3:  sources in banks (1, 2, 3) of the destination's bank 0
//   same2:   two sources in one bank
//   same3:   all three sources in one bank
//   add_same: v_add_u32 with both sources in one bank; add_diff: different banks
// Build: hipcc --offload-arch=gfx950 -O3 -o bank_rates bank_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define MX(d, a, b, c) "v_pk_maximum3_f16 v" #d ", v" #a ", v" #b ", v" #c "\n\t"
#define AD(d, a, b) "v_add_u32 v" #d ", v" #a ", v" #b "\n\t"
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", \
             "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", \
             "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79"

// destinations v40, v44, ... (bank 0); sources chosen per variant
#define BLOCK_BANKS3 MX(40, 61, 62, 63) MX(44, 65, 66, 67) MX(48, 69, 70, 71) MX(52, 73, 74, 75) \
                     MX(56, 61, 66, 71) MX(60, 65, 70, 75) MX(64, 69, 74, 63) MX(68, 73, 62, 67) \
                     MX(41, 62, 63, 64) MX(45, 66, 67, 68) MX(49, 70, 71, 72) MX(53, 74, 75, 76) \
                     MX(57, 62, 67, 72) MX(61, 66, 71, 76) MX(65, 70, 75, 64) MX(69, 74, 63, 68)
#define BLOCK_SAME2  MX(40, 61, 65, 63) MX(44, 65, 69, 67) MX(48, 69, 73, 71) MX(52, 73, 61, 75) \
                     MX(56, 61, 69, 71) MX(60, 65, 73, 75) MX(64, 69, 77, 63) MX(68, 73, 61, 67) \
                     MX(41, 62, 66, 64) MX(45, 66, 70, 68) MX(49, 70, 74, 72) MX(53, 74, 62, 76) \
                     MX(57, 62, 70, 72) MX(61, 66, 74, 76) MX(65, 70, 78, 64) MX(69, 74, 62, 68)
#define BLOCK_SAME3  MX(40, 61, 65, 69) MX(44, 65, 69, 73) MX(48, 69, 73, 77) MX(52, 73, 77, 61) \
                     MX(56, 61, 69, 77) MX(60, 65, 73, 61) MX(64, 69, 77, 65) MX(68, 73, 61, 69) \
                     MX(41, 62, 66, 70) MX(45, 66, 70, 74) MX(49, 70, 74, 78) MX(53, 74, 78, 62) \
                     MX(57, 62, 70, 78) MX(61, 66, 74, 62) MX(65, 70, 78, 66) MX(69, 74, 62, 70)
#define BLOCK_ADDSAME AD(40, 61, 65) AD(44, 65, 69) AD(48, 69, 73) AD(52, 73, 77) AD(56, 61, 69) AD(60, 65, 73) \
                      AD(64, 69, 77) AD(68, 73, 61) AD(41, 62, 66) AD(45, 66, 70) AD(49, 70, 74) AD(53, 74, 78) \
                      AD(57, 62, 70) AD(61, 66, 74) AD(65, 70, 78) AD(69, 74, 62)
#define BLOCK_ADDDIFF AD(40, 61, 66) AD(44, 65, 70) AD(48, 69, 74) AD(52, 73, 78) AD(56, 61, 70) AD(60, 65, 74) \
                      AD(64, 69, 78) AD(68, 73, 62) AD(41, 62, 67) AD(45, 66, 71) AD(49, 70, 75) AD(53, 74, 79) \
                      AD(57, 62, 71) AD(61, 66, 75) AD(65, 70, 79) AD(69, 74, 63)

#define KERNEL(NAME, BLOCK)                                                                     \
    __global__ void __launch_bounds__(256) NAME(uint32_t* out, int iters) {                    \
        for (int it = 0; it < iters; it++) {                                                    \
            _Pragma("unroll") for (int u = 0; u < 8; u++) { asm volatile(BLOCK ::: CLOB); }     \
        }                                                                                       \
        uint32_t r;                                                                             \
        asm volatile("v_mov_b32 %0, v40" : "=v"(r)::"v40");                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                         \
    }

KERNEL(k_banks3, BLOCK_BANKS3)
KERNEL(k_same2, BLOCK_SAME2)
KERNEL(k_same3, BLOCK_SAME3)
KERNEL(k_addsame, BLOCK_ADDSAME)
KERNEL(k_adddiff, BLOCK_ADDDIFF)

template <typename K>
void run(const char* name, K kern) {
    const int blocks = 256 * 8;
    uint32_t* out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<<<blocks, 256>>>(out, 20);
    (void)hipEventRecord(e0);
    kern<<<blocks, 256>>>(out, 1000);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double instrs = 1000.0 * 8 * 16 * blocks * 4;   // wave-level instructions
    printf("%-9s %.3f ms  %.2f cycles per wave-instruction per SIMD @2.4GHz\n", name, ms, 2.4e6 * ms / (instrs / 1024));
    (void)hipFree(out);
}

int main() {
    run("banks3", k_banks3);
    run("same2", k_same2);
    run("same3", k_same3);
    run("addsame", k_addsame);
    run("adddiff", k_adddiff);
    return 0;
}
