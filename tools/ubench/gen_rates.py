#!/usr/bin/env python3
"""Generates valu_rates2.hip: one throughput kernel per instruction (8
independent chains per lane, 8 waves/SIMD), to find which VALU opcodes issue
at full rate on gfx950.  Build: hipcc --offload-arch=gfx950 -O3."""
INSTRS = {
    "v_add_u32": "v_add_u32 %0, %0, %1",
    "v_add_u32_e64": "v_add_u32_e64 %0, %0, %1",
    "v_sub_u32": "v_sub_u32 %0, %0, %1",
    "v_and_b32": "v_and_b32 %0, %0, %1",
    "v_or_b32": "v_or_b32 %0, %0, %1",
    "v_xor_b32": "v_xor_b32 %0, %0, %1",
    "v_max_i32": "v_max_i32 %0, %0, %1",
    "v_max_u32": "v_max_u32 %0, %0, %1",
    "v_min_i32": "v_min_i32 %0, %0, %1",
    "v_max3_i32": "v_max3_i32 %0, %0, %1, %2",
    "v_add3_u32": "v_add3_u32 %0, %0, %1, %2",
    "v_med3_i32": "v_med3_i32 %0, %0, %1, %2",
    "v_lshlrev_b32": "v_lshlrev_b32 %0, 1, %0",
    "v_lshl_add_u32": "v_lshl_add_u32 %0, %0, 1, %1",
    "v_perm_b32": "v_perm_b32 %0, %0, %1, %2",
    "v_bfi_b32": "v_bfi_b32 %0, %1, %0, %2",
    "v_cndmask_b32": "v_cndmask_b32 %0, %0, %1, vcc",
    "v_mov_b32": "v_mov_b32 %0, %1",
    "v_add_u16": "v_add_u16 %0, %0, %1",
    "v_max_i16": "v_max_i16 %0, %0, %1",
    "v_max_u16": "v_max_u16 %0, %0, %1",
    "v_add_i16_clamp": "v_add_i16 %0, %0, %1 clamp",
    "v_max3_i16": "v_max3_i16 %0, %0, %1, %2",
    "v_pk_add_i16": "v_pk_add_i16 %0, %0, %1",
    "v_pk_add_i16_clamp": "v_pk_add_i16 %0, %0, %1 clamp",
    "v_pk_add_u16": "v_pk_add_u16 %0, %0, %1",
    "v_pk_sub_u16_clamp": "v_pk_sub_u16 %0, %0, %1 clamp",
    "v_pk_max_i16": "v_pk_max_i16 %0, %0, %1",
    "v_pk_max_u16": "v_pk_max_u16 %0, %0, %1",
    "v_pk_min_i16": "v_pk_min_i16 %0, %0, %1",
    "v_pk_mad_i16": "v_pk_mad_i16 %0, %0, %1, %2",
    "v_add_f32": "v_add_f32 %0, %0, %1",
    "v_max_f32": "v_max_f32 %0, %0, %1",
    "v_max3_f32": "v_max3_f32 %0, %0, %1, %2",
    "v_fma_f32": "v_fma_f32 %0, %0, %1, %2",
    "v_pk_add_f16": "v_pk_add_f16 %0, %0, %1",
    "v_pk_max_f16": "v_pk_max_f16 %0, %0, %1",
    "v_max_f16": "v_max_f16 %0, %0, %1",
    "v_pk_maximum3_f16": "v_pk_maximum3_f16 %0, %0, %1, %2",
    "v_maximum3_f32": "v_maximum3_f32 %0, %0, %1, %2",
    "v_dot2_i32_i16": "v_dot2_i32_i16 %0, %1, %2, %0",
    "v_sad_u16": "v_sad_u16 %0, %1, %2, %0",
    "mix_max3_add": "v_pk_maximum3_f16 %0, %0, %1, %2\\n\\tv_add_u32 %0, %0, %1",
    "mix_max3_2add": "v_pk_maximum3_f16 %0, %0, %1, %2\\n\\tv_add_u32 %0, %0, %1\\n\\tv_add_u32 %0, %0, %2",
    "mix_pkadd_max3": "v_pk_add_u16 %0, %0, %1\\n\\tv_pk_maximum3_f16 %0, %0, %1, %2",
    "v_pk_maximum3_f16x2": "v_pk_maximum3_f16 %0, %0, %1, %2\\n\\tv_pk_maximum3_f16 %0, %0, %2, %1",
    "v_add_u32x2": "v_add_u32 %0, %0, %1\\n\\tv_add_u32 %0, %0, %2",
    "v_mul_lo_u32": "v_mul_lo_u32 %0, %0, %1",
    "v_mul_hi_u32": "v_mul_hi_u32 %0, %0, %1",
    "v_mad_u32_u24": "v_mad_u32_u24 %0, %0, %1, %2",
    "v_mul_u32_u24": "v_mul_u32_u24 %0, %0, %1",
    "v_bfe_u32": "v_bfe_u32 %0, %0, 8, 8",
    "v_lshrrev_b32": "v_lshrrev_b32 %0, 8, %0",
    "v_and_or_b32": "v_and_or_b32 %0, %0, %1, %2",
    "v_lshl_or_b32": "v_lshl_or_b32 %0, %0, 4, %1",
}
import os
import sys
only = sys.argv[1:] if len(sys.argv) > 1 else list(INSTRS)
src = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdint>']
for name in only:
    asm = INSTRS[name].replace('%0', '%0').replace('"', '')
    src.append(f'''
__global__ void __launch_bounds__(256) k_{name}(uint32_t* out, int iters, uint32_t seed) {{
    uint32_t a0 = seed * (threadIdx.x + 1), a1 = a0 ^ 3, a2 = a0 ^ 5, a3 = a0 ^ 7, a4 = a0 ^ 11, a5 = a0 ^ 13, a6 = a0 ^ 17, a7 = a0 ^ 19;
    const uint32_t x = seed ^ 0x12345u, y = seed + 77u;
    for (int it = 0; it < iters; it++) {{
#pragma unroll
        for (int u = 0; u < 8; u++) {{
            asm volatile("{asm}" : "+v"(a0) : "v"(x), "v"(y));
            asm volatile("{asm}" : "+v"(a1) : "v"(x), "v"(y));
            asm volatile("{asm}" : "+v"(a2) : "v"(x), "v"(y));
            asm volatile("{asm}" : "+v"(a3) : "v"(x), "v"(y));
            asm volatile("{asm}" : "+v"(a4) : "v"(x), "v"(y));
            asm volatile("{asm}" : "+v"(a5) : "v"(x), "v"(y));
            asm volatile("{asm}" : "+v"(a6) : "v"(x), "v"(y));
            asm volatile("{asm}" : "+v"(a7) : "v"(x), "v"(y));
        }}
    }}
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}}''')
src.append('''
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
    printf("%-22s %.3f ms  %.2f cycles/wave-instr/SIMD @2.4GHz\\n", name, ms, 2.4 / (wi / 1024 / (ms * 1e6)));
    (void)hipFree(out);
}
int main() {''')
for name in only:
    src.append(f'    run("{name}", k_{name});')
src.append('    return 0;\n}')
open(os.environ.get('OUT', 'valu_rates2.hip'), 'w').write('\n'.join(src) + '\n')
