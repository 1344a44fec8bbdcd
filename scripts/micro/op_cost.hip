// Issue cost of single VALU instruction kinds (8 waves/SIMD, 8 independent
// chains per wave): cycles per wave64 instruction on one SIMD.  Instruction
// kinds are forced with inline asm so the compiler cannot fold them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
constexpr int kIters = 2048;

#define OP3(ins) asm volatile(ins " %0, %1, %2, %3" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]), "v"(c[i]))
#define OP2(ins) asm volatile(ins " %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]))

template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed, unsigned long long* clk) {
    constexpr int CH = 8;
    uint32_t a[CH], b[CH], c[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) { a[i] = seed * (threadIdx.x + i); b[i] = a[i] ^ 0x9e3779b9u; c[i] = a[i] + 17u; }
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            if constexpr (MODE == 0) OP3("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96 ;");
            if constexpr (MODE == 1) OP3("v_alignbit_b32");
            if constexpr (MODE == 2) OP2("v_xor_b32");
            if constexpr (MODE == 3) OP2("v_lshlrev_b32");
            if constexpr (MODE == 4) OP3("v_lshl_or_b32");
            if constexpr (MODE == 5) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(a[i]) : "v"(b[i]));
            if constexpr (MODE == 6) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(a[i]) : "v"(b[i]));
            if constexpr (MODE == 7) OP3("v_bfi_b32");
            if constexpr (MODE == 8) OP3("v_perm_b32");
            if constexpr (MODE == 9) OP3("v_add3_u32");
            if constexpr (MODE == 10) OP3("v_lshl_add_u32");
            if constexpr (MODE == 11) asm volatile("v_lshrrev_b64 %0, 1, %1" : "=v"(*(uint64_t*)&a[i & ~1]) : "v"(*(uint64_t*)&b[i & ~1]));
            if constexpr (MODE == 12) OP3("v_xad_u32");
            if constexpr (MODE == 13) asm volatile("v_xor_b32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(a[i]) : "v"(b[i]), "v"(c[i]));
            if constexpr (MODE == 14) OP3("v_and_or_b32");
            if constexpr (MODE == 15) OP3("v_or3_b32");
            if constexpr (MODE == 16) asm volatile("v_mov_b32_dpp %0, %1 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(a[i]) : "v"(b[i]));
            if constexpr (MODE == 20) OP2("v_add_u32");
            if constexpr (MODE == 21) asm volatile("v_addc_co_u32 %0, vcc, %1, %2, vcc" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]) : "vcc");
            if constexpr (MODE == 22) asm volatile("v_cmp_gt_i32 vcc, 0, %1\n v_cndmask_b32 %0, %0, %2, vcc" : "+v"(a[i]) : "v"(b[i]), "v"(c[i]) : "vcc");
            if constexpr (MODE == 23) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]) : "vcc");
            if constexpr (MODE == 24) OP2("v_and_b32");
            if constexpr (MODE == 25) OP2("v_or_b32");
            if constexpr (MODE == 26) asm volatile("v_not_b32 %0, %1" : "=v"(a[i]) : "v"(a[i]));
            if constexpr (MODE == 27) OP2("v_sub_u32");
            if constexpr (MODE == 28) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(b[i]));
            if constexpr (MODE == 29) OP2("v_lshrrev_b32");
            if constexpr (MODE == 30) OP3("v_bfe_u32");
            if constexpr (MODE == 31) OP2("v_mul_hi_u32");
            if constexpr (MODE == 32) OP2("v_mul_u32_u24");
            if constexpr (MODE == 33) asm volatile("v_cmp_gt_i32 vcc, 0, %1\n v_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(a[i]) : "v"(b[i]) : "vcc");
            if constexpr (MODE == 34) asm volatile("v_cmp_gt_i32 vcc, 0, %0" : : "v"(a[i]) : "vcc");
            if constexpr (MODE == 35) asm volatile("v_add_co_u32 %0, vcc, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]) : "vcc");
            if constexpr (MODE == 36) asm volatile("v_lshlrev_b32_e64 %0, 1, %1" : "=v"(a[i]) : "v"(a[i]));
            if constexpr (MODE == 37) asm volatile("v_lshrrev_b32_e32 %0, 1, %1" : "=v"(a[i]) : "v"(a[i]));
            if constexpr (MODE == 38) asm volatile("v_add_u32_e32 %0, %1, %1" : "=v"(a[i]) : "v"(a[i]));
            if constexpr (MODE == 39) asm volatile("v_pk_add_u16 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]));
            if constexpr (MODE == 40) asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]));
            if constexpr (MODE == 41) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(*(uint64_t*)&a[i & ~1]) : "v"(b[i]), "v"(c[i]) : "s40", "s41");
            if constexpr (MODE == 42) OP2("v_mul_lo_u32");
            if constexpr (MODE == 43) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(*(uint64_t*)&a[i & ~1]) : "v"(*(uint64_t*)&b[i & ~1]));
            if constexpr (MODE == 17) asm volatile("v_pk_mov_b32 %0, %1, %2 op_sel:[0,1]" : "=v"(*(uint64_t*)&a[i & ~1]) : "v"(*(uint64_t*)&b[i & ~1]), "v"(*(uint64_t*)&c[i & ~1]));
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) acc ^= a[i] ^ b[i] ^ c[i];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int MODE>
int run(const char* name, uint32_t* out, unsigned long long* clk, int cus) {
    const int wps = 8, blocks = cus * wps;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k<MODE>), dim3(blocks), dim3(256), 0, 0, out, 1u, clk);
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL((k<MODE>), dim3(blocks), dim3(256), 0, 0, out, 1u + r, clk);
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    unsigned long long h[2]; CHK(hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost));
    const double ghz = (double)h[0] / (double)h[1] * 0.1;
    const double wave_instr = (double)blocks * 4 * kIters * 8;
    const double cyc = (cus * 4.0) * (best * 1e-3 * ghz * 1e9) / wave_instr;
    printf("%-20s %.3f ms clk=%.2f GHz  cycles/wave-instr/SIMD=%.2f\n", name, best, ghz, cyc);
    return 0;
}

int main() {
    hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0)); const int cus = prop.multiProcessorCount;
    uint32_t* out; unsigned long long* clk;
    CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4)); CHK(hipMalloc(&clk, 16));
    run<0>("v_bitop3_b32", out, clk, cus);
    run<20>("v_add_u32", out, clk, cus);
    run<38>("v_add_u32 x+x", out, clk, cus);
    run<21>("v_addc_co_u32", out, clk, cus);
    run<35>("v_add_co_u32", out, clk, cus);
    run<34>("v_cmp_gt_i32 (vcc)", out, clk, cus);
    run<22>("v_cmp + v_cndmask", out, clk, cus);
    run<33>("v_cmp + v_addc", out, clk, cus);
    run<23>("v_cndmask_b32", out, clk, cus);
    run<24>("v_and_b32", out, clk, cus);
    run<25>("v_or_b32", out, clk, cus);
    run<26>("v_not_b32", out, clk, cus);
    run<27>("v_sub_u32", out, clk, cus);
    run<28>("v_mov_b32", out, clk, cus);
    run<29>("v_lshrrev_b32", out, clk, cus);
    run<36>("v_lshlrev_b32 imm", out, clk, cus);
    run<37>("v_lshrrev_b32 imm", out, clk, cus);
    run<30>("v_bfe_u32", out, clk, cus);
    run<31>("v_mul_hi_u32", out, clk, cus);
    run<32>("v_mul_u32_u24", out, clk, cus);
    run<39>("v_pk_add_u16", out, clk, cus);
    run<40>("v_xor_b32_sdwa", out, clk, cus);
    run<0>("v_bitop3_b32", out, clk, cus);
    run<1>("v_alignbit_b32", out, clk, cus);
    run<2>("v_xor_b32", out, clk, cus);
    run<3>("v_lshlrev_b32", out, clk, cus);
    run<4>("v_lshl_or_b32", out, clk, cus);
    run<5>("v_mov_dpp wave_shr", out, clk, cus);
    run<6>("v_mov_dpp row_shr", out, clk, cus);
    run<16>("v_mov_dpp row_shl", out, clk, cus);
    run<13>("v_xor_dpp wave_shr", out, clk, cus);
    run<7>("v_bfi_b32", out, clk, cus);
    run<8>("v_perm_b32", out, clk, cus);
    run<9>("v_add3_u32", out, clk, cus);
    run<10>("v_lshl_add_u32", out, clk, cus);
    run<11>("v_lshrrev_b64", out, clk, cus);
    run<12>("v_xad_u32", out, clk, cus);
    run<14>("v_and_or_b32", out, clk, cus);
    run<15>("v_or3_b32", out, clk, cus);
    run<17>("v_pk_mov_b32", out, clk, cus);
    run<41>("v_mad_u64_u32", out, clk, cus);
    run<42>("v_mul_lo_u32", out, clk, cus);
    run<43>("v_lshl_add_u64", out, clk, cus);
    return 0;
}
