// VALU issue-rate microbenchmark for the instruction mix of the step kernel:
// independent chains of v_bitop3 / v_alignbit / DPP wave shifts, several
// waves per SIMD, timed with hipEvents.  Prints wave-instructions per cycle
// per SIMD at the clock measured with s_memtime / s_memrealtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kIters = 4096;

// Round 4: the hg loop mix with the cross-lane move taken
// off the VALU and / or a 4-word interleave.
//   MODE 5: MODE 4 with the 2 DPP wave shifts replaced by ds_bpermute_b32 (LDS
//           pipe, no LDS allocation), requested one row ahead: the words a
//           chain needs next iteration are asked for at the end of this one.
//   MODE 6: quad layout -- 4 words per lane, cell 4b + j in word j bit b: per
//           quad 2 DPP + 2 v_alignbit + 8 + 4 x 7 v_bitop3 = 40 ops (MODE 4:
//           44 for two pairs).
//   MODE 7: MODE 6 with ds_bpermute one row ahead.
//   MODE 8: the row-pair-shared circuit (rule_b3s23_pair): two rows of a pair
//           arrive (per row 2 DPP + 2 v_alignbit + 4 v_bitop3), their P is formed
//           per word (v_xor + v_and + 2 v_bitop3) and each of the 2 x 2 words
//           runs the 4-v_bitop3 tail: 40 VALU per 4 word-generations.
// Round 5: the fused hash's price on MODE 8's mix.
//   MODE 9:  today's hash -- per output row and pair two v_mad_u64_u32 (the
//            even and odd word by their row keys, summed) and one ds_add_u64
//            (no return) into the lane's LDS sum of that generation.
//   MODE 10: the same two v_mad_u64_u32 per row, summed in registers (no
//            LDS): what register sums would save (+2 VGPRs per stage in the
//            kernel).
//   MODE 11: a "full-rate" hash for comparison: one v_dot4_u32_u8 per word
//            (bytes by 8-bit keys into a 32-bit sum) -- a weaker hash, priced
//            only to bound what any multiply-free scheme could gain.
__device__ __forceinline__ uint32_t rule7(uint32_t a0, uint32_t a1, uint32_t c0, uint32_t c1, uint32_t b0, uint32_t b1,
                                          uint32_t alive) {
    const uint32_t e1 = __builtin_amdgcn_bitop3_b32(a0, c0, b0, 0x69);
    const uint32_t e2 = __builtin_amdgcn_bitop3_b32(a0, c0, b0, 0x7e);
    const uint32_t f1 = __builtin_amdgcn_bitop3_b32(a1, c1, b1, 0x69);
    const uint32_t f2 = __builtin_amdgcn_bitop3_b32(a1, c1, b1, 0x7e);
    const uint32_t t1 = __builtin_amdgcn_bitop3_b32(e1, e2, f2, 0x56);
    const uint32_t t2 = __builtin_amdgcn_bitop3_b32(e1, alive, t1, 0x45);
    return __builtin_amdgcn_bitop3_b32(e2, f1, t2, 0x28);
}

template <int MODE, int CH>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed, unsigned long long* clk) {
    uint32_t a[CH], b[CH], c[CH], d[CH], pl[CH], pr[CH];
    unsigned long long hs[CH];
    uint32_t hs32[CH];
    __shared__ unsigned long long hsum_all[4 * 2 * 64];
    const int lane = threadIdx.x & 63;
    unsigned long long* hsum = hsum_all + (threadIdx.x >> 6) * 128;
    hsum[lane] = hsum[64 + lane] = 0;
    const int addr_l = ((lane + 63) & 63) * 4, addr_r = ((lane + 1) & 63) * 4;  // ds_bpermute byte addresses
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        a[i] = seed * (threadIdx.x + i); b[i] = a[i] ^ 0x9e3779b9u; c[i] = a[i] + 17u; d[i] = b[i] * 5u;
        pl[i] = a[i] >> 3; pr[i] = b[i] << 3;
        hs[i] = 0; hs32[i] = 0;
    }
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            if constexpr (MODE == 0) {  // 4 bitop3
                a[i] = __builtin_amdgcn_bitop3_b32(a[i], b[i], c[i], 0x96);
                b[i] = __builtin_amdgcn_bitop3_b32(a[i], b[i], c[i], 0xe8);
                c[i] = __builtin_amdgcn_bitop3_b32(a[i], b[i], c[i], 0x06);
                a[i] = __builtin_amdgcn_bitop3_b32(a[i], b[i], c[i], 0xe0);
            } else if constexpr (MODE == 1) {  // 4 alignbit
                a[i] = __builtin_amdgcn_alignbit(a[i], b[i], 31);
                b[i] = __builtin_amdgcn_alignbit(c[i], a[i], 1);
                c[i] = __builtin_amdgcn_alignbit(b[i], a[i], 31);
                a[i] = __builtin_amdgcn_alignbit(c[i], b[i], 1);
            } else if constexpr (MODE == 2) {  // 2 DPP wave shifts + 2 bitop3
                a[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a[i], 0x138, 0xf, 0xf, true) ^ b[i];
                b[i] = __builtin_amdgcn_bitop3_b32(a[i], b[i], c[i], 0x96);
                c[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)b[i], 0x130, 0xf, 0xf, true) ^ a[i];
                a[i] = __builtin_amdgcn_bitop3_b32(a[i], b[i], c[i], 0xe8);
            } else if constexpr (MODE == 4) {
                // round-3 loop mix per 32-bit word (multistep_hg_kernel on the pair layout):
                // a pair (e = a, o = b) arrives -- 2 DPP wave shifts, 2 v_alignbit, 4 v_bitop3 --
                // and each of its words goes through the 7-v_bitop3 full-sum rule with the two
                // previous rows' sums (kept in c and in the chain's state): 22 ops per pair
                const uint32_t e = a[i], o = b[i];
                const uint32_t left = (uint32_t)__builtin_amdgcn_mov_dpp((int)o, 0x138, 0xf, 0xf, true);
                const uint32_t right = (uint32_t)__builtin_amdgcn_mov_dpp((int)e, 0x130, 0xf, 0xf, true);
                const uint32_t we = __builtin_amdgcn_alignbit(o, left, 31);
                const uint32_t eo = __builtin_amdgcn_alignbit(right, e, 1);
                const uint32_t h0e = __builtin_amdgcn_bitop3_b32(we, e, o, 0x96);
                const uint32_t h1e = __builtin_amdgcn_bitop3_b32(we, e, o, 0xe8);
                const uint32_t h0o = __builtin_amdgcn_bitop3_b32(e, o, eo, 0x96);
                const uint32_t h1o = __builtin_amdgcn_bitop3_b32(e, o, eo, 0xe8);
                uint32_t out2[2];
                const uint32_t hh0[2] = {h0e, h0o}, hh1[2] = {h1e, h1o};
#pragma unroll
                for (int j = 0; j < 2; ++j) {  // rows A = c (plane 0) / c ^ 1 (plane 1), C = previous, B = new
                    const uint32_t a0 = c[i], a1 = c[i] ^ 0x5a5a5a5au, c0 = hh0[j ^ 1], c1 = hh1[j ^ 1];
                    const uint32_t e1 = __builtin_amdgcn_bitop3_b32(a0, c0, hh0[j], 0x69);
                    const uint32_t e2 = __builtin_amdgcn_bitop3_b32(a0, c0, hh0[j], 0x7e);
                    const uint32_t f1 = __builtin_amdgcn_bitop3_b32(a1, c1, hh1[j], 0x69);
                    const uint32_t f2 = __builtin_amdgcn_bitop3_b32(a1, c1, hh1[j], 0x7e);
                    const uint32_t t1 = __builtin_amdgcn_bitop3_b32(e1, e2, f2, 0x56);
                    const uint32_t t2 = __builtin_amdgcn_bitop3_b32(e1, j ? o : e, t1, 0x45);
                    out2[j] = __builtin_amdgcn_bitop3_b32(e2, f1, t2, 0x28);
                }
                c[i] = h0e;
                a[i] = out2[0];
                b[i] = out2[1];
            } else if constexpr (MODE == 5 || MODE == 6 || MODE == 7) {
                constexpr bool kQuad = MODE != 5, kDs = MODE != 6;
                constexpr int K = kQuad ? 4 : 2;
                uint32_t q[4] = {a[i], b[i], d[i], c[i] ^ a[i]};
                uint32_t left, right;
                if constexpr (kDs) {
                    left = pl[i];
                    right = pr[i];
                } else {
                    left = (uint32_t)__builtin_amdgcn_mov_dpp((int)q[K - 1], 0x138, 0xf, 0xf, true);
                    right = (uint32_t)__builtin_amdgcn_mov_dpp((int)q[0], 0x130, 0xf, 0xf, true);
                }
                uint32_t w[4], e[4], h0[4], h1[4], o[4];
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    w[j] = j == 0 ? __builtin_amdgcn_alignbit(q[K - 1], left, 31) : q[j - 1];
                    e[j] = j == K - 1 ? __builtin_amdgcn_alignbit(right, q[0], 1) : q[j + 1];
                    h0[j] = __builtin_amdgcn_bitop3_b32(w[j], q[j], e[j], 0x96);
                    h1[j] = __builtin_amdgcn_bitop3_b32(w[j], q[j], e[j], 0xe8);
                }
#pragma unroll
                for (int j = 0; j < K; ++j)
                    o[j] = rule7(c[i], c[i] ^ 0x5a5a5a5au, h0[(j + 1) % K], h1[(j + 1) % K], h0[j], h1[j], q[j]);
                c[i] = h0[0];
                a[i] = o[0];
                b[i] = o[1];
                if constexpr (kQuad) d[i] = o[2] ^ o[3];
                if constexpr (kDs) {  // next iteration's cross-lane words, one row ahead
                    pl[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr_l, (int)(kQuad ? (c[i] ^ a[i]) : b[i]));
                    pr[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr_r, (int)a[i]);
                }
            } else if constexpr (MODE == 8) {
                uint32_t hh0[2][2], hh1[2][2], rr[2][2];
                uint32_t rows[2][2] = {{a[i], b[i]}, {d[i], c[i] ^ a[i]}};
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const uint32_t e = rows[r][0], o = rows[r][1];
                    const uint32_t left = (uint32_t)__builtin_amdgcn_mov_dpp((int)o, 0x138, 0xf, 0xf, true);
                    const uint32_t right = (uint32_t)__builtin_amdgcn_mov_dpp((int)e, 0x130, 0xf, 0xf, true);
                    const uint32_t we = __builtin_amdgcn_alignbit(o, left, 31);
                    const uint32_t eo = __builtin_amdgcn_alignbit(right, e, 1);
                    hh0[r][0] = __builtin_amdgcn_bitop3_b32(we, e, o, 0x96);
                    hh1[r][0] = __builtin_amdgcn_bitop3_b32(we, e, o, 0xe8);
                    hh0[r][1] = __builtin_amdgcn_bitop3_b32(e, o, eo, 0x96);
                    hh1[r][1] = __builtin_amdgcn_bitop3_b32(e, o, eo, 0xe8);
                    rr[r][0] = e; rr[r][1] = o;
                }
                uint32_t out4[2][2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint32_t k = hh0[0][j] & hh0[1][j];
                    const uint32_t p0 = hh0[0][j] ^ hh0[1][j];
                    const uint32_t p1 = __builtin_amdgcn_bitop3_b32(hh1[0][j], hh1[1][j], k, 0x96);
                    const uint32_t p2 = __builtin_amdgcn_bitop3_b32(hh1[0][j], hh1[1][j], k, 0xe8);
#pragma unroll
                    for (int r = 0; r < 2; ++r) {  // x: the chain's previous rows (c: above, pl: below)
                        const uint32_t x0 = r ? pl[i] : c[i], x1 = r ? pr[i] : (c[i] ^ 0x5a5a5a5au), al = rr[r][j];
                        const uint32_t g1 = __builtin_amdgcn_bitop3_b32(p0, x0, al, 0x43);
                        const uint32_t g2 = __builtin_amdgcn_bitop3_b32(p1, p2, g1, 0x18);
                        const uint32_t g3 = __builtin_amdgcn_bitop3_b32(p2, x1, g2, 0x26);
                        out4[r][j] = __builtin_amdgcn_bitop3_b32(g3, al, g1, 0xd0);
                    }
                }
                c[i] = hh0[1][0]; pl[i] = hh0[0][1]; pr[i] = hh1[1][1];
                a[i] = out4[0][0]; b[i] = out4[0][1]; d[i] = out4[1][0] ^ out4[1][1];
            } else if constexpr (MODE == 9 || MODE == 10 || MODE == 11) {
                uint32_t hh0[2][2], hh1[2][2], rr[2][2];
                uint32_t rows[2][2] = {{a[i], b[i]}, {d[i], c[i] ^ a[i]}};
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const uint32_t e = rows[r][0], o = rows[r][1];
                    const uint32_t left = (uint32_t)__builtin_amdgcn_mov_dpp((int)o, 0x138, 0xf, 0xf, true);
                    const uint32_t right = (uint32_t)__builtin_amdgcn_mov_dpp((int)e, 0x130, 0xf, 0xf, true);
                    const uint32_t we = __builtin_amdgcn_alignbit(o, left, 31);
                    const uint32_t eo = __builtin_amdgcn_alignbit(right, e, 1);
                    hh0[r][0] = __builtin_amdgcn_bitop3_b32(we, e, o, 0x96);
                    hh1[r][0] = __builtin_amdgcn_bitop3_b32(we, e, o, 0xe8);
                    hh0[r][1] = __builtin_amdgcn_bitop3_b32(e, o, eo, 0x96);
                    hh1[r][1] = __builtin_amdgcn_bitop3_b32(e, o, eo, 0xe8);
                    rr[r][0] = e; rr[r][1] = o;
                }
                uint32_t out4[2][2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint32_t k = hh0[0][j] & hh0[1][j];
                    const uint32_t p0 = hh0[0][j] ^ hh0[1][j];
                    const uint32_t p1 = __builtin_amdgcn_bitop3_b32(hh1[0][j], hh1[1][j], k, 0x96);
                    const uint32_t p2 = __builtin_amdgcn_bitop3_b32(hh1[0][j], hh1[1][j], k, 0xe8);
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const uint32_t x0 = r ? pl[i] : c[i], x1 = r ? pr[i] : (c[i] ^ 0x5a5a5a5au), al = rr[r][j];
                        const uint32_t g1 = __builtin_amdgcn_bitop3_b32(p0, x0, al, 0x43);
                        const uint32_t g2 = __builtin_amdgcn_bitop3_b32(p1, p2, g1, 0x18);
                        const uint32_t g3 = __builtin_amdgcn_bitop3_b32(p2, x1, g2, 0x26);
                        out4[r][j] = __builtin_amdgcn_bitop3_b32(g3, al, g1, 0xd0);
                    }
                }
                // the hash of the two output rows (row keys: wave-uniform, per chain)
                const uint32_t ka = 0x9E3779B1u * (uint32_t)(it + i) | 1u, kb = ka + 0x6A09E666u;
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    if constexpr (MODE == 11) {
                        hs32[i] = __builtin_amdgcn_udot4(out4[r][0], ka, hs32[i], false);
                        hs32[i] = __builtin_amdgcn_udot4(out4[r][1], kb, hs32[i], false);
                    } else {
                        unsigned long long t = (unsigned long long)out4[r][0] * ka;
                        t += (unsigned long long)out4[r][1] * kb;
                        if constexpr (MODE == 9) __hip_atomic_fetch_add(&hsum[r * 64 + lane], t, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_WORKGROUP);
                        else hs[i] += t;
                    }
                }
                c[i] = hh0[1][0]; pl[i] = hh0[0][1]; pr[i] = hh1[1][1];
                a[i] = out4[0][0]; b[i] = out4[0][1]; d[i] = out4[1][0] ^ out4[1][1];
            } else {  // step-kernel mix: 1 DPP, 2 alignbit, 9 bitop3, 1 xor  (13)
                const uint32_t l = (uint32_t)__builtin_amdgcn_mov_dpp((int)c[i], 0x138, 0xf, 0xf, true);
                const uint32_t w = __builtin_amdgcn_alignbit(a[i], l, 31);
                const uint32_t e = __builtin_amdgcn_alignbit(b[i], a[i], 1);
                const uint32_t h0 = __builtin_amdgcn_bitop3_b32(w, a[i], e, 0x96);
                const uint32_t h1 = __builtin_amdgcn_bitop3_b32(w, a[i], e, 0xe8);
                const uint32_t g0 = h0 ^ c[i];
                const uint32_t g1 = __builtin_amdgcn_bitop3_b32(h1, h0, c[i], 0xd0);
                const uint32_t n0 = __builtin_amdgcn_bitop3_b32(b[i], h0, g0, 0x96);
                const uint32_t c0 = __builtin_amdgcn_bitop3_b32(b[i], h0, g0, 0xe8);
                const uint32_t pp = __builtin_amdgcn_bitop3_b32(c[i], h1, g1, 0x96);
                const uint32_t qq = __builtin_amdgcn_bitop3_b32(c[i], h1, g1, 0xe8);
                const uint32_t x = __builtin_amdgcn_bitop3_b32(qq, pp, c0, 0x06);
                c[i] = b[i]; b[i] = a[i];
                a[i] = __builtin_amdgcn_bitop3_b32(x, n0, a[i], 0xe0);
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) acc ^= a[i] ^ b[i] ^ c[i] ^ d[i] ^ pl[i] ^ pr[i] ^ (uint32_t)hs[i] ^ (uint32_t)(hs[i] >> 32) ^ hs32[i];
    __syncthreads();
    acc ^= (uint32_t)hsum[lane] ^ (uint32_t)(hsum[64 + lane] >> 32);
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int MODE, int CH>
int run(const char* name, int ops_per_chain_iter, int waves_per_simd, uint32_t* out, unsigned long long* clk, int cus,
        int words_per_iter = 0) {
    const int blocks = cus * waves_per_simd;  // 256-thread WG = 4 waves = 1 per SIMD
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k<MODE, CH>), dim3(blocks), dim3(256), 0, 0, out, 1u, clk);
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL((k<MODE, CH>), dim3(blocks), dim3(256), 0, 0, out, 1u + r, clk);
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    unsigned long long h[2]; CHK(hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost));
    const double ghz = (double)h[0] / (double)h[1] * 0.1;  // memrealtime = 100 MHz
    const double wave_instr = (double)blocks * 4 * kIters * CH * ops_per_chain_iter;
    const double per_simd_per_cycle = wave_instr / (cus * 4.0) / (best * 1e-3 * ghz * 1e9);
    printf("%-28s waves/SIMD=%d chains=%2d  %.3f ms  clk=%.2f GHz  wave-VALU/cycle/SIMD=%.3f  lane-ops/s=%.1fT", name,
           waves_per_simd, CH, best, ghz, per_simd_per_cycle, wave_instr * 64 / (best * 1e-3) / 1e12);
    if (words_per_iter) {
        const double wg = (double)blocks * 4 * kIters * CH * words_per_iter;  // wave word-generations
        printf("  word-gen/cycle/SIMD=%.4f", wg / (cus * 4.0) / (best * 1e-3 * ghz * 1e9));
    }
    printf("\n");
    return 0;
}

int main() {
    int cus = 0; hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0)); cus = prop.multiProcessorCount;
    uint32_t* out; unsigned long long* clk;
    CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4)); CHK(hipMalloc(&clk, 16));
    const bool r3 = getenv("VALU_RATE_R3") != nullptr;  // only the round-3 loop mix, at 1..8 waves/SIMD
    if (getenv("VALU_RATE_PAIR")) {
        // the per-row circuit (MODE 4, 22 VALU per 2 word-generations) beside
        // the row-pair-shared one (MODE 8, 40 VALU per 4 word-generations)
        for (int w : {2, 3, 4}) {
            run<4, 2>("per-row circuit (22 VALU/pair)", 22, w, out, clk, cus, 2);
            run<4, 4>("per-row circuit (22 VALU/pair)", 22, w, out, clk, cus, 2);
            run<8, 1>("pair-row circuit (40 VALU/2 pairs)", 40, w, out, clk, cus, 4);
            run<8, 2>("pair-row circuit (40 VALU/2 pairs)", 40, w, out, clk, cus, 4);
        }
        return 0;
    }
    if (getenv("VALU_RATE_HASH")) {
        // the pair-row mix (MODE 8, 40 VALU per 4 word-generations) unhashed,
        // with today's hash (+4 v_mad_u64_u32 + 2 ds_add_u64), with register
        // sums (+4 v_mad_u64_u32), and with a byte-dot hash (+4 v_dot4)
        for (int w : {2, 3, 4}) {
            run<8, 1>("pair-row, no hash", 40, w, out, clk, cus, 4);
            run<8, 2>("pair-row, no hash", 40, w, out, clk, cus, 4);
            run<9, 1>("pair-row, mad_u64 + ds_add", 44, w, out, clk, cus, 4);
            run<9, 2>("pair-row, mad_u64 + ds_add", 44, w, out, clk, cus, 4);
            run<10, 1>("pair-row, mad_u64 regs", 44, w, out, clk, cus, 4);
            run<10, 2>("pair-row, mad_u64 regs", 44, w, out, clk, cus, 4);
            run<11, 1>("pair-row, dot4 (weaker)", 44, w, out, clk, cus, 4);
            run<11, 2>("pair-row, dot4 (weaker)", 44, w, out, clk, cus, 4);
        }
        return 0;
    }
    if (getenv("VALU_RATE_R4")) {
        // word-generations per cycle per SIMD: a pair iteration advances 2
        // words, a quad iteration 4 (the ops column counts VALU only)
        for (int w : {1, 2, 3, 4, 6}) {
            run<4, 2>("R4 pair DPP (22 VALU/pair)", 22, w, out, clk, cus, 2);
            run<4, 4>("R4 pair DPP (22 VALU/pair)", 22, w, out, clk, cus, 2);
            run<5, 2>("R4 pair bpermute (20 VALU)", 20, w, out, clk, cus, 2);
            run<5, 4>("R4 pair bpermute (20 VALU)", 20, w, out, clk, cus, 2);
            run<6, 2>("R4 quad DPP (40 VALU/quad)", 40, w, out, clk, cus, 4);
            run<6, 4>("R4 quad DPP (40 VALU/quad)", 40, w, out, clk, cus, 4);
            run<7, 2>("R4 quad bpermute (38 VALU)", 38, w, out, clk, cus, 4);
            run<7, 4>("R4 quad bpermute (38 VALU)", 38, w, out, clk, cus, 4);
        }
        return 0;
    }
    for (int w : {1, 2, 3, 4, 5, 6, 8}) {
        if (r3) {
            run<4, 2>("hg loop mix (22 ops/pair)", 22, w, out, clk, cus);
            run<4, 4>("hg loop mix (22 ops/pair)", 22, w, out, clk, cus);
            run<0, 4>("bitop3 x4", 4, w, out, clk, cus);
            continue;
        }
        if (w == 3 || w == 6) continue;
        run<0, 4>("bitop3 x4", 4, w, out, clk, cus);
        run<1, 4>("alignbit x4", 4, w, out, clk, cus);
        run<2, 4>("dpp+xor/bitop3", 4, w, out, clk, cus);
        run<3, 2>("step mix (13 ops)", 13, w, out, clk, cus);
        run<3, 4>("step mix (13 ops)", 13, w, out, clk, cus);
    }
    return 0;
}
