// gol_stencil.h -- gfx950 (CDNA4) device code of the Life-like generation step.
//
// Replaces the reference's per-cell actor computation:
//   NextStateCellGathererActor.scala:32-36  ask <=8 neighbours GetStateFromEpoch
//   NextStateCellGathererActor.scala:39-46  gather, count, apply rule, commit e+1
//   package.scala:17-28                     the clipped Moore neighbourhood
// with one streaming stencil over a bit-packed board (DESIGN.md "Kernels").
//
// Work decomposition: each wave64 owns one column strip of one band of `band`
// output rows and streams down (or up: odd bands run bottom-up, so both
// neighbours of a band seam read it at the same time and the second read hits
// the Infinity Cache) keeping a ring of rows in registers.  Every input word
// is read from HBM once per pass and every output word written once.
//
// Neighbour count: vertical full adder (a + c + b) per column -> two bit
// planes, DPP wave_shr:1 / wave_shl:1 bring the neighbouring lane's column
// sums, v_alignbit funnel-shifts them to the x-1 / x+1 columns, and a
// bit-sliced adder gives the 3x3 box sum T9 (4 bit planes).  B3/S23 is
// "T9 == 3 | (alive & T9 == 4)"; the generic (birth, survive) path subtracts
// the centre and evaluates the masks with a v_bfi mux tree.
//
// Two kernels:
//   step_kernel      one generation per pass.  A strip is 64 lanes x VEC
//                    words; the bits beyond the strip's edges come from one
//                    extra dword load per row (lane 0: the word left of the
//                    strip, other lanes: the word right of it) that DPP's
//                    `old` operand hands to exactly the lanes without a
//                    source lane.
//   multistep_kernel G = 2..4 generations per pass (temporal blocking: HBM
//                    traffic per generation / G).  Lanes 0 and 63 are halo
//                    lanes holding the neighbouring strips' words; garbage
//                    enters their outermost bit and moves one bit per
//                    generation, far from the 32*VEC-bit lane edge, so the
//                    62 inner lanes are exact.  The intermediate generations
//                    live only in registers (one 3-row ring per stage) and
//                    are hashed there; G-row halos come from above/below.
#pragma once
#include <type_traits>
#include <utility>

#include "gol_kernels.h"

namespace gol {
namespace dev {

constexpr int kPF = 2;               // step_kernel: rows prefetched ahead
constexpr int kRing = kPF + 3;       // step_kernel: register ring of stream rows
constexpr int kMRing = 6;            // multistep kernels: input ring (multiple of 3)
constexpr int kMPF = 2;              // multistep_kernel: rows prefetched ahead
constexpr int kHgPF = 2;             // multistep_hg_kernel: rows prefetched ahead (< kMRing)
static_assert(kHgPF >= 1 && kHgPF < kMRing, "prefetch slots");
static_assert(kMRing % 6 == 0, "the paired-row schedule reads a row's parity from its ring slot (even ring), "
                                  "the stage rings index slots mod 3");
constexpr int kDppWaveShr1 = 0x138;  // lane i <- lane i-1 (lane 0 keeps `old`)
constexpr int kDppWaveShl1 = 0x130;  // lane i <- lane i+1 (lane 63 keeps `old`)
constexpr int kDppWaveRol1 = 0x134;  // lane i <- lane i+1, lane 63 <- lane 0
constexpr int kDppWaveRor1 = 0x13C;  // lane i <- lane i-1, lane 0 <- lane 63

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N-1>): a loop
// whose index is a compile-time constant in every copy, whatever the
// unroller's size heuristics (register-ring slots must never be indexed at
// run time, or the rings move to scratch).
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    return (m & a) | (~m & b);
}

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, kDppWaveShr1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_shl1(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, kDppWaveShl1, 0xf, 0xf, false);
}
// Same shifts with zeros where there is no source lane (no `old` operand).
__device__ __forceinline__ uint32_t dpp_shr1_zero(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kDppWaveShr1, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t dpp_shl1_zero(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kDppWaveShl1, 0xf, 0xf, true);
}
// Wave rotates (whole-row waves: the row wraps inside the wave).
__device__ __forceinline__ uint32_t dpp_ror1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kDppWaveRor1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_rol1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kDppWaveRol1, 0xf, 0xf, false);
}

// Bits [0, limit) of word `w` set (limit in cells).
__device__ __forceinline__ uint32_t col_mask(int64_t limit, int64_t w) {
    const int64_t lo = w * 32;
    if (lo + 32 <= limit) return 0xFFFFFFFFu;
    if (lo >= limit) return 0u;
    return (uint32_t)((1ull << (limit - lo)) - 1ull);
}

typedef uint32_t U32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t U32x4 __attribute__((ext_vector_type(4)));

template <int VEC>
struct Words {
    uint32_t w[VEC];
};

// Unconditional load (callers clamp the column into the row), so no
// exec-masked branch separates a load from its use and the compiler's
// counted vmcnt waits keep the prefetch ring in flight.  Plain (cacheable)
// loads: the halo rows and edge words are re-read by the neighbouring bands
// and strips (non-temporal loads measured -13..-20 %).
template <int VEC>
__device__ __forceinline__ void load_words(const uint32_t* rp, int col, Words<VEC>& d) {
    if constexpr (VEC == 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(rp + col);
        d.w[0] = v.x; d.w[1] = v.y; d.w[2] = v.z; d.w[3] = v.w;
    } else if constexpr (VEC == 2) {
        const uint2 v = *reinterpret_cast<const uint2*>(rp + col);
        d.w[0] = v.x; d.w[1] = v.y;
    } else {
        d.w[0] = rp[col];
    }
}

// load_words with the non-temporal hint (NT) or without.
template <int VEC, bool NT>
__device__ __forceinline__ void load_words_k(const uint32_t* rp, int col, Words<VEC>& d) {
    if constexpr (NT && VEC == 4) {
        const U32x4 v = __builtin_nontemporal_load(reinterpret_cast<const U32x4*>(rp + col));
        d.w[0] = v[0]; d.w[1] = v[1]; d.w[2] = v[2]; d.w[3] = v[3];
    } else if constexpr (NT && VEC == 2) {
        const U32x2 v = __builtin_nontemporal_load(reinterpret_cast<const U32x2*>(rp + col));
        d.w[0] = v[0]; d.w[1] = v[1];
    } else if constexpr (NT) {
        d.w[0] = __builtin_nontemporal_load(rp + col);
    } else {
        load_words<VEC>(rp, col, d);
    }
}

// Store one lane's VEC words of an output row through a buffer descriptor
// built from the (wave-uniform) row address: lanes that do not own their
// words and rows outside the band get an out-of-range offset / a zero-sized
// row and the hardware bounds check drops the store.  No exec-mask branch
// around the store, so the counted vmcnt waits of the loads that follow stay
// exact (a skippable store makes the compiler wait for the worse path).
template <int VEC, bool NT = false>
__device__ __forceinline__ void store_row(uint32_t* row, bool row_ok, int32_t row_bytes, int col, bool lane_ok,
                                          const Words<VEC>& d) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(row, (short)0, row_ok ? row_bytes : 0, 0x00020000);
    const int voff = lane_ok ? col * 4 : 0x7FFFFFF0;
    if constexpr (VEC == 4) {
        const U32x4 v = {d.w[0], d.w[1], d.w[2], d.w[3]};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, 0, NT ? 2 : 0);
    } else if constexpr (VEC == 2) {
        const U32x2 v = {d.w[0], d.w[1]};
        __builtin_amdgcn_raw_buffer_store_b64(v, rs, voff, 0, NT ? 2 : 0);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32(d.w[0], rs, voff, 0, NT ? 2 : 0);
    }
}

// Wave -> (row range, column strip, band of the range): range 0's bands
// come first, then range 1's (StepParams).  Wave-uniform.
// XCD-aware block order.  The dispatcher places block b on XCD b % 8, and
// the XCDs have separate L2s.  A strip's halo lanes make every wave-load of
// a 62-output-lane strip straddle cache lines shared with the neighbouring
// strips, so blocks of adjacent strips on different XCDs fetch those lines
// twice.  Within each group of 8 * C dispatched blocks, XCD x runs logical
// blocks x*C .. x*C + C - 1 (adjacent strips of one band); the logical order
// -- band-major, tail bands last -- is kept at the granularity of a group.
// Blocks past the last whole group keep their index.  Measured with
// scripts/micro/band_stream.hip (DESIGN.md §4 "Memory operations").
__device__ __forceinline__ int xcd_block(int b, int nblocks, int chunk) {
    const int group = 8 * chunk;
    if (chunk <= 1 || b >= nblocks / group * group) return b;
    const int g = b / group, r = b - g * group;
    return g * group + (r & 7) * chunk + (r >> 3);
}

// Launch clock probe (profiling only, p.clk non-null): wave 0 of every
// workgroup reads its CU's core-clock counter (s_memtime) and the 100 MHz
// reference counter (s_memrealtime) when it starts and when it ends, and adds
// both differences into the launch's slot with vector atomics (a sample of
// the workgroups, spread over sub-slots).  The core
// counters of different CUs are not aligned, so only same-wave differences
// are used; the host divides the two sums (gol_profile_clock).
struct ClockStart {
    unsigned long long mt, rt;
};

__device__ __forceinline__ ClockStart clock_probe_begin(const unsigned long long* clk) {
    if (clk == nullptr) return {0, 0};
    return {__builtin_amdgcn_s_memtime(), __builtin_amdgcn_s_memrealtime()};
}

__device__ __forceinline__ void clock_probe_end(unsigned long long* clk, ClockStart t0) {
    // One workgroup in kClockSampleEvery reports, into one of kClockSubSlots
    // cache lines: a single-generation launch has ~10^5 workgroups, and
    // atomics on one address serialise (every workgroup on two addresses
    // made the 65536^2 single-generation pass 4x slower).
    if (clk == nullptr || threadIdx.x != 0 || blockIdx.x % kClockSampleEvery != 0) return;
    const unsigned long long mt = __builtin_amdgcn_s_memtime(), rt = __builtin_amdgcn_s_memrealtime();
    unsigned long long* sub = clk + (blockIdx.x / kClockSampleEvery % kClockSubSlots) * kClockSubWords;
    atomicAdd(sub + 0, mt - t0.mt);
    atomicAdd(sub + 1, rt - t0.rt);
}

struct WaveTile {
    int range, strip, band;
};
__device__ __forceinline__ WaveTile wave_tile(const StepParams& p, int wave) {
    const int n0 = p.nbands[0] * p.strips;
    const int range = wave >= n0 ? 1 : 0;
    const int w = range ? wave - n0 : wave;
    return {range, w % p.strips, w / p.strips};
}

// Local row pointer for r in [-G, rows + G).  Wave-uniform and built from
// selects rather than branches: it runs once per stream row inside the
// unrolled loops.  Only tori shorter than a pass's halo (rows < G) take the
// one uniform branch, to wrap more than once.
__device__ __forceinline__ const uint32_t* row_ptr(const StepParams& p, int r, int G) {
    const bool top = r < 0, bot = r >= p.rows;
    int w = top ? r + p.rows : (bot ? r - p.rows : r);  // torus: one wrap
    if (p.wrap_y && p.rows < G) {
        w = r % p.rows;
        w = w < 0 ? w + p.rows : w;
    }
    const bool halo = !p.wrap_y && (top || bot);
    const uint32_t* base = halo ? (top ? p.halo_top : p.halo_bot) : p.cur;
    const int64_t idx = halo ? (top ? r + G : r - p.rows) : (p.wrap_y ? w : r);
    return base + idx * (halo ? p.halo_stride : p.pitch);
}

template <bool CLIPPED>
__device__ __forceinline__ bool row_visible(const StepParams& p, int r) {
    if constexpr (CLIPPED) {
        const int64_t g = p.grow0 + r;
        return g >= 0 && g < p.vis_rows;
    } else {
        return true;
    }
}

// v_bitop3_b32 truth tables: imm = f(S0 = 0xF0, S1 = 0xCC, S2 = 0xAA).
constexpr uint32_t kXor3 = 0x96;         // a ^ b ^ c
constexpr uint32_t kMaj = 0xE8;          // majority(a, b, c)
constexpr uint32_t kNotAXorBC = 0x06;    // ~a & (b ^ c)
constexpr uint32_t kAAndBOrC = 0xE0;     // a & (b | c)

#define GOL_BITOP3(a, b, c, imm) __builtin_amdgcn_bitop3_b32((a), (b), (c), (imm))

// Full-sum B3/S23 circuit (rule_b3s23_fullsum).  Truth tables index bit (a << 2 | b << 1 | c).
constexpr uint32_t kXnor3 = 0x69;      // ~(a ^ b ^ c): the plane's 3-sum is 0 or 2
constexpr uint32_t kNotAllEq = 0x7E;   // the plane's 3-sum is 1 or 2
constexpr uint32_t kRuleT1 = 0x56;
constexpr uint32_t kRuleT2 = 0x45;
constexpr uint32_t kRuleOut = 0x28;    // (a ^ b) & c

// B3/S23 from the full 9-cell sum S = a + c + b of three 2-bit terms (row or
// column 3-sums, bit planes x0/x1): alive next iff S == 3 or (S == 4 and the
// centre is alive).  Per bit plane one "sum is even" and one "terms not all
// equal" bitop3, then a 3-gate tail: 7 v_bitop3, where the centre-less count
// (n = S - centre, then ~qq & (pp ^ c0) & (n0 | alive)) takes 7 + the
// centre's removal.  Found by exhaustive search over 3-gate circuits on
// symmetric plane encodings (DESIGN.md §4 "Rule circuit"), checked on every
// input by tests/test_rule_circuit.py.  Only for tori: on clipped boards the
// visible centre (summed) and the alive centre differ at the sink cells.
__device__ __forceinline__ uint32_t rule_b3s23_fullsum(uint32_t a0, uint32_t a1, uint32_t c0, uint32_t c1,
                                                       uint32_t b0, uint32_t b1, uint32_t alive) {
    const uint32_t e1 = GOL_BITOP3(a0, c0, b0, kXnor3);
    const uint32_t e2 = GOL_BITOP3(a0, c0, b0, kNotAllEq);
    const uint32_t f1 = GOL_BITOP3(a1, c1, b1, kXnor3);
    const uint32_t f2 = GOL_BITOP3(a1, c1, b1, kNotAllEq);
    const uint32_t t1 = GOL_BITOP3(e1, e2, f2, kRuleT1);
    const uint32_t t2 = GOL_BITOP3(e1, alive, t1, kRuleT2);
    return GOL_BITOP3(e2, f1, t2, kRuleOut);
}

// Row-pair-shared B3/S23 (multistep_hg_kernel on tori).  Output rows m and
// m + 1 (m even) both sum h(m) + h(m + 1); their binary sum P (0..6, three
// planes) is formed once and each row adds its own third h:
//   S(m) = h(m - 1) + P,  S(m + 1) = P + h(m + 2).
// The 4-gate tail takes P, the third row's (x1 x0) and the centre; both
// rows' centres lie inside P's two rows, so P = 0 with a live centre never
// occurs and the tail may treat it as a don't-care.  It was found by
// exhaustive search over 4-gate 3-input circuits on the binary P (DESIGN.md
// section 4 "Row-pair-shared circuit", scripts/circuit_search/: no 3-gate
// tail exists for any 3-plane code of P, and no 3 gates over a + b separate
// its values) and is checked on every input by tests/test_rule_circuit.py.
// Per two rows: 4 + 2 x 4 gates instead of 2 x 7.
constexpr uint32_t kPairT1 = 0x43;
constexpr uint32_t kPairT2 = 0x18;
constexpr uint32_t kPairT3 = 0x26;
constexpr uint32_t kPairOut = 0xD0;

template <int VEC>
struct PairSum {
    uint32_t p0[VEC], p1[VEC], p2[VEC];
};

template <int VEC>
__device__ __forceinline__ void pair_sum(const uint32_t (&a0)[VEC], const uint32_t (&a1)[VEC],
                                         const uint32_t (&b0)[VEC], const uint32_t (&b1)[VEC], PairSum<VEC>& P) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        const uint32_t k = a0[j] & b0[j];
        P.p0[j] = a0[j] ^ b0[j];
        P.p1[j] = GOL_BITOP3(a1[j], b1[j], k, kXor3);
        P.p2[j] = GOL_BITOP3(a1[j], b1[j], k, kMaj);
    }
}

__device__ __forceinline__ uint32_t rule_b3s23_pair(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t x0, uint32_t x1,
                                                    uint32_t alive) {
    const uint32_t g1 = GOL_BITOP3(p0, x0, alive, kPairT1);
    const uint32_t g2 = GOL_BITOP3(p1, p2, g1, kPairT2);
    const uint32_t g3 = GOL_BITOP3(p2, x1, g2, kPairT3);
    return GOL_BITOP3(g3, alive, g1, kPairOut);
}

// Column sums of the visible rows: (v1 v0) = a + c + b (the full 3-cell
// column, seen by the columns left and right of it) and (p1 p0) = a + b (the
// column minus its centre, seen by the centre cell itself).
template <int VEC, bool CLIPPED>
__device__ __forceinline__ void column_sums(const Words<VEC>& A, const Words<VEC>& C, const Words<VEC>& B,
                                            bool va, bool vc, bool vb, const uint32_t (&cmask)[VEC],
                                            uint32_t (&v0)[VEC], uint32_t (&v1)[VEC], uint32_t (&p0)[VEC],
                                            uint32_t (&p1)[VEC]) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        uint32_t a = A.w[j], c = C.w[j], b = B.w[j];
        if constexpr (CLIPPED) {
            a = va ? (a & cmask[j]) : 0u;
            c = vc ? (c & cmask[j]) : 0u;
            b = vb ? (b & cmask[j]) : 0u;
        }
        v0[j] = GOL_BITOP3(a, c, b, kXor3);
        v1[j] = GOL_BITOP3(a, c, b, kMaj);
        p0[j] = a ^ b;
        p1[j] = a & b;
    }
}

// The rule on one lane's VEC words from the column sums of its words, of the
// word left of them (m0 m1) and of the word right of them (n0 n1).
//   n = v(x-1) + v(x+1) + (a + b)(x)   -- the 8 neighbours, three 2-bit terms
//   bit 0: n0 = xor3(w0, e0, p0), carry c0 = maj(w0, e0, p0)
//   bit 1: weight-2 terms w1 + e1 + p1 = pp + 2 qq, pp = xor3, qq = maj
//   n = n0 + 2 (pp + c0) + 4 qq
// B3/S23: next = (n == 3) | (alive & n == 2) = ~qq & (pp ^ c0) & (n0 | alive)
// (pp ^ c0 = 1 means exactly one of pp, c0 is set, so bit 2 is qq; n = 8 has
// pp = c0 = 0 and dies) -- two v_bitop3 after the adder.
//
// ILV (interleaved words, DESIGN.md "Data layout"): a group of ILV words
// holds 32 * ILV consecutive columns, column 32 ILV k + ILV b + j in bit b of
// word j of group k.  The column left of word j > 0 is word j - 1 itself and
// the column right of word j < ILV - 1 is word j + 1 itself; only word 0's west
// neighbour (the group's last word shifted up one bit, the bit shifted in
// being the previous group's last column) and the last word's east neighbour
// (the group's first word shifted down, the next group's first column coming
// in) need a funnel shift.  ILV = 1 is the row-major layout (two shifts per
// word), ILV = 2 the pair layout (one per word) -- v_alignbit issues at half
// the rate of v_bitop3 on gfx950.
template <int ILV, int VEC, typename T>
__device__ __forceinline__ void neighbours(const T (&v)[VEC], T l, T r, int j, T& w, T& e) {
    // l: the word left of word 0 (the previous lane's last), r: the word right
    // of word VEC - 1 (the next lane's first)
    const T lw = j == 0 ? l : v[j - 1];
    const T re = j == VEC - 1 ? r : v[j + 1];
    if constexpr (ILV == 1) {
        w = __builtin_amdgcn_alignbit(v[j], lw, 31);  // column x-1
        e = __builtin_amdgcn_alignbit(re, v[j], 1);   // column x+1
    } else {
        const int ph = j % ILV;
        w = ph == 0 ? __builtin_amdgcn_alignbit(v[j + ILV - 1], lw, 31) : lw;
        e = ph == ILV - 1 ? __builtin_amdgcn_alignbit(re, v[j - ILV + 1], 1) : re;
    }
}

template <int VEC, bool LIFE, int ILV, bool CLIPPED>
__device__ __forceinline__ void rule_words(const StepParams& p, const uint32_t (&v0)[VEC],
                                           const uint32_t (&v1)[VEC], const uint32_t (&p0)[VEC],
                                           const uint32_t (&p1)[VEC], uint32_t m0, uint32_t m1, uint32_t n0,
                                           uint32_t n1, const Words<VEC>& alive, Words<VEC>& out) {
    static_assert(VEC % ILV == 0, "whole interleave groups per lane");
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        uint32_t w0, e0, w1, e1;
        neighbours<ILV>(v0, m0, n0, j, w0, e0);
        neighbours<ILV>(v1, m1, n1, j, w1, e1);
        if constexpr (LIFE && !CLIPPED) {
            // full 9-cell sum S = v(x-1) + v(x) + v(x+1): the gate circuit of
            // rule_hg (rule_b3s23_fullsum); the centre-less pair p is unused
            out.w[j] = rule_b3s23_fullsum(w0, w1, v0[j], v1[j], e0, e1, alive.w[j]);
            continue;
        }
        const uint32_t nb0 = GOL_BITOP3(w0, e0, p0[j], kXor3);
        const uint32_t c0 = GOL_BITOP3(w0, e0, p0[j], kMaj);
        const uint32_t pp = GOL_BITOP3(w1, e1, p1[j], kXor3);
        const uint32_t qq = GOL_BITOP3(w1, e1, p1[j], kMaj);
        const uint32_t al = alive.w[j];
        if constexpr (LIFE) {
            const uint32_t x = GOL_BITOP3(qq, pp, c0, kNotAXorBC);
            out.w[j] = GOL_BITOP3(x, nb0, al, kAAndBOrC);
        } else {
            const uint32_t n1b = pp ^ c0, k = pp & c0;
            const uint32_t n2b = qq ^ k, n3b = qq & k;
            const uint32_t n0b = nb0;
            uint32_t L[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const uint32_t sm = ((p.survive >> k) & 1u) ? 0xFFFFFFFFu : 0u;
                const uint32_t bm = ((p.birth >> k) & 1u) ? 0xFFFFFFFFu : 0u;
                L[k] = bfi(al, sm, bm);
            }
            const uint32_t m01 = bfi(n0b, L[1], L[0]), m23 = bfi(n0b, L[3], L[2]);
            const uint32_t m45 = bfi(n0b, L[5], L[4]), m67 = bfi(n0b, L[7], L[6]);
            const uint32_t m03 = bfi(n1b, m23, m01), m47 = bfi(n1b, m67, m45);
            const uint32_t m07 = bfi(n2b, m47, m03);
            out.w[j] = bfi(n3b, L[8], m07);
        }
    }
}

// Fused state hash, a function of the cells alone: the
// canonical words E, O of column group g (columns 64g .. 64g + 63: E its even
// columns, O its odd ones) of global row y contribute
// (E A(y, 0) + O A(y, 1)) B(g) (mod 2^64), A(y, 1) = A(y, 0) + kHashOddAdd.
// On the pair layout (ILV = 2) a lane's device words ARE the canonical words,
// so a lane sums w * A over the rows it streams -- one v_mad_u64_u32 per word
// and generation, the row key A an SGPR computed once per row on the scalar
// unit -- and multiplies by its group key B once, when it flushes
// (hash_lane_total).  Row-major lanes (ILV = 1: clipped boards, tori with an
// odd word count) unzip each word into its even and odd columns first
// (unzip_bits) -- the canonical words of the pair the word belongs to.  A
// lane's words share B per group: VEC = 2 one group, VEC = 4 two (two sums;
// the row's first word index is even), VEC = 1 half a group (odd_lane: the
// upper half).
__device__ __forceinline__ uint32_t unzip_bits(uint32_t x) {
    // even bits -> 0..15, odd bits -> 16..31 (outer unshuffle, 4 delta swaps)
    uint32_t t = (x ^ (x >> 1)) & 0x22222222u;
    x ^= t ^ (t << 1);
    t = (x ^ (x >> 2)) & 0x0C0C0C0Cu;
    x ^= t ^ (t << 2);
    t = (x ^ (x >> 4)) & 0x00F000F0u;
    x ^= t ^ (t << 4);
    t = (x ^ (x >> 8)) & 0x0000FF00u;
    x ^= t ^ (t << 8);
    return x;
}

template <int VEC>
struct HashAcc {
    static constexpr int kGroups = VEC >= 2 ? VEC / 2 : 1;
    unsigned long long a[kGroups];
};

template <int VEC>
__device__ __forceinline__ void hash_clear(HashAcc<VEC>& h) {
#pragma unroll
    for (int k = 0; k < HashAcc<VEC>::kGroups; ++k) h.a[k] = 0;
}

// One output row with row keys ae = A(y, 0), ao = A(y, 1) (both 0: the row
// is not hashed); odd_lane: VEC = 1 lanes holding a group's second word.
template <int VEC, int ILV>
__device__ __forceinline__ void hash_row_keys(uint32_t ae, uint32_t ao, const Words<VEC>& o, bool odd_lane,
                                              HashAcc<VEC>& h) {
    if constexpr (ILV == 2) {
        static_assert(VEC % 2 == 0, "whole pairs per lane");
#pragma unroll
        for (int j = 0; j < VEC; ++j)
            h.a[j / 2] += (unsigned long long)o.w[j] * (unsigned long long)((j & 1) ? ao : ae);
    } else if constexpr (VEC == 1) {
        const uint32_t u = unzip_bits(o.w[0]);
        const uint32_t e = odd_lane ? u << 16 : u & 0xFFFFu;
        const uint32_t d = odd_lane ? u & 0xFFFF0000u : u >> 16;
        h.a[0] += (unsigned long long)e * ae + (unsigned long long)d * ao;
    } else {
#pragma unroll
        for (int j = 0; j < VEC; j += 2) {
            const uint32_t u0 = unzip_bits(o.w[j]), u1 = unzip_bits(o.w[j + 1]);
            const uint32_t e = (u0 & 0xFFFFu) | (u1 << 16), d = (u0 >> 16) | (u1 & 0xFFFF0000u);
            h.a[j / 2] += (unsigned long long)e * ae + (unsigned long long)d * ao;
        }
    }
}

// One output row at global row `grow`.
template <int VEC, int ILV>
__device__ __forceinline__ void hash_row(int64_t grow, const Words<VEC>& o, bool odd_lane, HashAcc<VEC>& h) {
    const uint32_t ae = hash_row_key(grow);
    hash_row_keys<VEC, ILV>(ae, ae + kHashOddAdd, o, odd_lane, h);
}

// The horizontal-first kernel keeps its per-generation sums in LDS, one u64
// per lane, pair and generation, added to with ds_add_u64 (no return): 2G
// fewer VGPRs than register sums, which at G = 6..8 is a wave per SIMD.
template <int VEC, int ILV>
__device__ __forceinline__ void hash_row_lds(uint32_t ae, uint32_t ao, const Words<VEC>& o, bool odd_lane,
                                             unsigned long long* slot) {
    HashAcc<VEC> t;
    hash_clear(t);
    hash_row_keys<VEC, ILV>(ae, ao, o, odd_lane, t);
#pragma unroll
    for (int k = 0; k < HashAcc<VEC>::kGroups; ++k) atomicAdd(slot + k * kWaveLanes, t.a[k]);
}

// The lane's contribution: its sums times their column-group keys (words
// col .. col + VEC - 1; col even when VEC >= 2), or 0 for a lane that owns no
// words.
template <int VEC>
__device__ __forceinline__ unsigned long long hash_lane_total(const HashAcc<VEC>& h, int col, bool owns) {
    unsigned long long t = 0;
#pragma unroll
    for (int k = 0; k < HashAcc<VEC>::kGroups; ++k)
        t += h.a[k] * (unsigned long long)hash_pair_key((uint32_t)(col / 2) + (uint32_t)k);
    return owns ? t : 0ull;
}

// wave reduce -> workgroup reduce -> one atomic per workgroup into a sharded slot
__device__ __forceinline__ void hash_flush(unsigned long long acc, unsigned long long* slots, int lane,
                                           int wave_in_wg) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, kWaveLanes);
    __shared__ unsigned long long part[kWavesPerWG];
    __syncthreads();
    if (lane == 0) part[wave_in_wg] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
#pragma unroll
        for (int w = 0; w < kWavesPerWG; ++w) t += part[w];
        atomicAdd(slots + (size_t)(blockIdx.x % kHashSlots) * kHashSlotStride, t);
    }
}

// All G generations of a multi-generation pass at once: the G wave reductions
// interleaved, one barrier, and workgroup thread s sums and adds generation
// s (hash_flush once per generation paid 2G barriers per workgroup: on small
// boards, where a wave streams a few dozen rows, that was a visible share).
template <int G>
__device__ __forceinline__ void hash_flush_gens(unsigned long long (&acc)[G], unsigned long long* slots, int lane,
                                                int wave_in_wg) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int s = 0; s < G; ++s) acc[s] += __shfl_xor(acc[s], off, kWaveLanes);
    __shared__ unsigned long long part[kWavesPerWG][G];
    if (lane == 0) {
#pragma unroll
        for (int s = 0; s < G; ++s) part[wave_in_wg][s] = acc[s];
    }
    __syncthreads();
    const int s = threadIdx.x;
    if (s < G) {
        unsigned long long t = 0;
#pragma unroll
        for (int w = 0; w < kWavesPerWG; ++w) t += part[w][s];
        atomicAdd(slots + (size_t)s * kHashGenStride + (size_t)(blockIdx.x % kHashSlots) * kHashSlotStride, t);
    }
}

// --------------------------------------------------------------------------
// One generation per pass.
// --------------------------------------------------------------------------
// Single-generation passes store non-temporally: the next plane is not
// re-read by this pass, and with the 4-row bands the store stream competes
// with the halo re-reads for the caches.  Same-box A/B
// (profiles/r02_g1_nt_ab.txt, 3 rounds): 65536^2 0.1963 -> 0.1891 ms,
// 262144^2 3.129 -> 3.003 ms, 262144 x 32768 0.399 -> 0.383 ms per
// generation.  The multi-generation kernels keep plain stores (round 1:
// -3..-8 % at G = 6 with non-temporal stores, profiles/r01_bandwidth.txt).
constexpr bool kG1NtStores = true;

template <int VEC, bool LIFE, bool HASH, bool CLIPPED, int ILV>
__global__ __launch_bounds__(kWaveLanes* kWavesPerWG) void step_kernel(const StepParams p) {
    const int lane = threadIdx.x & (kWaveLanes - 1);
    const int wave_in_wg = __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveLanes);
    const WaveTile tile = wave_tile(p, xcd_block(blockIdx.x, gridDim.x, p.xcd_chunk) * kWavesPerWG + wave_in_wg);
    const ClockStart clk0 = clock_probe_begin(p.clk);
    const int rg = tile.range, strip = tile.strip, bandi = tile.band;
    unsigned long long acc = 0;

    if (bandi < p.nbands[rg]) {
        HashAcc<VEC> hacc;
        hash_clear(hacc);
        const int r_begin = p.row_lo[rg] + bandi * p.band[rg];
        const int r_end = min(r_begin + p.band[rg], p.row_hi[rg]);
        const int nrows = r_end - r_begin;
        const int s0 = strip * (kWaveLanes * VEC);
        const int nact = min(kWaveLanes, (p.wwords - s0) / VEC);
        const int col = s0 + lane * VEC;
        const bool active = lane < nact;
        const int lcolumn = active ? col : s0;  // clamped load column
        // Edge words; an edge outside a clipped board is read from a clamped
        // in-row index and masked to zero.
        int lcol = s0 - 1;
        bool lvalid = true;
        if (lcol < 0) { lvalid = p.wrap_x != 0; lcol = p.wwords - 1; }
        int rcol = s0 + nact * VEC;
        bool rvalid = true;
        if (rcol >= p.wwords) { rvalid = p.wrap_x != 0; rcol = 0; }
        const int ecol = lane == 0 ? lcol : rcol;  // lane 0: left edge, others: right edge
        uint32_t cmask[VEC], omask[VEC], emask = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            cmask[j] = CLIPPED ? col_mask(p.vis_cols, col + j) : 0xFFFFFFFFu;
            omask[j] = CLIPPED ? col_mask(p.width, col + j) : 0xFFFFFFFFu;
        }
        if constexpr (CLIPPED) {
            const uint32_t lm = lvalid ? col_mask(p.vis_cols, lcol) : 0u;
            const uint32_t rm = rvalid ? col_mask(p.vis_cols, rcol) : 0u;
            emask = lane == 0 ? lm : rm;
        }
        const bool odd_lane = (col & 1) != 0;
        const bool up = (bandi & 1) != 0;
        // t-th stream row (t = 0 .. nrows+1) and i-th output row.
        auto row_of = [&](int t) -> int { return up ? r_end - t : r_begin - 1 + t; };
        auto out_of = [&](int i) -> int { return up ? r_end - 1 - i : r_begin + i; };

        // Ring of stream rows: the lane's VEC words + its edge word.  The edge
        // word rides the in-order vector memory pipe so the counted vmcnt
        // waits cover it like the row data (a scalar load would need an
        // out-of-order lgkmcnt(0) wait on every row).
        Words<VEC> ring[kRing];
        uint32_t edge[kRing];
        auto load_t = [&](int t, Words<VEC>& d, uint32_t& e) {
            const uint32_t* rp = row_ptr(p, row_of(t), 1);
            load_words<VEC>(rp, lcolumn, d);
            e = rp[ecol];
        };
        // output row i from stream rows i (above), i + 1 (centre), i + 2 (below)
        auto step_rows = [&](int i, const Words<VEC>& RA, const Words<VEC>& RC, const Words<VEC>& RB, uint32_t eA,
                             uint32_t eC, uint32_t eB, bool in_band) {
            const bool va = row_visible<CLIPPED>(p, row_of(i));
            const bool vc = row_visible<CLIPPED>(p, row_of(i + 1));
            const bool vb = row_visible<CLIPPED>(p, row_of(i + 2));
            uint32_t v0[VEC], v1[VEC], p0[VEC], p1[VEC];
            column_sums<VEC, CLIPPED>(RA, RC, RB, va, vc, vb, cmask, v0, v1, p0, p1);
            if constexpr (CLIPPED) {
                eA = va ? (eA & emask) : 0u;
                eC = vc ? (eC & emask) : 0u;
                eB = vb ? (eB & emask) : 0u;
            }
            const uint32_t te = eA ^ eC;
            const uint32_t ev0 = te ^ eB, ev1 = bfi(te, eB, eA);
            // Left / right neighbour column sums: the adjacent lane's, or --
            // where DPP has no source lane -- `old`, this lane's edge word.
            const uint32_t m0 = dpp_shr1(ev0, v0[VEC - 1]);
            const uint32_t m1 = dpp_shr1(ev1, v1[VEC - 1]);
            uint32_t n0 = dpp_shl1(ev0, v0[0]);
            uint32_t n1 = dpp_shl1(ev1, v1[0]);
            if (nact < kWaveLanes) {  // narrow strip: the last active lane is not lane 63
                const uint32_t r0 = __builtin_amdgcn_readlane(ev0, 1);  // lane 1 holds the right edge
                const uint32_t r1 = __builtin_amdgcn_readlane(ev1, 1);
                const bool last = lane == nact - 1;
                n0 = last ? r0 : n0;
                n1 = last ? r1 : n1;
            }
            Words<VEC> o;
            rule_words<VEC, LIFE, ILV, CLIPPED>(p, v0, v1, p0, p1, m0, m1, n0, n1, RC, o);
            if constexpr (CLIPPED) {
#pragma unroll
                for (int j = 0; j < VEC; ++j) o.w[j] &= omask[j];
            }
            const int r = out_of(i);
            store_row<VEC, kG1NtStores>(p.nxt + (int64_t)r * p.pitch, in_band, p.wwords * 4, col, active, o);
            if constexpr (HASH) {
                if (in_band) hash_row<VEC, ILV>(p.grow0 + r, o, odd_lane, hacc);
            }
        };
        auto step_i = [&](int i, int u, bool in_band) {
            const int ua = u % kRing, uc = (u + 1) % kRing, ub = (u + 2) % kRing;
            step_rows(i, ring[ua], ring[uc], ring[ub], edge[ua], edge[uc], edge[ub], in_band);
        };

        // The single-generation pass's own band heights (pick_band): the B + 2
        // stream rows issued at once, each once, and B steps.  The B - 2
        // middle rows are read by this wave alone -- the two edge rows and
        // the two halo rows are also a neighbouring band's halo or edge rows,
        // kept in the caches for that second reader -- so they load
        // non-temporally.
        auto band_path = [&](auto BB) __attribute__((always_inline)) {
            constexpr int B = decltype(BB)::value;
            Words<VEC> rs[B + 2];
            uint32_t es[B + 2];
            static_for<B + 2>([&](auto T) __attribute__((always_inline)) {
                constexpr int t = decltype(T)::value;
                const uint32_t* rp = row_ptr(p, row_of(t), 1);
                load_words_k<VEC, (t >= 2 && t <= B - 1)>(rp, lcolumn, rs[t]);
                es[t] = rp[ecol];
            });
            static_for<B>([&](auto I) __attribute__((always_inline)) {
                constexpr int i = decltype(I)::value;
                step_rows(i, rs[i], rs[i + 1], rs[i + 2], es[i], es[i + 1], es[i + 2], true);
            });
        };
        if (nrows == 4) {
            band_path(std::integral_constant<int, 4>{});
        } else if (nrows == 6) {
            band_path(std::integral_constant<int, 6>{});
        } else if (nrows == 8) {
            band_path(std::integral_constant<int, 8>{});
        } else {
            // Loads are never predicated: stream rows past the band's last one
            // are clamped to it, and steps past the band compute into the void
            // (their stores are skipped), so the loop body is straight-line.
            const int tmax = nrows + 1;
#pragma unroll
            for (int t = 0; t < kRing - 1; ++t) load_t(min(t, tmax), ring[t], edge[t]);
            for (int i0 = 0; i0 < nrows; i0 += kRing) {
#pragma unroll
                for (int u = 0; u < kRing; ++u) {
                    const int i = i0 + u;
                    const int sl = (u + kRing - 1) % kRing;
                    load_t(min(i + kRing - 1, tmax), ring[sl], edge[sl]);
                    step_i(i, u, i < nrows);
                }
            }
        }
        if constexpr (HASH) acc = hash_lane_total(hacc, col, active);
    }
    if constexpr (HASH) hash_flush(acc, p.hash_slots, lane, wave_in_wg);
    clock_probe_end(p.clk, clk0);
}

// --------------------------------------------------------------------------
// G generations per pass (temporal blocking).
// --------------------------------------------------------------------------
template <int VEC, int G, bool LIFE, bool HASH, bool CLIPPED, int ILV>
__global__ __launch_bounds__(kWaveLanes* kWavesPerWG) void multistep_kernel(const StepParams p) {
    static_assert(G >= 2 && G <= kMaxGensPerPass, "G");
    static_assert(G < 32 * VEC, "halo lane narrower than the garbage front");
    constexpr int kOut = (kWaveLanes - 2) * VEC;  // output words per strip
    const int lane = threadIdx.x & (kWaveLanes - 1);
    const int wave_in_wg = __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveLanes);
    const WaveTile tile = wave_tile(p, xcd_block(blockIdx.x, gridDim.x, p.xcd_chunk) * kWavesPerWG + wave_in_wg);
    const ClockStart clk0 = clock_probe_begin(p.clk);
    const int rg = tile.range, strip = tile.strip, bandi = tile.band;
    unsigned long long acc[G];
#pragma unroll
    for (int s = 0; s < G; ++s) acc[s] = 0;

    if (bandi < p.nbands[rg]) {
        const int r_begin = p.row_lo[rg] + bandi * p.band[rg];
        const int r_end = min(r_begin + p.band[rg], p.row_hi[rg]);
        const int nrows = r_end - r_begin;
        const int n_in = nrows + 2 * G;  // stream rows r_begin-G .. r_end+G-1
        const int s0 = strip * kOut;
        const int nout = min(kOut, p.wwords - s0);
        const int col = s0 + (lane - 1) * VEC;  // lane 0: the strip's left halo
        const bool owns = lane >= 1 && (lane - 1) * VEC < nout;
        int lcol;
        bool incol;
        if (p.wrap_x) {
            lcol = col % p.wwords;
            if (lcol < 0) lcol += p.wwords;
            incol = true;
        } else {
            incol = col >= 0 && col < p.wwords;
            lcol = incol ? col : 0;
        }
        uint32_t cmask[VEC], omask[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            cmask[j] = CLIPPED ? (incol ? col_mask(p.vis_cols, col + j) : 0u) : 0xFFFFFFFFu;
            omask[j] = CLIPPED ? (incol ? col_mask(p.width, col + j) : 0u) : 0xFFFFFFFFu;
        }
        const bool odd_lane = (col & 1) != 0;
        HashAcc<VEC> hacc[G];
#pragma unroll
        for (int s = 0; s < G; ++s) hash_clear(hacc[s]);
        const bool up = (bandi & 1) != 0;
        // stream row m <-> local board row (the same for every stage)
        auto brow = [&](int m) -> int { return up ? r_end - 1 + G - m : r_begin - G + m; };
        auto vis = [&](int m) -> bool { return row_visible<CLIPPED>(p, brow(m)); };

        Words<VEC> in[kMRing];
        Words<VEC> st[G - 1][3];  // stage s (1..G-1) rows, slot = stream row % 3
#pragma unroll
        for (int k = 0; k < kMRing; ++k)
#pragma unroll
            for (int j = 0; j < VEC; ++j) in[k].w[j] = 0u;
#pragma unroll
        for (int s = 0; s < G - 1; ++s)
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int j = 0; j < VEC; ++j) st[s][k].w[j] = 0u;

        auto load_m = [&](int m, Words<VEC>& d) { load_words<VEC>(row_ptr(p, brow(m), G), lcol, d); };
        // one stencil application: rows above/centre/below -> out
        auto apply = [&](const Words<VEC>& A, const Words<VEC>& C, const Words<VEC>& B, int mc,
                         Words<VEC>& o) {
            uint32_t v0[VEC], v1[VEC], p0[VEC], p1[VEC];
            column_sums<VEC, CLIPPED>(A, C, B, vis(mc - 1), vis(mc), vis(mc + 1), cmask, v0, v1, p0, p1);
            // halo lanes 0 / 63 read zeros beyond their outer edge (bound_ctrl)
            const uint32_t m0 = dpp_shr1_zero(v0[VEC - 1]);
            const uint32_t m1 = dpp_shr1_zero(v1[VEC - 1]);
            const uint32_t n0 = dpp_shl1_zero(v0[0]);
            const uint32_t n1 = dpp_shl1_zero(v1[0]);
            rule_words<VEC, LIFE, ILV, CLIPPED>(p, v0, v1, p0, p1, m0, m1, n0, n1, C, o);
            if constexpr (CLIPPED) {
#pragma unroll
                for (int j = 0; j < VEC; ++j) o.w[j] &= omask[j];
            }
        };

        // Stream row q (slot u = q % kMRing): prefetch row q + kMPF, stage s
        // produces stream row q - s.
        auto row_step = [&](const int q, const int u) {
            load_m(min(q + kMPF, n_in - 1), in[(u + kMPF) % kMRing]);
            // stage 1: stream row q-1 from input rows q-2, q-1, q
            Words<VEC> o;
            apply(in[(u + kMRing - 2) % kMRing], in[(u + kMRing - 1) % kMRing], in[u], q - 1, o);
#pragma unroll
            for (int s = 1; s <= G; ++s) {
                const int m = q - s;  // stream row produced by stage s
                const bool own_row = m >= G && m < n_in - G;
                if (s < G) {
                    st[s - 1][((u - s) % 3 + 3) % 3] = o;
                    if constexpr (HASH) {
                        if (own_row) hash_row<VEC, ILV>(p.grow0 + brow(m), o, odd_lane, hacc[s - 1]);
                    }
                    // stage s+1: stream row q-s-1 from stage-s rows q-s-2, q-s-1, q-s
                    apply(st[s - 1][((u - s - 2) % 3 + 3) % 3], st[s - 1][((u - s - 1) % 3 + 3) % 3],
                          st[s - 1][((u - s) % 3 + 3) % 3], m - 1, o);
                } else {
                    const int r = brow(m);
                    store_row<VEC>(p.nxt + (int64_t)r * p.pitch, own_row, p.wwords * 4, lcol, owns, o);
                    if constexpr (HASH) {
                        if (own_row) hash_row<VEC, ILV>(p.grow0 + r, o, odd_lane, hacc[G - 1]);
                    }
                }
            }
        };

#pragma unroll
        for (int t = 0; t < kMPF; ++t) load_m(min(t, n_in - 1), in[t]);
        for (int q0 = 0; q0 < n_in; q0 += kMRing) {
#pragma unroll
            for (int u = 0; u < kMRing; ++u) row_step(q0 + u, u);
        }
        if constexpr (HASH) {
#pragma unroll
            for (int s = 0; s < G; ++s) acc[s] = hash_lane_total(hacc[s], col, owns);
        }
    }
    if constexpr (HASH) {
        hash_flush_gens<G>(acc, p.hash_slots, lane, wave_in_wg);
    }
    clock_probe_end(p.clk, clk0);
}

// --------------------------------------------------------------------------
// G generations per pass, horizontal-first count (variant 2).
//
// On arrival every row r (input or stage output) gets its horizontal 3-sum
// h = W(r) + r + E(r) (2 v_alignbit + 2 v_bitop3, 2 DPP moves per lane),
// shared by the three output rows that read it.  Output row m then needs
//   g(m) = h(m) - r(m)                 (the centre-less pair W + E, 2 ops)
//   n = h(m-1) + h(m+1) + g(m)         (one carry-save layer, 4 ops)
//   rule                               (2 ops for B3/S23)
// ~12 + 2/VEC VALU per word-generation instead of ~15.  Each ring row keeps
// (h0, h1, r) -- three planes -- so the rings hold more registers.
// --------------------------------------------------------------------------
constexpr uint32_t kAndOrNotC = 0xD0;  // a & (b | ~c)

template <int VEC, bool CLIPPED>
struct HRow {
    uint32_t h0[VEC], h1[VEC], r[VEC];  // r: the visible row
    uint32_t a[CLIPPED ? VEC : 1];       // clipped: the real row (alive bits)
};

template <int VEC, bool CLIPPED, int ILV, bool WR = false>
__device__ __forceinline__ void arrive(const Words<VEC>& raw, bool vis, const uint32_t (&cmask)[VEC],
                                       HRow<VEC, CLIPPED>& o) {
    uint32_t rv[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        rv[j] = CLIPPED ? (vis ? (raw.w[j] & cmask[j]) : 0u) : raw.w[j];
        if constexpr (CLIPPED) o.a[j] = raw.w[j];
    }
    // halo lanes read zeros at the wave's ends; a whole-row wave wraps
    const uint32_t left = WR ? dpp_ror1(rv[VEC - 1]) : dpp_shr1_zero(rv[VEC - 1]);
    const uint32_t right = WR ? dpp_rol1(rv[0]) : dpp_shl1_zero(rv[0]);
    static_assert(ILV == 1 || !CLIPPED, "clipped boards are row-major");
#pragma unroll
    for (int j = 0; j < VEC; ++j) {  // interleaved groups: see rule_words
        uint32_t w, e;
        neighbours<ILV>(rv, left, right, j, w, e);
        o.h0[j] = GOL_BITOP3(w, rv[j], e, kXor3);
        o.h1[j] = GOL_BITOP3(w, rv[j], e, kMaj);
        o.r[j] = rv[j];
    }
}

template <int VEC, bool LIFE, bool CLIPPED>
__device__ __forceinline__ void rule_hg(const StepParams& p, const HRow<VEC, CLIPPED>& A,
                                        const HRow<VEC, CLIPPED>& C, const HRow<VEC, CLIPPED>& B,
                                        const uint32_t (&omask)[VEC], Words<VEC>& out) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        if constexpr (LIFE && !CLIPPED) {
            // S = h(m-1) + h(m) + h(m+1): 7 v_bitop3 instead of g = h - r
            // (1 v_xor + 1 v_bitop3) and the centre-less count's 6
            out.w[j] = rule_b3s23_fullsum(A.h0[j], A.h1[j], C.h0[j], C.h1[j], B.h0[j], B.h1[j], C.r[j]);
            continue;
        }
        const uint32_t g0 = C.h0[j] ^ C.r[j];
        const uint32_t g1 = GOL_BITOP3(C.h1[j], C.h0[j], C.r[j], kAndOrNotC);
        const uint32_t nb0 = GOL_BITOP3(A.h0[j], B.h0[j], g0, kXor3);
        const uint32_t c0 = GOL_BITOP3(A.h0[j], B.h0[j], g0, kMaj);
        const uint32_t pp = GOL_BITOP3(A.h1[j], B.h1[j], g1, kXor3);
        const uint32_t qq = GOL_BITOP3(A.h1[j], B.h1[j], g1, kMaj);
        const uint32_t al = CLIPPED ? C.a[j] : C.r[j];
        uint32_t res;
        if constexpr (LIFE) {
            const uint32_t x = GOL_BITOP3(qq, pp, c0, kNotAXorBC);
            res = GOL_BITOP3(x, nb0, al, kAAndBOrC);
        } else {
            const uint32_t n1b = pp ^ c0, k = pp & c0;
            const uint32_t n2b = qq ^ k, n3b = qq & k;
            uint32_t L[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                const uint32_t sm = ((p.survive >> q) & 1u) ? 0xFFFFFFFFu : 0u;
                const uint32_t bm = ((p.birth >> q) & 1u) ? 0xFFFFFFFFu : 0u;
                L[q] = bfi(al, sm, bm);
            }
            const uint32_t m01 = bfi(nb0, L[1], L[0]), m23 = bfi(nb0, L[3], L[2]);
            const uint32_t m45 = bfi(nb0, L[5], L[4]), m67 = bfi(nb0, L[7], L[6]);
            const uint32_t m03 = bfi(n1b, m23, m01), m47 = bfi(n1b, m67, m45);
            const uint32_t m07 = bfi(n2b, m47, m03);
            res = bfi(n3b, L[8], m07);
        }
        out.w[j] = CLIPPED ? (res & omask[j]) : res;
    }
}

// The horizontal-first B3/S23 torus kernels share each even/odd row pair's
// middle sum (rule_b3s23_pair).  They run at the occupancy their registers
// give (G <= 10: 3 or more waves per SIMD); forced to more they spill.
template <int VEC, bool LIFE, bool CLIPPED>
constexpr bool kPairRows = LIFE && !CLIPPED && VEC <= 2;

// WR: a whole-row wave (gol_kernels.h whole_row_fits) -- 64 output lanes,
// the row's wrap a wave rotate, one strip.
template <int VEC, int G, bool LIFE, bool HASH, bool CLIPPED, int ILV, bool WR = false>
__global__ __launch_bounds__(kWaveLanes* kWavesPerWG) void multistep_hg_kernel(const StepParams p) {
    static_assert(VEC <= 2, "16-byte lanes run the vertical-first kernel");
    static_assert(G >= 2 && G <= kMaxGensPerPass, "G");
    static_assert(G < 32 * VEC, "halo lane narrower than the garbage front");
    static_assert(!WR || (LIFE && !CLIPPED && ILV == 2), "whole-row waves: B3/S23 tori in the pair layout");
    constexpr int kHaloLanes = WR ? 0 : 1;  // per side
    constexpr int kOut = (kWaveLanes - 2 * kHaloLanes) * VEC;
    const int lane = threadIdx.x & (kWaveLanes - 1);
    const int wave_in_wg = __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveLanes);
    const WaveTile tile = wave_tile(p, xcd_block(blockIdx.x, gridDim.x, p.xcd_chunk) * kWavesPerWG + wave_in_wg);
    const ClockStart clk0 = clock_probe_begin(p.clk);
    const int rg = tile.range, strip = tile.strip, bandi = tile.band;
    unsigned long long acc[G];
#pragma unroll
    for (int s = 0; s < G; ++s) acc[s] = 0;
    __shared__ unsigned long long hash_lds[HASH ? kWavesPerWG * G * HashAcc<VEC>::kGroups * kWaveLanes : 1];

    if (bandi < p.nbands[rg]) {
        const int r_begin = p.row_lo[rg] + bandi * p.band[rg];
        const int r_end = min(r_begin + p.band[rg], p.row_hi[rg]);
        const int nrows = r_end - r_begin;
        const int n_in = nrows + 2 * G;
        const int s0 = strip * kOut;
        const int nout = min(kOut, p.wwords - s0);
        const int col = s0 + (lane - kHaloLanes) * VEC;
        const bool owns = lane >= kHaloLanes && (lane - kHaloLanes) * VEC < nout;
        // The last strip of a row owns fewer than 62 lanes' words (4 of 62 pairs
        // at 262144 columns, 32 at 65536): lanes past its right halo lane would
        // only compute garbage.  Switch them off -- an exec-masked lane issues
        // nothing of its own and toggles no register bits, and this kernel is
        // held at its power limit (DESIGN.md §4 "Clock").  DPP reads a
        // switched-off lane as zero (bound_ctrl), as it reads past lane 63.
        // The hashed instances keep every lane: hash_flush reduces across all 64.
        if constexpr (!HASH && !WR) {
            if (lane > (nout + VEC - 1) / VEC + 1) return;
        }
        int lcol;
        bool incol;
        if (p.wrap_x) {
            lcol = col % p.wwords;
            if (lcol < 0) lcol += p.wwords;
            incol = true;
        } else {
            incol = col >= 0 && col < p.wwords;
            lcol = incol ? col : 0;
        }
        uint32_t cmask[VEC], omask[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            cmask[j] = CLIPPED ? (incol ? col_mask(p.vis_cols, col + j) : 0u) : 0xFFFFFFFFu;
            omask[j] = CLIPPED ? (incol ? col_mask(p.width, col + j) : 0u) : 0xFFFFFFFFu;
        }
        const bool odd_lane = (col & 1) != 0;
        constexpr int kNP = HashAcc<VEC>::kGroups;
        // this lane's LDS sums: generation s, pair k at hsum[(s * kNP + k) * kWaveLanes]
        unsigned long long* hsum = hash_lds + (size_t)wave_in_wg * G * kNP * kWaveLanes + lane;
        if constexpr (HASH) {
#pragma unroll
            for (int k = 0; k < G * kNP; ++k) hsum[k * kWaveLanes] = 0ull;
        }
        const bool up = (bandi & 1) != 0;
        auto brow = [&](int m) -> int { return up ? r_end - 1 + G - m : r_begin - G + m; };
        auto vis = [&](int m) -> bool { return row_visible<CLIPPED>(p, brow(m)); };

        Words<VEC> in[kMRing];
        HRow<VEC, CLIPPED> hr[G][3];  // ring s: arrivals of stage-s rows (stage 0 = input), slot = row % 3
        PairSum<VEC> pst[kPairRows<VEC, LIFE, CLIPPED> ? G : 1];  // stage s's last even-row P
#pragma unroll
        for (int s = 0; s < (kPairRows<VEC, LIFE, CLIPPED> ? G : 1); ++s)
#pragma unroll
            for (int j = 0; j < VEC; ++j) pst[s].p0[j] = pst[s].p1[j] = pst[s].p2[j] = 0u;
#pragma unroll
        for (int k = 0; k < kMRing; ++k)
#pragma unroll
            for (int j = 0; j < VEC; ++j) in[k].w[j] = 0u;
#pragma unroll
        for (int s = 0; s < G; ++s)
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int j = 0; j < VEC; ++j) {
                    hr[s][k].h0[j] = hr[s][k].h1[j] = hr[s][k].r[j] = 0u;
                    if constexpr (CLIPPED) hr[s][k].a[j] = 0u;
                }

        auto load_m = [&](int m, Words<VEC>& d) { load_words<VEC>(row_ptr(p, brow(m), G), lcol, d); };

        // Hash row keys: stage s at stream row q hashes stream row q - s, so a
        // shift register holds the keys of stream rows q .. q - G, 0 for rows
        // outside the band's own rows.  Each row's keys are computed once, on
        // the scalar unit, and no branch guards the multiply-adds.
        uint32_t kae[G + 1], kao[G + 1];
#pragma unroll
        for (int k = 0; k <= G; ++k) kae[k] = kao[k] = 0u;

        // Stream row q (ring slot u = q % kMRing): prefetch row q + kHgPF,
        // input row q arrives at ring 0, stage s produces stream row q - s.
        // Stage s has valid inputs only from q = 2s on (its rows m < s are
        // built from the clamped rows before the band and are never stored,
        // hashed or read by a valid row), so the pipeline fill -- the first
        // kFill rows, q known at compile time -- skips those stage steps.
        auto row_step = [&](const int q, const int u, const bool fill) __attribute__((always_inline)) {
            load_m(min(q + kHgPF, n_in - 1), in[(u + kHgPF) % kMRing]);
            if constexpr (HASH) {
#pragma unroll
                for (int k = G; k >= 1; --k) {
                    kae[k] = kae[k - 1];
                    kao[k] = kao[k - 1];
                }
                const bool own_q = q >= G && q < n_in - G;
                const uint32_t ae = hash_row_key(p.grow0 + brow(q));
                kae[0] = own_q ? ae : 0u;
                kao[0] = own_q ? ae + kHashOddAdd : 0u;
            }
            arrive<VEC, CLIPPED, ILV, WR>(in[u], vis(q), cmask, hr[0][u % 3]);
#pragma unroll
            for (int s = 1; s <= G; ++s) {
                // stages s.. have no valid row yet; a paired stage also runs the
                // step before its first valid row, to form that row's P when odd
                if (fill && q < 2 * s - (kPairRows<VEC, LIFE, CLIPPED> ? 1 : 0)) break;
                // stage s: stream row m = q - s from ring s-1 rows m-1, m, m+1
                const int m = q - s;
                Words<VEC> o;
                const HRow<VEC, CLIPPED>& A = hr[s - 1][((u - s - 1) % 3 + 3) % 3];
                const HRow<VEC, CLIPPED>& C = hr[s - 1][((u - s) % 3 + 3) % 3];
                const HRow<VEC, CLIPPED>& B = hr[s - 1][((u - s + 1) % 3 + 3) % 3];
                if constexpr (kPairRows<VEC, LIFE, CLIPPED>) {
                    // q - u is a multiple of kMRing (even), so m's parity is u - s's
                    if (((u - s) & 1) == 0) {
                        pair_sum<VEC>(C.h0, C.h1, B.h0, B.h1, pst[s - 1]);  // h(m) + h(m + 1)
#pragma unroll
                        for (int j = 0; j < VEC; ++j)
                            o.w[j] = rule_b3s23_pair(pst[s - 1].p0[j], pst[s - 1].p1[j], pst[s - 1].p2[j],
                                                     A.h0[j], A.h1[j], C.r[j]);
                    } else {  // h(m - 1) + h(m), formed by the even row before
#pragma unroll
                        for (int j = 0; j < VEC; ++j)
                            o.w[j] = rule_b3s23_pair(pst[s - 1].p0[j], pst[s - 1].p1[j], pst[s - 1].p2[j],
                                                     B.h0[j], B.h1[j], C.r[j]);
                    }
                } else {
                    rule_hg<VEC, LIFE, CLIPPED>(p, A, C, B, omask, o);
                }
                const bool own_row = m >= G && m < n_in - G;
                if constexpr (HASH) {
                    hash_row_lds<VEC, ILV>(kae[s], kao[s], o, odd_lane, hsum + (s - 1) * kNP * kWaveLanes);
                }
                if (s < G) {
                    arrive<VEC, CLIPPED, ILV, WR>(o, vis(m), cmask, hr[s][((u - s) % 3 + 3) % 3]);
                } else {
                    const int r = brow(m);
                    store_row<VEC>(p.nxt + (int64_t)r * p.pitch, own_row, p.wwords * 4, lcol, owns, o);
                }
            }
        };

#pragma unroll
        for (int t = 0; t < kHgPF; ++t) load_m(min(t, n_in - 1), in[t]);
        constexpr int kFill = (2 * G + kMRing - 1) / kMRing * kMRing;  // whole ring turns
        // The peeled fill is one long straight-line block; only the B3/S23
        // instances keep their rings in registers through it (the generic-rule
        // mux tree makes the scheduler spill), so they alone skip the dead
        // fill steps.
        int q_begin = 0;
        if constexpr (LIFE) {
            static_for<kFill>([&](auto Q) __attribute__((always_inline)) { row_step(Q.value, Q.value % kMRing, true); });
            q_begin = kFill;
        }
        for (int q0 = q_begin; q0 < n_in; q0 += kMRing) {
#pragma unroll
            for (int u = 0; u < kMRing; ++u) row_step(q0 + u, u, false);
        }
        if constexpr (HASH) {
#pragma unroll
            for (int s = 0; s < G; ++s) {
                HashAcc<VEC> h;
#pragma unroll
                for (int k = 0; k < kNP; ++k) {
                    h.a[k] = hsum[(s * kNP + k) * kWaveLanes];
                }
                acc[s] = hash_lane_total(h, col, owns);
            }
        }
    }
    if constexpr (HASH) {
        hash_flush_gens<G>(acc, p.hash_slots, lane, wave_in_wg);
    }
    clock_probe_end(p.clk, clk0);
}

// The horizontal-first kernel keeps three planes per ring row: at 16-byte
// lanes it needs 183-270 registers or spills (1-1.6 KB scratch per lane), so
// VEC = 4 (gol_set_tuning's words_per_lane = 4) runs the vertical-first
// kernel.  Its generic-rule and clipped instances deeper than
// kMaxGensVec4Generic spill and are neither built nor launched (gol_set_tuning
// in gol_capi.cpp refuses such a tuning).
template <int VEC, int G, bool LIFE, bool CLIPPED>
constexpr bool kBuilt = G == 1 || VEC <= 2 || (LIFE && !CLIPPED) || G <= kMaxGensVec4Generic;

template <int VEC, int G, bool LIFE, bool HASH, bool CLIPPED, int ILV>
hipError_t launch_one(const StepParams& p, int gx, int gy, hipStream_t st) {
    const dim3 grid(gx, gy), block(kWaveLanes * kWavesPerWG);
    if constexpr (G == 1) {
        return launch_kernel(step_kernel<VEC, LIFE, HASH, CLIPPED, ILV>, grid, block, st, p);
    } else if constexpr (!kBuilt<VEC, G, LIFE, CLIPPED>) {
        return hipErrorInvalidValue;
    } else if constexpr (VEC <= 2) {
        if constexpr (VEC == kWholeRowVec && G == kWholeRowGens && LIFE && !CLIPPED && ILV == 2) {
            if (p.whole_row)
                return launch_kernel(multistep_hg_kernel<VEC, G, LIFE, HASH, CLIPPED, ILV, true>, grid, block, st, p);
        }
        if (p.whole_row) return hipErrorInvalidValue;  // no whole-row instance (checked by the host layer)
        return launch_kernel(multistep_hg_kernel<VEC, G, LIFE, HASH, CLIPPED, ILV>, grid, block, st, p);
    } else {
        if (p.whole_row) return hipErrorInvalidValue;
        return launch_kernel(multistep_kernel<VEC, G, LIFE, HASH, CLIPPED, ILV>, grid, block, st, p);
    }
}

// Resident 256-thread workgroups per CU for a kernel instance (occupancy API).
template <int VEC, int G, bool LIFE, bool HASH, bool CLIPPED, int ILV>
int blocks_one() {
    auto query = [](auto kernel) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, kWaveLanes * kWavesPerWG, 0) != hipSuccess) {
            (void)hipGetLastError();  // the failed query's own status: reported as 0 (unknown), not left pending
            return 0;
        }
        return n;
    };
    if constexpr (G == 1) {
        return query(step_kernel<VEC, LIFE, HASH, CLIPPED, ILV>);
    } else if constexpr (!kBuilt<VEC, G, LIFE, CLIPPED>) {
        return 0;
    } else if constexpr (VEC <= 2) {
        return query(multistep_hg_kernel<VEC, G, LIFE, HASH, CLIPPED, ILV>);
    } else {
        return query(multistep_kernel<VEC, G, LIFE, HASH, CLIPPED, ILV>);
    }
}

// The instances a launch can select: clipped boards (generic rule, row-major
// words), tori (B3/S23 fast path or generic rule) in row-major or pair layout
// (even lane widths).  `F` is called with the instance's template arguments
// as std::integral_constant values.
template <int VEC, typename F>
auto dispatch_kind(bool life, bool hash, bool clipped, int ilv, F&& f) {
    using T = std::true_type;
    using N = std::false_type;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    if (clipped) return hash ? f(N{}, T{}, T{}, I1{}) : f(N{}, N{}, T{}, I1{});
    if constexpr (VEC % 2 == 0) {
        if (ilv == 2) {
            if (life) return hash ? f(T{}, T{}, N{}, I2{}) : f(T{}, N{}, N{}, I2{});
            return hash ? f(N{}, T{}, N{}, I2{}) : f(N{}, N{}, N{}, I2{});
        }
    }
    if (life) return hash ? f(T{}, T{}, N{}, I1{}) : f(T{}, N{}, N{}, I1{});
    return hash ? f(N{}, T{}, N{}, I1{}) : f(N{}, N{}, N{}, I1{});
}

template <int VEC, int G>
int blocks_variant(bool life, bool hash, bool clipped, int ilv) {
    if (VEC % ilv != 0) return 0;
    return dispatch_kind<VEC>(life, hash, clipped, ilv, [&](auto L, auto H, auto C, auto I) {
        return blocks_one<VEC, G, decltype(L)::value, decltype(H)::value, decltype(C)::value, decltype(I)::value>();
    });
}

template <int G>
int blocks_gens(int vec, bool life, bool hash, bool clipped, int ilv) {
    switch (vec) {
        case 4: return blocks_variant<4, G>(life, hash, clipped, ilv);
        case 2: return blocks_variant<2, G>(life, hash, clipped, ilv);
        default: return blocks_variant<1, G>(life, hash, clipped, ilv);
    }
}

template <int VEC, int G>
hipError_t launch_variant(const StepParams& p, bool life, bool hash, bool clipped, int ilv, int gx, int gy,
                          hipStream_t st) {
    if (VEC % ilv != 0) return hipErrorInvalidValue;  // checked by the host layer
    return dispatch_kind<VEC>(life, hash, clipped, ilv, [&](auto L, auto H, auto C, auto I) {
        return launch_one<VEC, G, decltype(L)::value, decltype(H)::value, decltype(C)::value, decltype(I)::value>(
            p, gx, gy, st);
    });
}

template <int G>
hipError_t launch_gens(const StepParams& p, int vec, bool life, bool hash, bool clipped, int ilv, int gx, int gy,
                       hipStream_t st) {
    switch (vec) {
        case 4: return launch_variant<4, G>(p, life, hash, clipped, ilv, gx, gy, st);
        case 2: return launch_variant<2, G>(p, life, hash, clipped, ilv, gx, gy, st);
        case 1: return launch_variant<1, G>(p, life, hash, clipped, ilv, gx, gy, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace dev

// Defined one per translation unit (gol_step_g<G>.hip).
hipError_t launch_step_g1(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g2(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g3(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g4(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g5(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g6(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g7(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g8(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g9(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g10(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g11(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
hipError_t launch_step_g12(const StepParams&, int, bool, bool, bool, int, int, int, hipStream_t);
int blocks_step_g1(int, bool, bool, bool, int);
int blocks_step_g2(int, bool, bool, bool, int);
int blocks_step_g3(int, bool, bool, bool, int);
int blocks_step_g4(int, bool, bool, bool, int);
int blocks_step_g5(int, bool, bool, bool, int);
int blocks_step_g6(int, bool, bool, bool, int);
int blocks_step_g7(int, bool, bool, bool, int);
int blocks_step_g8(int, bool, bool, bool, int);
int blocks_step_g9(int, bool, bool, bool, int);
int blocks_step_g10(int, bool, bool, bool, int);
int blocks_step_g11(int, bool, bool, bool, int);
int blocks_step_g12(int, bool, bool, bool, int);

}  // namespace gol
