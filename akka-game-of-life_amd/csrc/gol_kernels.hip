// gol_kernels.hip -- gfx950 (CDNA4) kernels for the Life-like generation step.
//
// Replaces the reference's per-cell actor computation:
//   NextStateCellGathererActor.scala:32-36  ask <=8 neighbours GetStateFromEpoch
//   NextStateCellGathererActor.scala:39-46  gather, count, apply rule, commit e+1
//   package.scala:17-28                     the clipped Moore neighbourhood
// with one streaming stencil over a bit-packed board (DESIGN.md "Kernels").
//
// Work decomposition: each wave64 owns one column strip (64 lanes x VEC words
// = 64*VEC*32 cells) of one band of `band` rows and streams down (or up: odd
// bands run bottom-up so band seams are read by both neighbours at the same
// time and the second read hits the Infinity Cache) through the band keeping
// a ring of PF+3 rows in registers.  Every input word is loaded from HBM once
// per generation (plus 2 halo rows per band), every output word stored once.
//
// Per lane and row: one 4/8/16-byte coalesced load; the bit to the left of the
// lane's first word and to the right of its last word come from the
// neighbouring lanes via DPP wave_shr:1 / wave_shl:1 on the column sums, and
// at the strip's edges from two wave-uniform scalar (SMEM) loads.
//
// Neighbour count: vertical full adder (a + c + b) per column -> two bit
// planes, funnel shifts (v_alignbit) to the left/right columns, then a
// bit-sliced adder gives the 3x3 box sum T9 (4 bit planes).  B3/S23 is
// "T9 == 3 | (alive & T9 == 4)"; the generic (birth, survive) path subtracts
// the centre and evaluates the masks with a v_bfi mux tree.
#include "gol_kernels.h"

namespace gol {

namespace {

constexpr int kPF = 2;               // rows prefetched ahead of the compute row
constexpr int kRing = kPF + 3;       // register ring: rows r-1, r, r+1 + kPF ahead
constexpr int kDppWaveShr1 = 0x138;  // lane i <- lane i-1 (lane 0 keeps `old`)
constexpr int kDppWaveShl1 = 0x130;  // lane i <- lane i+1 (lane 63 keeps `old`)

typedef const __attribute__((address_space(4))) uint32_t* const_u32_ptr;

__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    return (m & a) | (~m & b);
}

// Wave-uniform scalar load (s_load_dword through the constant address space;
// the current plane is read-only for the whole launch).
__device__ __forceinline__ uint32_t sload(const uint32_t* p, int64_t idx) {
    return ((const_u32_ptr)p)[idx];
}

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, kDppWaveShr1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_shl1(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, kDppWaveShl1, 0xf, 0xf, false);
}

// Bits [0, limit) of word `w` set (limit in cells).
__device__ __forceinline__ uint32_t col_mask(int64_t limit, int64_t w) {
    const int64_t lo = w * 32;
    if (lo + 32 <= limit) return 0xFFFFFFFFu;
    if (lo >= limit) return 0u;
    return (uint32_t)((1ull << (limit - lo)) - 1ull);
}

template <int VEC>
struct Words {
    uint32_t w[VEC];
};

// Unconditional load: lanes past the strip's end read a clamped in-row
// address (their results are never stored and never reach an active lane),
// so no exec-masked branch separates the load from its use and the
// compiler keeps the prefetch ring in flight.
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

template <int VEC>
__device__ __forceinline__ void store_words(uint32_t* rp, int col, bool active, const Words<VEC>& d) {
    if (active) {
        if constexpr (VEC == 4) {
            *reinterpret_cast<uint4*>(rp + col) = make_uint4(d.w[0], d.w[1], d.w[2], d.w[3]);
        } else if constexpr (VEC == 2) {
            *reinterpret_cast<uint2*>(rp + col) = make_uint2(d.w[0], d.w[1]);
        } else {
            rp[col] = d.w[0];
        }
    }
}

// Per-wave constant state.
template <int VEC>
struct StripCtx {
    int lane, col, lcolumn, nact;  // lcolumn: clamped load column
    bool active;
    int64_t lcol, rcol;   // edge words (left of the strip, right of the strip)
    bool lvalid, rvalid;
    uint32_t cmask[VEC];  // clipped: visible-column masks of the lane's words
    uint32_t omask[VEC];  // clipped: in-board masks of the lane's words
    uint32_t lmask, rmask;  // clipped: visible masks of the edge words
};

template <int VEC, bool LIFE, bool CLIPPED>
__device__ __forceinline__ void compute_row(const StepParams& p, const StripCtx<VEC>& s,
                                            const Words<VEC>& A, const Words<VEC>& C,
                                            const Words<VEC>& B, uint32_t aL, uint32_t cL,
                                            uint32_t bL, uint32_t aR, uint32_t cR, uint32_t bR,
                                            bool va, bool vc, bool vb, Words<VEC>& out) {
    uint32_t a[VEC], c[VEC], b[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        if constexpr (CLIPPED) {
            a[j] = va ? (A.w[j] & s.cmask[j]) : 0u;
            c[j] = vc ? (C.w[j] & s.cmask[j]) : 0u;
            b[j] = vb ? (B.w[j] & s.cmask[j]) : 0u;
        } else {
            a[j] = A.w[j]; c[j] = C.w[j]; b[j] = B.w[j];
        }
    }
    if constexpr (CLIPPED) {
        aL = va ? (aL & s.lmask) : 0u; cL = vc ? (cL & s.lmask) : 0u; bL = vb ? (bL & s.lmask) : 0u;
        aR = va ? (aR & s.rmask) : 0u; cR = vc ? (cR & s.rmask) : 0u; bR = vb ? (bR & s.rmask) : 0u;
    }
    // Vertical 3-sums (v1 v0) = a + c + b per column.
    uint32_t v0[VEC], v1[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        const uint32_t t = a[j] ^ c[j];
        v0[j] = t ^ b[j];
        v1[j] = bfi(t, b[j], a[j]);
    }
    // Strip-edge column sums (wave-uniform, scalar ALU).
    const uint32_t tl = aL ^ cL, tr = aR ^ cR;
    const uint32_t ev0L = tl ^ bL, ev1L = bfi(tl, bL, aL);
    const uint32_t ev0R = tr ^ bR, ev1R = bfi(tr, bR, aR);
    // Column sums of the word left of word 0 and right of word VEC-1.
    const uint32_t m0 = dpp_shr1(ev0L, v0[VEC - 1]);
    const uint32_t m1 = dpp_shr1(ev1L, v1[VEC - 1]);
    uint32_t n0 = dpp_shl1(ev0R, v0[0]);
    uint32_t n1 = dpp_shl1(ev1R, v1[0]);
    if (s.nact < kWaveLanes) {  // narrow strip: the last active lane is not lane 63
        const bool last = s.lane == s.nact - 1;
        n0 = last ? ev0R : n0;
        n1 = last ? ev1R : n1;
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        const uint32_t p0 = j == 0 ? m0 : v0[j - 1];
        const uint32_t p1 = j == 0 ? m1 : v1[j - 1];
        const uint32_t q0 = j == VEC - 1 ? n0 : v0[j + 1];
        const uint32_t q1 = j == VEC - 1 ? n1 : v1[j + 1];
        const uint32_t w0 = __builtin_amdgcn_alignbit(v0[j], p0, 31);  // column x-1
        const uint32_t e0 = __builtin_amdgcn_alignbit(q0, v0[j], 1);   // column x+1
        const uint32_t w1 = __builtin_amdgcn_alignbit(v1[j], p1, 31);
        const uint32_t e1 = __builtin_amdgcn_alignbit(q1, v1[j], 1);
        // T9 = (w1 w0) + (v1 v0) + (e1 e0) = s3 s2 s1 s0
        const uint32_t t0 = w0 ^ v0[j];
        const uint32_t s0 = t0 ^ e0;
        const uint32_t c0 = bfi(t0, e0, w0);
        const uint32_t t1 = w1 ^ v1[j];
        const uint32_t pp = t1 ^ e1;
        const uint32_t qq = bfi(t1, e1, w1);
        const uint32_t s1 = pp ^ c0;
        const uint32_t r2 = pp & c0;
        const uint32_t s2 = qq ^ r2;
        const uint32_t alive = C.w[j];
        uint32_t res;
        if constexpr (LIFE) {
            // T9 mod 8 == 3, or alive and T9 mod 8 == 4 (T9 in {8,9} maps to {0,1}).
            res = bfi(s2, alive & ~(s1 | s0), s1 & s0);
        } else {
            const uint32_t s3 = qq & r2;
            // n = T9 - visible centre (a 1-bit borrow chain).
            const uint32_t cv = c[j];
            const uint32_t n0b = s0 ^ cv, b0 = cv & ~s0;
            const uint32_t n1b = s1 ^ b0, b1 = b0 & ~s1;
            const uint32_t n2b = s2 ^ b1, b2 = b1 & ~s2;
            const uint32_t n3b = s3 ^ b2;
            uint32_t L[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const uint32_t sm = ((p.survive >> k) & 1u) ? 0xFFFFFFFFu : 0u;
                const uint32_t bm = ((p.birth >> k) & 1u) ? 0xFFFFFFFFu : 0u;
                L[k] = bfi(alive, sm, bm);
            }
            const uint32_t m01 = bfi(n0b, L[1], L[0]), m23 = bfi(n0b, L[3], L[2]);
            const uint32_t m45 = bfi(n0b, L[5], L[4]), m67 = bfi(n0b, L[7], L[6]);
            const uint32_t m03 = bfi(n1b, m23, m01), m47 = bfi(n1b, m67, m45);
            const uint32_t m07 = bfi(n2b, m47, m03);
            res = bfi(n3b, L[8], m07);
        }
        if constexpr (CLIPPED) res &= s.omask[j];
        out.w[j] = res;
    }
}

template <int VEC, bool LIFE, bool HASH, bool CLIPPED>
__global__ __launch_bounds__(kWaveLanes* kWavesPerWG) void step_kernel(const StepParams p) {
    const int lane = threadIdx.x & (kWaveLanes - 1);
    const int wave_in_wg = __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveLanes);
    const int wave = blockIdx.x * kWavesPerWG + wave_in_wg;
    const int rg = blockIdx.y;
    const int strip = wave % p.strips;
    const int bandi = wave / p.strips;
    const bool wave_valid = bandi < p.nbands[rg];
    unsigned long long acc = 0;

    if (wave_valid) {
        StripCtx<VEC> s;
        s.lane = lane;
        const int r_begin = p.row_lo[rg] + bandi * p.band;
        const int r_end = min(r_begin + p.band, p.row_hi[rg]);
        const int nrows = r_end - r_begin;
        const int s0 = strip * (kWaveLanes * VEC);
        s.nact = min(kWaveLanes, (p.wwords - s0) / VEC);
        s.col = s0 + lane * VEC;
        s.active = lane < s.nact;
        s.lcolumn = s.active ? s.col : s0;
        // Edge words; an edge outside a clipped board is loaded from a
        // clamped in-row index and masked to zero (lmask/rmask).
        s.lcol = s0 - 1;
        s.lvalid = true;
        if (s.lcol < 0) {
            s.lvalid = p.wrap_x != 0;
            s.lcol = p.wwords - 1;
        }
        s.rcol = s0 + s.nact * VEC;
        s.rvalid = true;
        if (s.rcol >= p.wwords) {
            s.rvalid = p.wrap_x != 0;
            s.rcol = 0;
        }
        if constexpr (CLIPPED) {
#pragma unroll
            for (int j = 0; j < VEC; ++j) {
                s.cmask[j] = col_mask(p.vis_cols, s.col + j);
                s.omask[j] = col_mask(p.width, s.col + j);
            }
            s.lmask = s.lvalid ? col_mask(p.vis_cols, s.lcol) : 0u;
            s.rmask = s.rvalid ? col_mask(p.vis_cols, s.rcol) : 0u;
        }
        // Odd bands stream bottom-up (boustrophedon): both neighbours of a
        // band seam read it at the same time.
        const bool up = (bandi & 1) != 0;
        // t-th row of the stream (t = 0 .. nrows+1) and i-th output row.
        auto row_of = [&](int t) -> int { return up ? r_end - t : r_begin - 1 + t; };
        auto out_of = [&](int i) -> int { return up ? r_end - 1 - i : r_begin + i; };
        auto row_ptr = [&](int r) -> const uint32_t* {
            return r < 0 ? p.halo_top : (r >= p.rows ? p.halo_bot : p.cur + (int64_t)r * p.pitch);
        };
        auto row_vis = [&](int r) -> bool {
            if constexpr (CLIPPED) {
                const int64_t g = p.grow0 + r;
                return g >= 0 && g < p.vis_rows;
            } else {
                return true;
            }
        };

        Words<VEC> ring[kRing];
        uint32_t eL[kRing], eR[kRing];
        auto load_t = [&](int t, Words<VEC>& d, uint32_t& el, uint32_t& er) {
            const uint32_t* rp = row_ptr(row_of(t));
            load_words<VEC>(rp, s.lcolumn, d);
            el = sload(rp, s.lcol);
            er = sload(rp, s.rcol);
        };

        // Hash: global word index g = (grow0 + r) * wwords + col + j (mod 2^32).
        uint32_t lk1[VEC], lk2[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            lk1[j] = (uint32_t)(s.col + j) * kHashK1;
            lk2[j] = (uint32_t)(s.col + j) * kHashK2;
        }

        auto emit = [&](int i, const Words<VEC>& o) {
            const int r = out_of(i);
            store_words<VEC>(p.nxt + (int64_t)r * p.pitch, s.col, s.active, o);
            if constexpr (HASH) {
                const uint32_t gb = (uint32_t)((uint64_t)(p.grow0 + r) * (uint64_t)p.wwords);
                const uint32_t rb1 = gb * kHashK1, rb2 = gb * kHashK2;
#pragma unroll
                for (int j = 0; j < VEC; ++j) {
                    const uint32_t k1 = rb1 + lk1[j];
                    const uint32_t k2 = (rb2 + lk2[j]) | 1u;
                    acc += (unsigned long long)(o.w[j] ^ k1) * (unsigned long long)k2;
                }
            }
        };

        auto step_i = [&](int i, int u, bool in_band) {
            // slots of rows t = i, i+1, i+2 are u, u+1, u+2 (mod kRing)
            Words<VEC> o;
            const int ua = u % kRing, uc = (u + 1) % kRing, ub = (u + 2) % kRing;
            compute_row<VEC, LIFE, CLIPPED>(p, s, ring[ua], ring[uc], ring[ub], eL[ua], eL[uc],
                                            eL[ub], eR[ua], eR[uc], eR[ub], row_vis(row_of(i)),
                                            row_vis(row_of(i + 1)), row_vis(row_of(i + 2)), o);
            if (in_band) emit(i, o);
        };

        // Loads are never predicated: stream rows past the band's last one
        // are clamped to it (an L2 hit), and steps past the band compute
        // into the void (their stores are skipped).  The loop body is then
        // straight-line, so the compiler's counted vmcnt waits keep kPF rows
        // in flight.
        const int tmax = nrows + 1;
#pragma unroll
        for (int t = 0; t < kRing - 1; ++t) load_t(min(t, tmax), ring[t], eL[t], eR[t]);
        for (int i0 = 0; i0 < nrows; i0 += kRing) {
#pragma unroll
            for (int u = 0; u < kRing; ++u) {
                const int i = i0 + u;
                const int sl = (u + kRing - 1) % kRing;
                load_t(min(i + kRing - 1, tmax), ring[sl], eL[sl], eR[sl]);
                step_i(i, u, i < nrows);
            }
        }
        if (!s.active) acc = 0;
    }

    if constexpr (HASH) {
        // wave reduce -> workgroup reduce -> one atomic per workgroup into a sharded slot
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, kWaveLanes);
        __shared__ unsigned long long part[kWavesPerWG];
        if (lane == 0) part[wave_in_wg] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long t = 0;
#pragma unroll
            for (int w = 0; w < kWavesPerWG; ++w) t += part[w];
            atomicAdd(p.hash_slots + (size_t)((blockIdx.x + blockIdx.y) % kHashSlots) * kHashSlotStride, t);
        }
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// oracle/gol_oracle.c oracle_seed_packed, on device.
__global__ void seed_kernel(uint32_t* plane, int64_t pitch, int32_t wwords, int64_t width,
                            int64_t grow0, int32_t rows, uint64_t seed) {
    const int64_t total = (int64_t)rows * wwords;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = k / wwords, c = k % wwords;
        const uint64_t i = (uint64_t)(grow0 + r) * (uint64_t)wwords + (uint64_t)c;
        const uint64_t z = splitmix64(seed + 0x9E3779B97F4A7C15ull * (i + 1));
        plane[r * pitch + c] = (uint32_t)(z >> 32) & col_mask(width, c);
    }
}

__global__ void hash_kernel(const uint32_t* plane, int64_t pitch, int32_t wwords, int64_t grow0,
                            int32_t rows, unsigned long long* slots) {
    const int64_t total = (int64_t)rows * wwords;
    unsigned long long acc = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = k / wwords, c = k % wwords;
        const uint32_t g = (uint32_t)((uint64_t)(grow0 + r) * (uint64_t)wwords + (uint64_t)c);
        acc += (unsigned long long)(plane[r * pitch + c] ^ (g * kHashK1)) *
               (unsigned long long)((g * kHashK2) | 1u);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, kWaveLanes);
    if ((threadIdx.x & (kWaveLanes - 1)) == 0)
        atomicAdd(slots + (size_t)(blockIdx.x % kHashSlots) * kHashSlotStride, acc);
}

// out[0..63]   = dpp_shr1(old=0xA0A0A0A0, in[lane])
// out[64..127] = dpp_shl1(old=0xB0B0B0B0, in[lane])
// out[128..191]= alignbit(in[lane], in[(lane+63)%64], 31)
// out[192..255]= sload(in, 5) (wave-uniform scalar load)
__global__ void selftest_kernel(const uint32_t* in, uint32_t* out) {
    const int lane = threadIdx.x;
    const uint32_t v = in[lane];
    out[lane] = dpp_shr1(0xA0A0A0A0u, v);
    out[64 + lane] = dpp_shl1(0xB0B0B0B0u, v);
    out[128 + lane] = __builtin_amdgcn_alignbit(v, in[(lane + 63) % 64], 31);
    out[192 + lane] = sload(in, 5);
}

template <int VEC, bool LIFE, bool HASH, bool CLIPPED>
hipError_t launch_t(const StepParams& p, int gx, int gy, hipStream_t st) {
    hipLaunchKernelGGL((step_kernel<VEC, LIFE, HASH, CLIPPED>), dim3(gx, gy), dim3(kWaveLanes * kWavesPerWG),
                       0, st, p);
    return hipGetLastError();
}

template <int VEC>
hipError_t launch_v(const StepParams& p, bool life, bool hash, bool clipped, int gx, int gy, hipStream_t st) {
    if (clipped) {
        return hash ? launch_t<VEC, false, true, true>(p, gx, gy, st)
                    : launch_t<VEC, false, false, true>(p, gx, gy, st);
    }
    if (life) {
        return hash ? launch_t<VEC, true, true, false>(p, gx, gy, st)
                    : launch_t<VEC, true, false, false>(p, gx, gy, st);
    }
    return hash ? launch_t<VEC, false, true, false>(p, gx, gy, st)
                : launch_t<VEC, false, false, false>(p, gx, gy, st);
}

}  // namespace

hipError_t launch_step(const StepParams& p, int vec, bool life, bool hash, bool clipped, int grid_x,
                       int grid_y, hipStream_t stream) {
    switch (vec) {
        case 4: return launch_v<4>(p, life, hash, clipped, grid_x, grid_y, stream);
        case 2: return launch_v<2>(p, life, hash, clipped, grid_x, grid_y, stream);
        case 1: return launch_v<1>(p, life, hash, clipped, grid_x, grid_y, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_seed(uint32_t* plane, int64_t pitch, int32_t wwords, int64_t width, int64_t grow0,
                       int32_t rows, uint64_t seed, hipStream_t stream) {
    const int64_t total = (int64_t)rows * wwords;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(seed_kernel, dim3(blocks), dim3(256), 0, stream, plane, pitch, wwords, width, grow0,
                       rows, seed);
    return hipGetLastError();
}

hipError_t launch_hash(const uint32_t* plane, int64_t pitch, int32_t wwords, int64_t grow0, int32_t rows,
                       unsigned long long* slots, hipStream_t stream) {
    const int64_t total = (int64_t)rows * wwords;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(hash_kernel, dim3(blocks), dim3(256), 0, stream, plane, pitch, wwords, grow0, rows,
                       slots);
    return hipGetLastError();
}

hipError_t launch_selftest(const uint32_t* in, uint32_t* out, hipStream_t stream) {
    hipLaunchKernelGGL(selftest_kernel, dim3(1), dim3(64), 0, stream, in, out);
    return hipGetLastError();
}

}  // namespace gol
