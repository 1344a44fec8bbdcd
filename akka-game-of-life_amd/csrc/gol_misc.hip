// gol_misc.hip -- board seeding, standalone state hash, the cross-lane self
// test, and the launch dispatcher over pass depths.
#include <algorithm>

#include "gol_stencil.h"

namespace gol {

namespace {

typedef const __attribute__((address_space(4))) uint32_t* const_u32_ptr;

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// The pair layout (DESIGN.md "Data layout"; oracle/gol_oracle.c
// oracle_to_pairs): row-major words (w0, w1) = columns 0..31, 32..63 <->
// (e, o) = their even and odd columns.
__device__ __forceinline__ uint32_t even_bits(uint32_t x) {  // bits 0, 2, .., 30 -> 0 .. 15
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    x = (x | (x >> 8)) & 0x0000FFFFu;
    return x;
}
__device__ __forceinline__ uint32_t spread_bits(uint32_t x) {  // bits 0 .. 15 -> 0, 2, .., 30
    x &= 0x0000FFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

// Device word j of the pair whose row-major words are w[0..2).
__device__ __forceinline__ uint32_t device_word(const uint32_t* w, int j) {
    return even_bits(w[0] >> j) | (even_bits(w[1] >> j) << 16);
}
// Row-major word i of the pair whose device words are q[0..2).
__device__ __forceinline__ uint32_t row_major_word(const uint32_t* q, int i) {
    return spread_bits(q[0] >> (16 * i)) | (spread_bits(q[1] >> (16 * i)) << 1);
}

// oracle/gol_oracle.c oracle_seed_packed, on device: the seeded stand-in for
// BoardCreator.scala:23 (Random.nextBoolean() per cell).  On an interleaved
// layout each thread derives its device word from the row-major words of its
// pair.
__global__ void seed_kernel(uint32_t* plane, int64_t pitch, int32_t wwords, int64_t width, int64_t grow0,
                            int32_t rows, uint64_t seed, int ilv) {
    const int64_t total = (int64_t)rows * wwords;
    auto word = [&](int64_t r, int64_t c) -> uint32_t {
        const uint64_t i = (uint64_t)(grow0 + r) * (uint64_t)wwords + (uint64_t)c;
        const uint64_t z = splitmix64(seed + 0x9E3779B97F4A7C15ull * (i + 1));
        return (uint32_t)(z >> 32) & dev::col_mask(width, c);
    };
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = k / wwords, c = k % wwords;
        uint32_t w;
        if (ilv == 2) {
            const int64_t c0 = c - c % 2;
            const uint32_t g[2] = {word(r, c0), word(r, c0 + 1)};
            w = device_word(g, (int)(c % 2));
        } else {
            w = word(r, c);
        }
        plane[r * pitch + c] = w;
    }
}

// One thread per pair: row-major <-> device words.
__global__ void convert_kernel(const uint32_t* src, uint32_t* dst, int64_t pitch, int64_t dst_pitch, int32_t ngroups,
                               int32_t rows, int to_device) {
    const int64_t total = (int64_t)rows * ngroups;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = k / ngroups, c = 2 * (k % ngroups);
        const uint32_t in[2] = {src[r * pitch + c], src[r * pitch + c + 1]};
#pragma unroll
        for (int i = 0; i < 2; ++i) dst[r * dst_pitch + c + i] = to_device ? device_word(in, i) : row_major_word(in, i);
    }
}

// The state hash of `rows` rows: pair-layout words are
// the canonical words; a row-major word c is unzipped into its even and odd
// columns, the lower (c even) or upper (c odd) halves of its pair's E and O.
__global__ void hash_kernel(const uint32_t* plane, int64_t pitch, int32_t wwords, int64_t grow0, int32_t rows,
                            int ilv, unsigned long long* slots) {
    const int64_t total = (int64_t)rows * wwords;
    unsigned long long acc = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = k / wwords, c = k % wwords;
        const uint32_t ae = hash_row_key(grow0 + r), ao = ae + kHashOddAdd;
        const uint32_t w = plane[r * pitch + c];
        unsigned long long t;
        if (ilv == 2) {
            t = (unsigned long long)w * ((c & 1) ? ao : ae);
        } else {
            const uint32_t u = dev::unzip_bits(w);
            const uint32_t e = (c & 1) ? u << 16 : u & 0xFFFFu;
            const uint32_t o = (c & 1) ? u & 0xFFFF0000u : u >> 16;
            t = (unsigned long long)e * ae + (unsigned long long)o * ao;
        }
        acc += t * hash_pair_key((uint32_t)(c / 2));
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, kWaveLanes);
    if ((threadIdx.x & (kWaveLanes - 1)) == 0)
        atomicAdd(slots + (size_t)(blockIdx.x % kHashSlots) * kHashSlotStride, acc);
}

// out[0..63]    = dpp wave_shr:1 (old = 0xA0A0A0A0) of in[lane]
// out[64..127]  = dpp wave_shl:1 (old = 0xB0B0B0B0) of in[lane]
// out[128..191] = alignbit(in[lane], in[(lane+63)%64], 31)
// out[192..255] = in[5] via a wave-uniform scalar load
// One wave per generation g: lane k takes accumulator k and clears it, the
// wave sums them (mod 2^64) and lane 0 stores the sum to folded[g] -- mapped
// page-locked host memory, read by the host after the stream synchronises.
static_assert(kHashSlots == kWaveLanes, "one accumulator per lane");
__global__ __launch_bounds__(kWaveLanes) void fold_kernel(unsigned long long* slots, uint32_t gens,
                                                          unsigned long long* folded) {
    const uint32_t g = blockIdx.x;
    const int lane = threadIdx.x;
    unsigned long long* a = slots + (size_t)g * kHashGenStride + (size_t)lane * kHashSlotStride;
    unsigned long long h = *a;
    *a = 0ull;  // the slots are left clear for the next hashed pass (ctx->slots_clean)
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) h += __shfl_xor(h, off, kWaveLanes);
    if (lane == 0) folded[g] = h;  // vector store
}

__global__ void selftest_kernel(const uint32_t* in, uint32_t* out) {
    const int lane = threadIdx.x;
    const uint32_t v = in[lane];
    out[lane] = dev::dpp_shr1(0xA0A0A0A0u, v);
    out[64 + lane] = dev::dpp_shl1(0xB0B0B0B0u, v);
    out[128 + lane] = __builtin_amdgcn_alignbit(v, in[(lane + 63) % 64], 31);
    out[192 + lane] = ((const_u32_ptr)in)[5];
}

}  // namespace

int strip_words(int vec, int gens) { return (gens == 1 ? kWaveLanes : kWaveLanes - 2) * vec; }

hipError_t launch_step(const StepParams& p, int vec, int gens, bool life, bool hash, bool clipped, int ilv,
                       int grid_x, int grid_y, hipStream_t stream) {
    switch (gens) {
        case 1: return launch_step_g1(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 2: return launch_step_g2(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 3: return launch_step_g3(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 4: return launch_step_g4(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 5: return launch_step_g5(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 6: return launch_step_g6(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 7: return launch_step_g7(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 8: return launch_step_g8(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 9: return launch_step_g9(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 10: return launch_step_g10(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 11: return launch_step_g11(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        case 12: return launch_step_g12(p, vec, life, hash, clipped, ilv, grid_x, grid_y, stream);
        default: return hipErrorInvalidValue;
    }
}

int resident_blocks_per_cu(int vec, int gens, bool life, bool hash, bool clipped, int ilv) {
    switch (gens) {
        case 1: return blocks_step_g1(vec, life, hash, clipped, ilv);
        case 2: return blocks_step_g2(vec, life, hash, clipped, ilv);
        case 3: return blocks_step_g3(vec, life, hash, clipped, ilv);
        case 4: return blocks_step_g4(vec, life, hash, clipped, ilv);
        case 5: return blocks_step_g5(vec, life, hash, clipped, ilv);
        case 6: return blocks_step_g6(vec, life, hash, clipped, ilv);
        case 7: return blocks_step_g7(vec, life, hash, clipped, ilv);
        case 8: return blocks_step_g8(vec, life, hash, clipped, ilv);
        case 9: return blocks_step_g9(vec, life, hash, clipped, ilv);
        case 10: return blocks_step_g10(vec, life, hash, clipped, ilv);
        case 11: return blocks_step_g11(vec, life, hash, clipped, ilv);
        case 12: return blocks_step_g12(vec, life, hash, clipped, ilv);
        default: return 0;
    }
}

hipError_t launch_seed(uint32_t* plane, int64_t pitch, int32_t wwords, int64_t width, int64_t grow0, int32_t rows,
                       uint64_t seed, int ilv, hipStream_t stream) {
    if (ilv != 1 && ilv != 2) return hipErrorInvalidValue;
    const int64_t total = (int64_t)rows * wwords;
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 8192));
    return launch_kernel(seed_kernel, dim3(blocks), dim3(256), stream, plane, pitch, wwords, width, grow0, rows, seed,
                         ilv);
}

hipError_t launch_convert(const uint32_t* src, uint32_t* dst, int64_t pitch, int32_t wwords, int32_t rows,
                          bool to_device, int ilv, hipStream_t stream, int64_t dst_pitch) {
    if (dst_pitch <= 0) dst_pitch = pitch;
    if (ilv != 2 || wwords % 2 != 0) return hipErrorInvalidValue;
    const int64_t total = (int64_t)rows * (wwords / 2);
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 8192));
    return launch_kernel(convert_kernel, dim3(blocks), dim3(256), stream, src, dst, pitch, dst_pitch, wwords / 2,
                         rows, to_device ? 1 : 0);
}

hipError_t launch_hash(const uint32_t* plane, int64_t pitch, int32_t wwords, int64_t grow0, int32_t rows, int ilv,
                       unsigned long long* slots, hipStream_t stream) {
    const int64_t total = (int64_t)rows * wwords;
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 4096));
    if (ilv != 1 && ilv != 2) return hipErrorInvalidValue;
    return launch_kernel(hash_kernel, dim3(blocks), dim3(256), stream, plane, pitch, wwords, grow0, rows, ilv,
                         slots);
}

hipError_t launch_fold(unsigned long long* slots, uint32_t gens, unsigned long long* folded, hipStream_t stream) {
    if (gens == 0) return hipSuccess;
    return launch_kernel(fold_kernel, dim3(gens), dim3(kWaveLanes), stream, slots, gens, folded);
}

hipError_t launch_selftest(const uint32_t* in, uint32_t* out, hipStream_t stream) {
    return launch_kernel(selftest_kernel, dim3(1), dim3(64), stream, in, out);
}

}  // namespace gol
