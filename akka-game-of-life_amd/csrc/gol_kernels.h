// gol_kernels.h -- internal interface between the C-ABI host layer
// (gol_capi.cpp and the units gol_ctx.h lists) and the gfx950 kernels
// (gol_stencil.h, gol_step_g<G>.hip, gol_misc.hip).  Not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <tuple>
#include <type_traits>
#include <utility>

namespace gol {

constexpr int kWaveLanes = 64;   // CDNA wavefront
#ifndef GOL_WAVES_PER_WG
#define GOL_WAVES_PER_WG 4
#endif
constexpr int kWavesPerWG = GOL_WAVES_PER_WG;  // waves per workgroup (256-thread workgroups)
constexpr int kHashSlots = 64;   // sharded hash accumulators (one cache line each)
constexpr int kHashSlotStride = 8;  // u64 per slot => 64 B apart
constexpr int kHashGenStride = kHashSlots * kHashSlotStride;  // u64 per generation
constexpr int kMaxGensPerPass = 12;  // temporal blocking depth supported by the kernels
// Deepest pass of the 16-byte-lane (words_per_lane = 4) generic-rule and
// clipped instances that keeps every variable in registers: deeper ones spill
// (448-640 B of scratch per lane), so they are not built (gol_stencil.h
// kBuilt) and gol_set_tuning / the planner never ask for them.
constexpr int kMaxGensVec4Generic = 7;

// State hash keys (oracle/gol_oracle.c
// oracle_hash_packed, oracle/oracle.py np_hash).  The hash is a function of
// the cells alone: the canonical words E (even columns) and O (odd columns)
// of column group g = columns 64g .. 64g + 63 of global row y contribute
// (E * A(y, 0) + O * A(y, 1)) * B(g) mod 2^64 -- on the pair layout exactly
// the device words, elsewhere their unzipped row-major words.
//   A(y, 0) = ((t ^ (t >> 15)) << 1) | 1,  t = y * kHashRowMul (mod 2^32)
//   A(y, 1) = A(y, 0) + kHashOddAdd        (even: stays odd)
//   B(g)    = murmur3 fmix32(g + kHashPairAdd) | 1
// Both keys odd, so a single-word change always changes the sum.
constexpr uint32_t kHashRowMul = 0x9E3779B1u;
constexpr uint32_t kHashOddAdd = 0x6A09E666u;
constexpr uint32_t kHashPairAdd = 0x7F4A7C15u;

// Launch `kernel` and return the status of this launch alone.
// hipLaunchKernel returns it directly; hipGetLastError() after a
// triple-chevron launch would instead report -- and clear -- whatever status
// an earlier call of this thread left pending (DESIGN.md section 2 "HIP
// status discipline").  The arguments are converted to the kernel's parameter
// types first, as a direct call would.
template <typename... KArgs, typename... Args>
hipError_t launch_kernel(void (*kernel)(KArgs...), dim3 grid, dim3 block, hipStream_t stream, Args&&... args) {
    static_assert(sizeof...(KArgs) == sizeof...(Args), "kernel argument count");
    std::tuple<std::remove_cv_t<KArgs>...> vals(std::forward<Args>(args)...);
    return std::apply(
        [&](auto&... v) {
            void* argv[] = {static_cast<void*>(&v)...};
            return hipLaunchKernel(reinterpret_cast<const void*>(kernel), grid, block, argv, 0, stream);
        },
        vals);
}

__host__ __device__ __forceinline__ uint32_t hash_row_key(int64_t y) {
    const uint32_t t = (uint32_t)y * kHashRowMul;
    return ((t ^ (t >> 15)) << 1) | 1u;
}

__host__ __device__ __forceinline__ uint32_t hash_pair_key(uint32_t k) {
    uint32_t h = k + kHashPairAdd;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h | 1u;
}

// One launch advances G generations (G = `gens`, 1..kMaxGensPerPass) over up
// to two local row ranges, each cut into bands of its own height: the whole
// shard (one range, or a bulk range plus a tail of shorter bands), or the two
// boundary row blocks of a sharded pass.  Waves are numbered range 0's bands
// first, then range 1's (the order the dispatcher hands them out).
struct StepParams {
    const uint32_t* cur;       // local row 0 of the current plane
    uint32_t* nxt;             // local row 0 of the next plane
    const uint32_t* halo_top;  // rows -G .. -1 (halo_stride apart)
    const uint32_t* halo_bot;  // rows rows .. rows+G-1
    unsigned long long* hash_slots;  // G * kHashGenStride u64, or null
    int64_t pitch;             // words between rows (multiple of 64)
    int64_t grow0;             // global row of local row 0
    int64_t vis_rows;          // global rows [0, vis_rows) are visible (clipped)
    int64_t vis_cols;          // columns [0, vis_cols) are visible (clipped)
    int64_t width;             // cells per row
    int32_t wwords;            // words per row = ceil(width / 32)
    int32_t rows;              // local rows
    int32_t row_lo[2];
    int32_t row_hi[2];
    int32_t nbands[2];
    int32_t band[2];           // output rows streamed by one wave, per range
    int32_t strips;            // column strips per row
    int32_t wrap_x;            // torus in x
    int32_t wrap_y;            // unsharded torus: local rows wrap modulo `rows`
    int32_t whole_row;         // one strip = the whole torus row (kWholeRow*: wave-rotate neighbours, no halo lanes)
    int64_t halo_stride;       // words between halo rows (0: one row repeated)
    uint32_t birth;
    uint32_t survive;
    int32_t xcd_chunk;         // consecutive blocks kept on one XCD (gol_stencil.h xcd_block; <= 1: off)
    unsigned long long* clk;   // launch clock probe slot (kClockSlotWords u64), or null (gol_stencil.h clock_probe_*)
};

// Per launch: kClockSubSlots sub-slots one 64-B line apart, each summing
// core-clock ticks and 100 MHz reference ticks of the sampled workgroups.
constexpr int kClockSubSlots = 64;
constexpr int kClockSubWords = 8;
constexpr int kClockSampleEvery = 4;
constexpr int kClockSlotWords = kClockSubSlots * kClockSubWords;

// Strip geometry of a launch: words covered per wave.
int strip_words(int vec, int gens);

// Whole-row waves: a B3/S23 torus in the pair layout whose row is exactly one
// wave of 2-word lanes (64 pairs, 4096 columns -- BASELINE.json configs[1])
// runs its kWholeRowGens-deep passes as one strip without halo lanes: the
// lane-edge words come from a wave rotate, so every lane is an output lane
// and the row takes one wave per band instead of two (62 + 2 pairs).
constexpr int kWholeRowGens = 10;
constexpr int kWholeRowVec = 2;
inline bool whole_row_fits(int vec, int gens, bool life, bool clipped, int ilv, bool torus, int64_t wwords) {
    return torus && life && !clipped && ilv == 2 && vec == kWholeRowVec && gens == kWholeRowGens &&
           wwords == (int64_t)kWaveLanes * kWholeRowVec;
}

// vec: words per lane (1, 2 or 4); gens: generations per pass; life: B3/S23
// fast path (torus only); hash: fuse the per-generation state hash; clipped:
// reference geometry; ilv: the plane's interleave (1 row-major, 2 pairs;
// vec a multiple of it).  Multi-generation passes at vec <= 2 run the
// horizontal-first kernel, at vec = 4 the vertical-first one.
hipError_t launch_step(const StepParams& p, int vec, int gens, bool life, bool hash, bool clipped, int ilv,
                       int grid_x, int grid_y, hipStream_t stream);

// Resident 256-thread workgroups per CU of the step kernel instance a launch
// with these parameters uses (hipOccupancyMaxActiveBlocksPerMultiprocessor);
// 0 if unknown.
int resident_blocks_per_cu(int vec, int gens, bool life, bool hash, bool clipped, int ilv);

// Seeded board in the device layout (ilv: words per interleave group).
hipError_t launch_seed(uint32_t* plane, int64_t pitch, int32_t wwords, int64_t width,
                       int64_t grow0, int32_t rows, uint64_t seed, int ilv, hipStream_t stream);

// Row-major words <-> pair-interleaved words (ilv 2), `rows` rows of `wwords`
// (even) words, `pitch` words apart in the source and `dst_pitch` (<= 0:
// `pitch`) in the destination (src != dst).
hipError_t launch_convert(const uint32_t* src, uint32_t* dst, int64_t pitch, int32_t wwords, int32_t rows,
                          bool to_device, int ilv, hipStream_t stream, int64_t dst_pitch = 0);

// Partial state hash of `rows` device rows of interleave `ilv` (1 or 2).
hipError_t launch_hash(const uint32_t* plane, int64_t pitch, int32_t wwords, int64_t grow0,
                       int32_t rows, int ilv, unsigned long long* slots, hipStream_t stream);

// folded[g] = sum of generation g's hash accumulators, g < gens, which it
// clears; `folded` may be mapped host memory (8 bytes per generation cross
// PCIe instead of the 4 KiB of accumulators).
hipError_t launch_fold(unsigned long long* slots, uint32_t gens, unsigned long long* folded, hipStream_t stream);

// DPP / lane-shift self test: out[64*4] (see gol_selftest in gol_capi.cpp).
hipError_t launch_selftest(const uint32_t* in, uint32_t* out, hipStream_t stream);

}  // namespace gol
