// gol_schedule.cpp -- the pass schedule of a context: which kernel instance,
// lane width, band heights, tail split and XCD block order a pass of G
// generations launches with (automatic tuning, scripts/tune.py sweeps on
// MI355X, profiles/r01_* .. r04_*: results never depend on these choices),
// the launches of a pass (whole shard, or the interior and boundary rows of a
// sharded one) and the pass planner.  DESIGN.md section 4.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>
#include <functional>

#include "gol_ctx.h"


namespace {

constexpr int kDefaultXcdChunk = 8;

// Blocks per XCD chunk of the step kernels' block order (gol_stencil.h
// xcd_block).  GOL_XCD_CHUNK overrides (A/B experiments; 1 = dispatch order).
int xcd_chunk_env() {  // 0: not set
    static const int c = [] {
        const char* e = getenv("GOL_XCD_CHUNK");
        if (!e) return 0;
        const int v = atoi(e);
        return v < 1 ? 1 : (v > 64 ? 64 : v);
    }();
    return c;
}

// Multi-generation passes: kDefaultXcdChunk.  Single-generation passes (the
// 6-row band paths, whose seams are read by two bands at about the same time):
// four bands' blocks per XCD, so three of every four band seams stay in one
// XCD's L2.  Same-box sweep (profiles/r03_g1_xcd_chunk.txt, HBM fraction by
// kernel time, chunk 8 / 16 / 32 / 64): 262144^2 (8 blocks per band) 0.76-0.78
// / 0.79-0.80 / 0.80 / 0.75-0.77, 65536^2 (2 blocks per band) 0.75 / 0.75 /
// 0.73-0.75 / 0.72.
int xcd_chunk(int gens, int strips) {
    if (int c = xcd_chunk_env()) return c;
    if (gens != 1) return kDefaultXcdChunk;
    const int blocks_per_band = (strips + gol::kWavesPerWG - 1) / gol::kWavesPerWG;
    return std::min(64, std::max(kDefaultXcdChunk, 4 * blocks_per_band));
}

// Words per lane for a single-generation pass: 16-byte lane loads where the
// row fills whole waves of them.
int default_vec(int64_t wwords) {
    return (wwords % 4 == 0 && wwords >= 256) ? 4 : (wwords % 2 == 0 && wwords >= 128) ? 2 : 1;
}

// `resident`: waves the whole GPU holds at once for this kernel (0: unknown).
int pick_band(const gol_ctx* ctx, int64_t rows, int strips, int gens, int64_t resident) {
    if (ctx->band_rows > 0) return ctx->band_rows;
    // Single-generation passes: 6-row bands -- short streams, many in
    // flight, each band's 8 rows issued at once by step_kernel's straight-line
    // band path; the band seams (2 halo rows per 6) hit the caches.  Same-box
    // sweep with the band paths (profiles/r03_g1_band_heights.txt, HBM
    // fraction by kernel time, bands 4 / 6 / 8): 262144^2 0.738 / 0.774 /
    // 0.755, x 32768 0.734 / 0.762 / 0.749, 65536^2 0.752 / 0.760 / 0.753
    // (round 2, ring loop only: 4 rows best, profiles/r02_g1_band_sweep.txt).
    if (gens == 1) return 6;
    // Multi-generation passes recompute 2G halo rows per band: keep bands
    // >= 64 rows, aim at ~8192 waves, cap at 256 rows.
    const int64_t bands = std::max<int64_t>(1, 8192 / std::max(1, strips));
    int64_t band = (rows + bands - 1) / bands;
    band = std::max<int64_t>(band, 64);
    band = std::min<int64_t>(band, 256);
    // Wave quantization on wide boards: when a pass is only a few rounds of
    // resident waves, the last round is partly empty.  Model a pass as
    // ceil(waves / resident) rounds of (band + 2G) stream rows and shrink the
    // band (down to 60 %) when that fills the rounds better.  Measured on
    // the N = 8 per-rank shape (262144 x 32768, 1.7 rounds at band 256):
    // band 216 1.5-10 % faster on two boxes; with more rounds the effect is
    // within box-to-box noise (profiles/r01_band_quantization.txt).  Narrow
    // boards (< 32 strips) keep the plain choice (the model mispredicts 65536^2).
    // Narrow boards at 7- and 8-generation passes (4 waves per SIMD): 256-row
    // bands with the tail split below.  Same-box sweep at 65536^2, G = 8
    // (profiles/r02_band_sweep.txt): 0.0384 ms per generation vs 0.0405 for
    // the plain choice (137 rows, no tail) and 0.0471 for 256 rows without
    // the tail; at G = 6 the plain choice stays best.
    if (strips < 32 && gens >= 7 && resident > 0) return (int)std::min<int64_t>(256, std::max<int64_t>(rows, 1));
    // Wide boards at 7- to 12-generation passes, when the pass is many rounds
    // of resident waves: the tallest band (up to 1024 rows at G >= 10, 768
    // below) that still leaves >= 3.5 rounds, the tail split evening out the
    // end.  A band of B rows recomputes ~(G - 1) / B of its stage rows as
    // halo, so taller bands issue fewer VALU per cell.  Same-box sweep on the
    // bench's window (profiles/r03_band_262144.txt, 5 rounds, 262144^2,
    // passes 12 + 8): 1024 + 768 116.1k, 768 + 512 115.9k, 576 + 384 115.5k,
    // the previous 384 + ~256 114.4k GCUPS; on the N = 8 per-rank shape
    // (262144 x 32768, < 2 rounds) taller bands lost up to 6 %
    // (profiles/r03_band_32768.txt), so it keeps the rules below.
    if (strips >= 32 && gens >= 7 && resident > 0) {
        const int cap = gens >= 10 ? 1024 : 768;
        for (const int b : {1024, 768, 512}) {
            if (b > cap) continue;
            const int64_t waves = (rows + b - 1) / b * strips;
            if (2 * waves >= 7 * resident) return (int)std::min<int64_t>(b, std::max<int64_t>(rows, 1));
        }
    }
    // Wide boards at 10- to 12-generation passes (3 waves per SIMD, 2G halo
    // rows per band): 384-row bands when that is still >= 3 rounds of
    // resident waves, else 256, both with the tail split.  Same-box sweep at
    // G = 12 (profiles/r02_deep_band_sweep.txt, 4 rounds, ms per generation):
    // 262144^2 0.5660 (384) vs 0.5821 (the plain choice), x 131072 0.2882 vs
    // 0.2926, x 65536 0.1464 vs 0.1483, x 32768 0.0745 (256) vs 0.0761.
    if (strips >= 32 && gens >= 10 && resident > 0) {
        const int64_t waves384 = (rows + 383) / 384 * strips;
        return (int)std::min<int64_t>(waves384 >= 3 * resident ? 384 : 256, std::max<int64_t>(rows, 1));
    }
    if (resident > 0 && strips >= 32) {
        auto cost = [&](int64_t b) -> double {
            const int64_t waves = (rows + b - 1) / b * strips;
            return (double)((waves + resident - 1) / resident) * (double)(b + 2 * gens);
        };
        const int64_t full = (rows + band - 1) / band * strips;
        if (full >= resident && full <= 3 * resident) {
            int64_t best = band;
            double best_cost = cost(band);
            for (int64_t b = band - 1; b >= std::max<int64_t>(64, band * 6 / 10); --b) {
                const double c = cost(b);
                if (c < best_cost * 0.99) {
                    best = b;
                    best_cost = c;
                }
            }
            band = best;
        }
    }
    return (int)band;
}

// Small boards (round 6).  The rules above were measured on boards of
// >= 65536 columns and rows, where a pass is at least one round of resident
// waves.  On a small board they leave the GPU nearly empty -- a 4096^2 pass
// of G = 10 in 256-row bands is 2 strips x 16 bands = 32 waves, each
// streaming 276 rows through 10 stages one dependent instruction after the
// other (14.4 us per generation).  When the chosen band gives fewer waves than
// the GPU holds at once, the band is cut to about 1.5 rounds of resident waves
// (rows x strips / (1.5 resident), a multiple of 4, >= 4 rows), trading the
// taller bands' smaller halo share for parallelism.  Same-box sweep of depth x
// band (scripts/small_sweep.py, profiles/r06_small_sweep.txt, us per
// generation, unhashed): 4096^2 14.4 -> 2.3 at G = 10 in 4-row bands, 8192^2
// 14.4 -> 3.1-3.3, 16384^2 14.3 -> 5.3, 32768^2 18.1 -> 11.9; G = 10 stays the
// best depth (or within 3 % of it) at every size, hashed or not, so the
// planner plans hashed passes on these boards with the unhashed cost row
// (small_board below).  Returns the band, or 0 when the board fills the GPU
// (the rules above stand).
int small_board_band(const gol_ctx* ctx, int64_t rows, int strips, int gens, int band, int64_t resident) {
    if (ctx->band_rows > 0 || gens <= 1 || resident <= 0 || strips <= 0 || band <= 0) return 0;
    const int64_t waves = (rows + band - 1) / band * strips;
    if (waves >= resident) return 0;
    int64_t b = (2 * rows * strips + 3 * resident - 1) / (3 * resident);
    b = std::max<int64_t>((b + 3) / 4 * 4, 4);
    return (int)std::min<int64_t>(b, band);
}

// Tail split of a pass's rows (DESIGN.md §4 "Band schedule").  The
// dispatcher hands workgroups to CUs as slots free up, so a pass of a few
// rounds of resident waves ends with uneven per-SIMD tails: the CUs that got
// the last full-height bands finish late.  The last `frac` x resident waves
// therefore cover their rows in bands of band / div, dispatched after the
// bulk.  Default: one resident round's worth of waves in bands of band / 4
// for tall (>= 768-row) bands, band / 6 below.  Round 1 chose band / 3
// (profiles/r01_tail_sweep.txt: +4 % on the N = 8 per-rank shape 262144 x
// 32768, +2 % at x 65536, +1 % at x 131072 and 262144^2).  Round 6 re-swept
// the divisor on the paired G = 10 kernels, scored per probed GHz
// (scripts/band_scan.py, profiles/r06_tail/; tail1_* and tail2_* against /3,
// tail3_* against /4).  /4 over /3: 262144^2 (1024-row bands) +1.6 %, hashed
// +1.8 %; 65536^2 (256) +4.0 %; 262144^2 at G = 12 -0.3 %.  /6 over /4:
// 131072^2 (384) +2.4 %, 262144 x 32768 (256) +2.4 %, hashed +2.9 %,
// 262144 x 65536 (384) +0.2 %, 65536^2 -0.1 %, 262144^2 -3.6 %.
// GOL_TAIL="frac,div" overrides it (A/B sweeps); frac 0 disables it.
struct TailSplit {
    int32_t rows = 0;  // rows at the end of the range in short bands (0: none)
    int32_t band = 0;
};

constexpr double kTailFrac = 1.0;
constexpr int kTailDiv = 6;
constexpr int kTailDivTall = 4;  // bands of >= kTailTallBand rows
constexpr int kTailTallBand = 768;

TailSplit tail_split(const gol_ctx* ctx, int64_t rows, int strips, int band, int64_t resident, int gens) {
    double frac = kTailFrac;
    int div = band >= kTailTallBand ? kTailDivTall : kTailDiv;
    const char* env = getenv("GOL_TAIL");
    if (env && *env) {
        if (sscanf(env, "%lf,%d", &frac, &div) != 2) frac = 0.0;
    } else if (ctx->band_rows > 0) {
        return {};  // a fixed band (tuning) is taken literally
    }
    TailSplit t;
    // narrow boards (< 32 strips, e.g. 65536^2 with 17) measured neutral to
    // -3.6 % at G = 6 (profiles/r01_tail_sweep.txt, r01_band_sweep.txt): off
    // unless forced; at G >= 7 they take 256-row bands (pick_band), which need it
    if (frac <= 0.0 || div < 2 || resident <= 0 || strips <= 0 || (!env && strips < 32 && gens < 7)) return t;
    const int64_t waves = (rows + band - 1) / band * strips;
    if (waves <= resident) return t;  // a single round: nothing to even out
    const int b2 = std::max(8, band / div);
    int64_t trows = (int64_t)(frac * (double)resident / strips) * b2;
    trows = std::min<int64_t>(trows, rows / 2) / b2 * b2;
    if (trows <= 0) return t;
    t.rows = (int32_t)trows;
    t.band = b2;
    return t;
}

// Planned (not fixed) passes deeper than kMaxGensPlannedGeneric run only on
// the B3/S23 torus kernels: the generic-rule and clipped instances hold their
// rule masks / visibility planes in registers and drop to 2 waves per SIMD at
// G >= 10 (scripts/resource_usage.py), and the cost table is measured on the
// B3/S23 torus.
constexpr int kMaxGensPlannedGeneric = 8;

// Pass planner (DESIGN.md section 4 "Pass planner").  Relative time of one
// pass of G generations (G = 1..12, G = 6 -> 1), from scripts/depth_sweep.py
// (min of 3 rounds, reseeded board) on the row-pair-shared B3/S23 kernels
// (profiles/r04_pair_depth_sweep.txt; round 4).  Up to G = 6 a pass costs
// about the same (the sweep over the plane is HBM-bound); deeper passes cost
// more but less per generation.  The paired kernels hold 3 waves per SIMD up
// to G = 10 and 2 at G = 11 and 12 (rings of 174-197 VGPRs), so G = 10 is the
// cheapest per generation on both wide (>= 32 column strips) and narrow
// boards, unhashed and hashed, except narrow hashed boards where G = 7 ties it.
// Earlier rounds' per-row circuit tables: profiles/r01_depth_sweep.txt,
// r02_depth_sweep_deep.txt, r02_hash_deep_ab.txt.
constexpr double kPassCost[2][2][gol::kMaxGensPerPass + 1] = {
    // [hashed][wide]; G = 0 .. 12
    {{0, 0.755, 0.984, 0.995, 0.987, 0.964, 1.00, 1.068, 1.274, 1.346, 1.459, 1.893, 2.022},   // narrow (65536^2)
     {0, 0.739, 1.084, 1.088, 1.045, 1.020, 1.00, 1.073, 1.223, 1.340, 1.446, 1.696, 1.809}},  // wide (262144^2)
    {{0, 0.642, 0.846, 0.859, 0.880, 0.894, 1.00, 1.077, 1.353, 1.449, 1.553, 2.109, 2.256},   // narrow, hashed
     {0, 0.615, 0.904, 0.908, 0.883, 0.861, 1.00, 1.084, 1.278, 1.382, 1.496, 1.806, 1.941}}}; // wide, hashed

}  // namespace

namespace golc {

int ensure_slots(gol_ctx* ctx, uint32_t gens) {
    if (gens <= ctx->slots_gens) return GOL_OK;
    // one allocation for a whole gol_step chunk (1024 generations, 4 MiB):
    // a hipFree + hipMalloc between two hashed calls would synchronise the
    // device inside the caller's step
    gens = std::max<uint32_t>(gens, 1024);
    // the context forgets both buffers before freeing them, so a failure on
    // the way leaves nothing to free twice (destroy_impl frees what is set)
    ctx->slots_gens = 0;
    ctx->slots_clean = 0;
    unsigned long long* old_dev = ctx->slots;
    unsigned long long* old_host = ctx->host_folded;
    ctx->slots = ctx->host_folded = ctx->host_folded_dev = nullptr;
    if (old_dev) HIP_CHECK(ctx, hipFree(old_dev));
    if (old_host) HIP_CHECK(ctx, hipHostFree(old_host));
    HIP_CHECK(ctx, hipMalloc(&ctx->slots, (size_t)gens * gol::kHashGenStride * sizeof(unsigned long long)));
    // coherent: fold_kernel's stores reach host memory without a cache flush
    HIP_CHECK(ctx, hipHostMalloc((void**)&ctx->host_folded, (size_t)gens * sizeof(unsigned long long),
                                 hipHostMallocMapped | hipHostMallocCoherent));
    HIP_CHECK(ctx, hipHostGetDevicePointer((void**)&ctx->host_folded_dev, ctx->host_folded, 0));
    ctx->slots_gens = gens;  // only once every buffer exists
    return GOL_OK;
}

int clear_slots(gol_ctx* ctx, uint32_t gens) {
    const bool clean = ctx->slots_clean >= gens;
    ctx->slots_clean = 0;  // in use until read_hashes clears them again
    if (!clean)
        HIP_CHECK(ctx, hipMemsetAsync(ctx->slots, 0, (size_t)gens * gol::kHashGenStride * sizeof(unsigned long long),
                                      ctx->compute));
    return GOL_OK;
}

// Per call (scripts/tick_cost.py): a hashed step(1) on the 7 x 7 default
// board went from 22.0 us (memset + pass + 4 KiB readback) to 20.4 (pass +
// fold into mapped memory); configs[1]'s hashed 1000 generations from 1.96 to
// 1.72 ms (8 bytes per generation cross PCIe instead of 4 KiB).
int read_hashes(gol_ctx* ctx, uint32_t gens, uint64_t* out) {
    HIP_CHECK(ctx, gol::launch_fold(ctx->slots, gens, ctx->host_folded_dev, ctx->compute));
    HIP_CHECK(ctx, hipStreamSynchronize(ctx->compute));
    std::memcpy(out, ctx->host_folded, gens * sizeof(uint64_t));
    ctx->slots_clean = gens;
    return GOL_OK;
}

// Words per lane for a pass of `gens` generations.  Multi-generation strips
// carry 62 output lanes, so a row of w words needs ceil(w / (62 v)) strips;
// prefer 16-byte lanes unless 8-byte lanes waste clearly fewer lanes.
int lane_words(const gol_ctx* ctx, int gens) {
    // the pair layout needs whole pairs per lane: 8- or 16-byte lanes
    if (ctx->vec_fixed > 0) return std::max(ctx->vec_fixed, ctx->ilv);
    const int64_t w = ctx->wwords;
    if (gens == 1) return ctx->ilv == 2 ? std::max(default_vec(w), 2) : default_vec(w);
    // the horizontal-first kernel keeps 3 planes per ring row: 8-byte lanes
    // (95 VGPRs at G = 6, 5 waves/SIMD) beat 16-byte lanes (183 VGPRs, 2 waves;
    // those run the vertical-first kernel, +9 % at 262144^2 and +24 % at
    // 65536^2 for 8-byte horizontal-first lanes, profiles/r01_variant_ab.txt)
    const bool ok2 = w % 2 == 0 && w >= 2 * 62;
    return ok2 || ctx->ilv == 2 ? 2 : 1;
}

// Resident waves on the whole GPU for a launch (cached occupancy query).
int64_t resident_waves(const gol_ctx* ctx, int vec, int gens, bool life, bool hash, bool clipped) {
    const int key = ((((vec * 16 + gens) * 2 + (life ? 1 : 0)) * 2 + (hash ? 1 : 0)) * 2 + (clipped ? 1 : 0)) * 8 +
                    ctx->ilv;
    auto it = ctx->occupancy_cache.find(key);
    if (it != ctx->occupancy_cache.end()) return it->second;
    const int blocks = gol::resident_blocks_per_cu(vec, gens, life, hash, clipped, ctx->ilv);
    const int64_t waves = (int64_t)blocks * gol::kWavesPerWG * ctx->num_cus;
    ctx->occupancy_cache[key] = waves;
    return waves;
}

void preload_instances(gol_ctx* ctx) {
    const bool clipped = ctx->topology == GOL_REF_CLIPPED;
    const bool life = !clipped && ctx->birth == GOL_RULE_LIFE_BIRTH && ctx->survive == GOL_RULE_LIFE_SURVIVE;
    // unbuilt instances (16-byte generic / clipped lanes deeper than
    // kMaxGensVec4Generic, gol_stencil.h kBuilt) report 0 blocks without a load
    for (int G = 1; G <= gol::kMaxGensPerPass; ++G)
        for (int h = 0; h < 2; ++h) (void)resident_waves(ctx, lane_words(ctx, G), G, life, h != 0, clipped);
}

// Launch one pass of `gens` generations over local row ranges [lo0,hi0)
// (+ [lo1,hi1) if n == 2).  Only the main launch of a pass (whole shard, or
// the interior rows of a sharded shard) is bracketed by profiling events: it
// is the dominant kernel.
int launch_ranges(gol_ctx* ctx, int gens, const uint32_t* cur, uint32_t* nxt, const uint32_t* htop,
                  const uint32_t* hbot, int64_t halo_stride, bool wrap_y, unsigned long long* slots, int n,
                  const int32_t* lo, const int32_t* hi, int prof_kind, hipStream_t stream, const PlaneGeom* geom) {
    if (!stream) stream = ctx->compute;
    gol::StepParams p{};
    p.cur = cur;
    p.nxt = nxt;
    p.halo_top = htop;
    p.halo_bot = hbot;
    p.halo_stride = halo_stride;
    p.wrap_y = wrap_y ? 1 : 0;
    p.hash_slots = slots;
    p.pitch = ctx->pitch;
    p.grow0 = geom ? geom->grow0 : ctx->row0;
    p.vis_rows = ctx->topology == GOL_TORUS ? ctx->height : ctx->vis_h;
    p.vis_cols = ctx->topology == GOL_TORUS ? ctx->width : ctx->vis_w;
    p.width = ctx->width;
    p.wwords = ctx->wwords;
    p.rows = geom ? geom->rows : (int32_t)ctx->rows;
    const int vec = lane_words(ctx, gens);
    const bool clipped = ctx->topology == GOL_REF_CLIPPED;
    const bool life = !clipped && ctx->birth == GOL_RULE_LIFE_BIRTH && ctx->survive == GOL_RULE_LIFE_SURVIVE;
    p.whole_row = gol::whole_row_fits(vec, gens, life, clipped, ctx->ilv, ctx->topology == GOL_TORUS, ctx->wwords)
                      ? 1 : 0;
    const int sw = p.whole_row ? gol::kWaveLanes * vec : gol::strip_words(vec, gens);
    p.strips = (int32_t)((ctx->wwords + sw - 1) / sw);
    int64_t maxlen = 0;
    for (int k = 0; k < n; ++k) maxlen = std::max<int64_t>(maxlen, hi[k] - lo[k]);
    const int64_t resident = (n == 1 && gens > 1) ? resident_waves(ctx, vec, gens, life, slots != nullptr, clipped) : 0;
    int band = pick_band(ctx, maxlen, p.strips, gens, resident);
    const int small = n == 1 ? small_board_band(ctx, maxlen, p.strips, gens, band, resident) : 0;
    if (small > 0) band = small;
    int32_t rlo[2] = {0, 0}, rhi[2] = {0, 0}, rband[2] = {band, band};
    int nr = n;
    for (int k = 0; k < n; ++k) {
        rlo[k] = lo[k];
        rhi[k] = hi[k];
    }
    if (n == 1 && gens > 1 && small == 0) {  // a small board's pass is ~1.5 rounds: no tail to even out
        const TailSplit t = tail_split(ctx, hi[0] - lo[0], p.strips, band, resident, gens);
        if (t.rows > 0) {  // bulk [lo, hi - t.rows) in `band` rows, tail in t.band rows
            nr = 2;
            rhi[0] = hi[0] - t.rows;
            rlo[1] = rhi[0];
            rhi[1] = hi[0];
            rband[1] = t.band;
        }
    }
    int64_t waves = 0;
    for (int k = 0; k < 2; ++k) {
        p.row_lo[k] = rlo[k];
        p.row_hi[k] = rhi[k];
        p.band[k] = rband[k];
        p.nbands[k] = k < nr ? (rhi[k] - rlo[k] + rband[k] - 1) / rband[k] : 0;
        waves += (int64_t)p.nbands[k] * p.strips;
    }
    if (waves == 0) return GOL_OK;
    p.wrap_x = ctx->topology == GOL_TORUS ? 1 : 0;
    p.birth = ctx->birth;
    p.survive = ctx->survive;
    p.xcd_chunk = xcd_chunk(gens, p.strips);
    const int gx = (int)((waves + gol::kWavesPerWG - 1) / gol::kWavesPerWG);
    EventPair* ev = nullptr;
    p.clk = nullptr;
    if (ctx->prof && prof_kind != kProfNone) {
        ev = next_event_pair(ctx);
        if (!ev) return set_err(ctx, GOL_EHIP, "profiling event allocation failed");
        ev->kind = prof_kind;
        if (prof_kind == kProfMain && ctx->clk_buf && ctx->clk_used < kClockSlots) {
            ev->clk_slot = (int)ctx->clk_used++;
            p.clk = ctx->clk_buf + (size_t)ev->clk_slot * gol::kClockSlotWords;
        }
        HIP_CHECK(ctx, hipEventRecord(ev->start, stream));
    }
    HIP_CHECK(ctx, gol::launch_step(p, vec, gens, life, slots != nullptr, clipped, ctx->ilv, gx, 1, stream));
    if (ev) {
        HIP_CHECK(ctx, hipEventRecord(ev->stop, stream));
        if (prof_kind == kProfMain) ctx->prof_gens += (uint64_t)gens;
    }
    return GOL_OK;
}

// The interior rows [G, rows - G) of a sharded pass on the compute stream:
// they read no halo, so they are enqueued before the exchange (one_pass) and
// run while it is in flight.  Shards of <= 2G rows have no interior.  A
// missing neighbour (clipped board ends) reads dead rows: zero_row holds
// kMaxGensPerPass of them at the halo pitch.
int sharded_interior(gol_ctx* ctx, int G, unsigned long long* slots, bool has_up, bool has_down) {
    const int32_t rows = (int32_t)ctx->rows;
    if (rows <= 2 * G) return GOL_OK;
    const uint32_t* htop = has_up ? ctx->halo_top : ctx->zero_row;
    const uint32_t* hbot = has_down ? ctx->halo_bot : ctx->zero_row;
    const int32_t lo[1] = {G}, hi[1] = {rows - G};
    return launch_ranges(ctx, G, ctx->plane[ctx->cur], ctx->plane[ctx->cur ^ 1], htop, hbot, ctx->pitch, false, slots,
                         1, lo, hi, kProfMain);
}

// The rest of a sharded pass once every event in `halo_ready` has fired: the
// two boundary row blocks on the edge stream, or the whole shard when it has
// no interior.  The boundary launch runs concurrently with the tail of the
// interior one (its waves take the slots the interior's waves free) instead
// of after it; the compute stream then waits for it, so the next pass, a
// snapshot or a hash sees the whole plane.
int sharded_boundary(gol_ctx* ctx, int G, unsigned long long* slots, bool has_up, bool has_down,
                     const hipEvent_t* halo_ready, int nready) {
    uint32_t* cur = ctx->plane[ctx->cur];
    uint32_t* nxt = ctx->plane[ctx->cur ^ 1];
    const int32_t rows = (int32_t)ctx->rows;
    const int64_t pitch = ctx->pitch;
    const uint32_t* htop = has_up ? ctx->halo_top : ctx->zero_row;
    const uint32_t* hbot = has_down ? ctx->halo_bot : ctx->zero_row;
    if (rows > 2 * G) {
        // The exchange events follow this pass's ev_ready, recorded on the
        // compute stream after the previous pass's boundary rows: every
        // reader of the plane the boundary kernels overwrite has finished.
        for (int k = 0; k < nready; ++k) HIP_CHECK(ctx, hipStreamWaitEvent(ctx->edge, halo_ready[k], 0));
        const int32_t blo[2] = {0, rows - G}, bhi[2] = {G, rows};
        int rc = launch_ranges(ctx, G, cur, nxt, htop, hbot, pitch, false, slots, 2, blo, bhi, kProfBoundary,
                               ctx->edge);
        if (rc) return rc;
        HIP_CHECK(ctx, hipEventRecord(ctx->ev_edge, ctx->edge));
        HIP_CHECK(ctx, hipStreamWaitEvent(ctx->compute, ctx->ev_edge, 0));
        return GOL_OK;
    }
    for (int k = 0; k < nready; ++k) HIP_CHECK(ctx, hipStreamWaitEvent(ctx->compute, halo_ready[k], 0));
    const int32_t lo[1] = {0}, hi[1] = {rows};
    return launch_ranges(ctx, G, cur, nxt, htop, hbot, pitch, false, slots, 1, lo, hi, kProfMain);
}

// Kernels of one sharded pass whose halos are already on their way (the
// in-process group): the interior rows, then the boundary rows after
// `halo_ready`.
int sharded_pass_kernels(gol_ctx* ctx, int G, unsigned long long* slots, bool has_up, bool has_down,
                         const hipEvent_t* halo_ready, int nready) {
    if (int rc = sharded_interior(ctx, G, slots, has_up, has_down)) return rc;
    return sharded_boundary(ctx, G, slots, has_up, has_down, halo_ready, nready);
}

// Deepest pass the context may run.  Every shard of a ring must pick the
// same depths (their halo messages must match), so a sharded pass is capped
// by the smallest shard of the decomposition, floor(H / N) (a 1-rank ring
// sends G of its own rows: G <= H).
int depth_cap(const gol_ctx* ctx) {
    int64_t G = ctx->gens_per_pass > 0 ? ctx->gens_per_pass
                                       : (life_torus(ctx) ? gol::kMaxGensPerPass : kMaxGensPlannedGeneric);
    G = std::min<int64_t>(G, gol::kMaxGensPerPass);
    // 16-byte lanes (forced by tuning): the generic-rule / clipped instances
    // deeper than this spill and are not built (gol_set_tuning refuses them
    // as fixed depths with words_per_lane = 4)
    if (ctx->vec_fixed == 4 && !life_torus(ctx)) G = std::min<int64_t>(G, gol::kMaxGensVec4Generic);
    if (in_ring(ctx)) G = std::min<int64_t>(G, ctx->height / ctx->nranks);
    if (ctx->group) G = std::min<int64_t>(G, group_min_rows(ctx->group));
    return (int)std::max<int64_t>(G, 1);
}

// A B3/S23 torus stepped whole (no ring, no group) whose 10-generation
// passes fall under small_board_band.  There the hashed passes follow the
// unhashed cost row: the hashed narrow row (measured at 65536^2) ties G = 7
// with G = 10, but on small boards a launch costs nearly the same at any
// depth and G = 7 runs 1.4 x the launches.  Same-box sweep, 1000 generations,
// hashed, us per generation, G = 7 / 10 (scripts/small_depth.py,
// profiles/r06_small_depth.txt): 1024^2 2.99 / 2.72, 4096^2 3.27 / 2.96,
// 8192^2 5.15 / 4.08, 16384^2 6.97 / 7.08, 32768^2 15.33 / 15.33.
static bool small_board(const gol_ctx* ctx) {
    if (sharded(ctx) || ctx->group || !life_torus(ctx) || depth_cap(ctx) < 10) return false;
    const int G = 10;
    const int vec = lane_words(ctx, G);
    const int sw = gol::strip_words(vec, G);
    const int strips = (int)((ctx->wwords + sw - 1) / sw);
    const int64_t resident = resident_waves(ctx, vec, G, true, true, false);
    const int band = pick_band(ctx, ctx->rows, strips, G, resident);
    return small_board_band(ctx, ctx->rows, strips, G, band, resident) > 0;
}

// Depths of the passes that advance `n` generations.  A fixed
// gens_per_pass (tuning) is taken literally (the last pass shorter);
// otherwise the plan minimises the summed pass cost (a DP over n, n <= 1024:
// callers plan per chunk), deepest passes first (12 + 8 ran 3 % faster than
// 8 + 12 from the bench's fresh board with the per-row circuit,
// profiles/r02_plan_mix_ab.txt).
// Deterministic in (width, height, N, n), so all shards of a ring plan alike.
std::vector<int> plan_passes(const gol_ctx* ctx, uint32_t n, bool hashed) {
    const int cap = depth_cap(ctx);
    std::vector<int> plan;
    if (ctx->gens_per_pass > 0 || cap == 1) {
        for (uint32_t g = 0; g < n; g += plan.back()) plan.push_back((int)std::min<uint32_t>(cap, n - g));
        return plan;
    }
    const int sw = gol::strip_words(lane_words(ctx, 6), 6);
    const bool wide = (ctx->wwords + sw - 1) / sw >= 32;
    const double* cost = kPassCost[hashed && !small_board(ctx) ? 1 : 0][wide ? 1 : 0];
    std::vector<double> best(n + 1, 0.0);
    std::vector<int> pick(n + 1, 1);
    for (uint32_t k = 1; k <= n; ++k) {
        best[k] = 1e300;
        for (int G = 1; G <= cap && (uint32_t)G <= k; ++G) {
            const double c = best[k - G] + cost[G];
            if (c < best[k] - 1e-12) {
                best[k] = c;
                pick[k] = G;
            }
        }
    }
    for (uint32_t k = n; k > 0; k -= (uint32_t)pick[k]) plan.push_back(pick[k]);
    std::sort(plan.begin(), plan.end(), std::greater<int>());
    return plan;
}

}  // namespace golc
