// gol_capi.cpp -- C ABI of libgol (include/gol.h): shard contexts, device
// planes, the per-generation schedule (interior || RCCL halo exchange, then
// boundary rows), hashing, snapshots, checkpoints and kernel timing.
//
// Reference correspondence (src/main/scala/gameoflife/ of the reference):
//   gol_create   <- BoardCreator.createAllInitialActors (BoardCreator.scala:79-89)
//   gol_seed     <- initialState = Random.nextBoolean() per cell (BoardCreator.scala:23)
//   gol_step     <- NextStep tick -> CurrentEpochMsg -> gatherer -> SetNewStateMsg
//                   (BoardCreator.scala:113-116, CellActor.scala:63-91,
//                    NextStateCellGathererActor.scala:25-48)
//   gol_snapshot <- CellStateMsg -> LoggerActor (CellActor.scala:89, LoggerActor.scala:30-46)
//   gol_comm_*   <- cross-backend GetStateFromEpoch/StateForEpoch over Akka remote
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gol.h"
#include "gol_kernels.h"

namespace {

std::mutex g_err_mu;
std::string g_err;  // process-wide last error (gol_create failures)

// What a profiled event pair brackets (gol_profile_stats).
enum ProfKind { kProfNone = -1, kProfMain = 0, kProfExchange = 1, kProfBoundary = 2 };

struct EventPair {
    hipEvent_t start = nullptr, stop = nullptr;
    int clk_slot = -1;  // this launch's clock-probe slot (gol_stencil.h clock_probe_*), or -1
    int kind = kProfMain;
    int ref = -1;       // exchange / boundary pairs: index of the same pass's interior pair (this fold window)
};

// Clock-probe slots per context (one per profiled launch between folds).
constexpr uint32_t kClockSlots = 1024;  // 4 KiB each

}  // namespace

// In-process shard group: shards in row order, linked into a ring (torus) or
// a chain (clipped); each shard's comm stream pulls its neighbours' edge rows.
struct gol_group {
    std::vector<gol_ctx*> shards;
    bool torus = true;
    std::string err;
};

struct LoopRing;

struct gol_ctx {
    // geometry
    int64_t width = 0, height = 0, row0 = 0, rows = 0;
    int32_t wwords = 0;
    int64_t pitch = 0;
    int32_t topology = GOL_TORUS;
    uint32_t birth = 0, survive = 0;
    int64_t vis_w = 0, vis_h = 0;
    int ilv = 1;         // device words per interleave group: 1 row-major, 2 pairs
    int device = 0;
    int vec_fixed = 0;  // words per lane forced by gol_set_tuning (0: per-pass automatic)
    // device state
    uint32_t* plane[2] = {nullptr, nullptr};
    int cur = 0;
    uint32_t* halo_top = nullptr;  // RCCL receive buffers (sharded)
    uint32_t* halo_bot = nullptr;
    uint32_t* zero_row = nullptr;
    unsigned long long* slots = nullptr;  // [gens][kHashSlots * kHashSlotStride]
    uint32_t slots_gens = 0;
    std::vector<unsigned long long> host_slots;
    uint64_t epoch = 0;
    hipStream_t compute = nullptr, comm = nullptr;
    hipStream_t edge = nullptr;  // boundary-row kernels of a sharded pass (concurrent with the interior)
    hipEvent_t ev_ready = nullptr, ev_halo = nullptr, ev_edge = nullptr;
    // asynchronous snapshot (gol_snapshot_async / gol_snapshot_wait): the
    // board at the snapshot epoch, row-major, copied to the host on `xfer`
    // while later passes run on `compute`
    uint32_t* snap = nullptr;
    hipStream_t xfer = nullptr;
    hipEvent_t ev_snap_ready = nullptr, ev_snap_done = nullptr;
    bool snap_pending = false;
    uint64_t snap_epoch = 0;
    // RCCL
    ncclComm_t nccl = nullptr;
    int rank = 0, nranks = 1;
    // loopback ring (gol_comm_init_loopback): the same halo exchange between
    // contexts of one process, for tests; exclusive with nccl
    std::shared_ptr<LoopRing> loop;
    // in-process shard group (gol_group_*): halos by device-to-device copies
    gol_group* group = nullptr;
    int gindex = 0;
    // tuning
    int32_t band_rows = 0;                                   // 0: automatic
    int32_t gens_per_pass = 0;                               // temporal blocking depth (0: automatic)
    // profiling
    bool prof = false;
    std::vector<EventPair> evs;
    size_t evs_used = 0;
    double prof_ms = 0.0;
    uint64_t prof_launches = 0;
    uint64_t prof_gens = 0;  // generations covered by the profiled launches
    unsigned long long* clk_buf = nullptr;  // kClockSlots x kClockSlotWords u64 (device)
    uint32_t clk_used = 0;                  // slots handed out since the last fold
    double prof_clk_ms_ghz = 0.0, prof_clk_ms = 0.0;  // time-weighted probe clock
    double prof_xchg_ms = 0.0, prof_bnd_ms = 0.0;     // halo exchanges (comm stream), boundary launches (edge)
    double prof_xchg_exposed_ms = 0.0, prof_tail_ms = 0.0;  // ... how far they end after the interior launch
    uint64_t prof_xchg = 0, prof_bnd = 0;
    uint64_t halo_sent = 0, halo_recv = 0;             // bytes posted to the ring since the last reset
    // occupancy
    int num_cus = 0;
    std::map<int, int64_t> occupancy_cache;
    std::string err;
};

namespace {

int set_err(gol_ctx* ctx, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) {
        ctx->err = buf;
    } else {
        std::lock_guard<std::mutex> lk(g_err_mu);
        g_err = buf;
    }
    return code;
}

// HIP status discipline: a failing HIP call also
// leaves its status pending on the calling thread (hipGetLastError).  A
// failure libgol reports through its own return code is taken off the
// thread here, so no later call -- ours or the caller's -- inherits it.
int hip_fail(gol_ctx* ctx, hipError_t e, const char* expr, const char* file, int line) {
    (void)hipGetLastError();
    return set_err(ctx, GOL_EHIP, "%s failed: %s (%s:%d)", expr, hipGetErrorString(e), file, line);
}

#define HIP_CHECK(ctx, expr)                                                   \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) return hip_fail((ctx), e_, #expr, __FILE__, __LINE__); \
    } while (0)

// A status whose failure only gets logged (teardown, best-effort calls):
// reported on stderr and taken off the thread.
void hip_note(hipError_t e, const char* what) {
    if (e == hipSuccess) return;
    (void)hipGetLastError();
    fprintf(stderr, "libgol: %s: %s (%d)\n", what, hipGetErrorString(e), (int)e);
}

// RCCL runs HIP calls of its own on the calling thread and does not take the
// statuses it discards off the thread.  After every RCCL call libgol makes,
// such a leftover is taken here -- where it arose -- counted, and logged once
// per (call, status) pair, so it can neither be pinned on a later launch
// nor reach the caller.  gol_diag_absorbed reports the count.
std::mutex g_absorb_mu;
uint64_t g_absorbed = 0;
std::string g_absorbed_last;
std::map<std::string, int> g_absorb_seen;

// `pending_before`: the thread's status before the RCCL call
// (hipPeekAtLastError).  If the caller had left one pending, whatever is
// pending now may be the caller's own: it is left in place, not taken, counted
// or attributed to RCCL.
void absorb_rccl_status(const char* call, hipError_t pending_before) {
    if (pending_before != hipSuccess) return;
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return;
    char msg[256];
    snprintf(msg, sizeof msg, "%s left HIP status %s (%d) on the calling thread", call, hipGetErrorString(e), (int)e);
    std::lock_guard<std::mutex> lk(g_absorb_mu);
    ++g_absorbed;
    g_absorbed_last = msg;
    if (g_absorb_seen[msg]++ == 0) fprintf(stderr, "libgol: %s (absorbed)\n", msg);
}

#define NCCL_CHECK(ctx, expr)                                                                       \
    do {                                                                                            \
        const hipError_t pre_ = hipPeekAtLastError();                                               \
        ncclResult_t r_ = (expr);                                                                   \
        absorb_rccl_status(#expr, pre_);                                                            \
        if (r_ != ncclSuccess)                                                                      \
            return set_err((ctx), GOL_ECOMM, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(r_), \
                           __FILE__, __LINE__);                                                     \
    } while (0)

int64_t group_min_rows(const gol_group* g);
size_t group_size(const gol_group* g);

// Any attached communicator runs the ring schedule, a 1-rank one included: its
// up and down neighbours are the rank itself, so the torus halo rows go out
// and come back through ncclSend / ncclRecv to self (the "self-ring" -- the
// RCCL path exercised bit-exactly on a one-GPU box).
bool sharded(const gol_ctx* c) {
    return c->nccl != nullptr || c->loop != nullptr || (c->group != nullptr && group_size(c->group) > 1);
}

bool in_ring(const gol_ctx* c) { return c->nccl != nullptr || c->loop != nullptr; }

// The B3/S23 torus: the only boards the fast-path kernel instances serve.
bool life_torus(const gol_ctx* c) {
    return c->topology == GOL_TORUS && c->birth == GOL_RULE_LIFE_BIRTH && c->survive == GOL_RULE_LIFE_SURVIVE;
}

int bind(gol_ctx* ctx) {
    HIP_CHECK(ctx, hipSetDevice(ctx->device));
    return GOL_OK;
}

int ensure_slots(gol_ctx* ctx, uint32_t gens) {
    if (gens <= ctx->slots_gens) return GOL_OK;
    // one allocation for a whole gol_step chunk (1024 generations, 4 MiB):
    // a hipFree + hipMalloc between two hashed calls would synchronise the
    // device inside the caller's step
    gens = std::max<uint32_t>(gens, 1024);
    if (ctx->slots) HIP_CHECK(ctx, hipFree(ctx->slots));
    ctx->slots = nullptr;
    const size_t n = (size_t)gens * gol::kHashSlots * gol::kHashSlotStride;
    HIP_CHECK(ctx, hipMalloc(&ctx->slots, n * sizeof(unsigned long long)));
    ctx->slots_gens = gens;
    ctx->host_slots.resize(n);
    return GOL_OK;
}

// Sum the kHashSlots accumulators of each generation (mod 2^64).
void fold_slots(const gol_ctx* ctx, uint32_t gens, uint64_t* out) {
    for (uint32_t g = 0; g < gens; ++g) {
        uint64_t h = 0;
        const unsigned long long* s =
            ctx->host_slots.data() + (size_t)g * gol::kHashSlots * gol::kHashSlotStride;
        for (int k = 0; k < gol::kHashSlots; ++k) h += s[(size_t)k * gol::kHashSlotStride];
        out[g] = h;
    }
}

EventPair* next_event_pair(gol_ctx* ctx);

// Clock one launch ran at, from its probe slot (gol_stencil.h
// clock_probe_*): core-clock ticks over 100 MHz reference ticks, summed over
// the launch's workgroups.
double slot_clock_ghz(const unsigned long long* w) {
    unsigned long long mt = 0, rt = 0;
    for (int k = 0; k < gol::kClockSubSlots; ++k) {
        mt += w[k * gol::kClockSubWords + 0];
        rt += w[k * gol::kClockSubWords + 1];
    }
    return rt ? (double)mt / (double)rt * 0.1 : 0.0;
}

int fold_profile(gol_ctx* ctx) {
    std::vector<float> times(ctx->evs_used, 0.f);
    for (size_t i = 0; i < ctx->evs_used; ++i) {
        HIP_CHECK(ctx, hipEventSynchronize(ctx->evs[i].stop));
        HIP_CHECK(ctx, hipEventElapsedTime(&times[i], ctx->evs[i].start, ctx->evs[i].stop));
    }
    // every probed launch has finished (its stop event fired): read the slots
    std::vector<unsigned long long> clk;
    if (ctx->clk_used > 0) {
        clk.resize((size_t)ctx->clk_used * gol::kClockSlotWords);
        HIP_CHECK(ctx, hipMemcpy(clk.data(), ctx->clk_buf, clk.size() * sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost));
    }
    for (size_t i = 0; i < ctx->evs_used; ++i) {
        const float ms = times[i];
        const int kind = ctx->evs[i].kind, ref = ctx->evs[i].ref;
        // exposed part: how long after its pass's interior launch this ended
        float after = 0.f;
        if ((kind == kProfExchange || kind == kProfBoundary) && ref >= 0 && (size_t)ref < i) {
            HIP_CHECK(ctx, hipEventElapsedTime(&after, ctx->evs[ref].stop, ctx->evs[i].stop));
            after = std::max(after, 0.f);
        }
        if (kind == kProfExchange) {
            ctx->prof_xchg_ms += ms;
            ctx->prof_xchg += 1;
            ctx->prof_xchg_exposed_ms += after;
            continue;
        }
        if (kind == kProfBoundary) {
            ctx->prof_bnd_ms += ms;
            ctx->prof_bnd += 1;
            ctx->prof_tail_ms += after;
            continue;
        }
        ctx->prof_ms += ms;
        ctx->prof_launches += 1;
        const int slot = ctx->evs[i].clk_slot;
        if (slot >= 0 && (size_t)slot < (size_t)ctx->clk_used) {
            const double ghz = slot_clock_ghz(clk.data() + (size_t)slot * gol::kClockSlotWords);
            if (ghz > 0.0) {
                ctx->prof_clk_ms_ghz += ghz * ms;
                ctx->prof_clk_ms += ms;
            }
        }
        ctx->evs[i].clk_slot = -1;
    }
    ctx->evs_used = 0;
    if (ctx->clk_used > 0) {
        HIP_CHECK(ctx, hipMemsetAsync(ctx->clk_buf, 0,
                                      (size_t)ctx->clk_used * gol::kClockSlotWords * sizeof(unsigned long long),
                                      ctx->compute));
        HIP_CHECK(ctx, hipStreamSynchronize(ctx->compute));
        ctx->clk_used = 0;
    }
    return GOL_OK;
}

EventPair* next_event_pair(gol_ctx* ctx) {
    constexpr size_t kMaxPairs = 4096;
    if (ctx->evs_used == ctx->evs.size()) {
        if (ctx->evs.size() >= kMaxPairs) {
            if (fold_profile(ctx) != GOL_OK) return nullptr;
        } else {
            EventPair e;
            if (hipEventCreate(&e.start) != hipSuccess || hipEventCreate(&e.stop) != hipSuccess) {
                (void)hipGetLastError();  // reported by the caller as GOL_EHIP
                if (e.start) hip_note(hipEventDestroy(e.start), "hipEventDestroy");
                return nullptr;
            }
            ctx->evs.push_back(e);
        }
    }
    EventPair* ev = &ctx->evs[ctx->evs_used++];
    ev->kind = kProfMain;
    ev->clk_slot = -1;
    ev->ref = -1;
    return ev;
}

// Automatic tuning (scripts/tune.py sweeps on MI355X, profiles/r01_*):
// results never depend on these choices.

// Device layout of a board: words per interleave
// group.  Tori keep their columns interleaved so the stencil needs fewer
// funnel shifts: pairs (one v_alignbit and one DPP move per word and
// generation) where a row holds whole pairs; every other board stays
// row-major (any width).  A function of the geometry alone -- no setting or
// environment variable changes it -- and invisible at the boundary: host
// buffers are row-major and the state hash reads the cells through canonical
// words (section 5), so the same board hashes alike in either layout.
int device_ilv(int32_t topology, int64_t wwords) {
    if (topology != GOL_TORUS) return 1;
    return wwords % 2 == 0 ? 2 : 1;
}

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

// Tail split of a pass's rows (DESIGN.md §4 "Band schedule").  The
// dispatcher hands workgroups to CUs as slots free up, so a pass of a few
// rounds of resident waves ends with uneven per-SIMD tails: the CUs that got
// the last full-height bands finish late.  The last `frac` x resident waves
// therefore cover their rows in bands of band / div, dispatched after the
// bulk.  Default: one resident round's worth of waves in bands of band / 3
// (profiles/r01_tail_sweep.txt, reseeded boards, min of 4 rounds: +4 % on the
// N = 8 per-rank shape 262144 x 32768, +2 % at x 65536, +1 % at x 131072 and
// 262144^2; neutral to -3.6 % at 65536^2, so boards of < 32 strips keep one
// band height).  GOL_TAIL="frac,div" overrides it (A/B
// sweeps, scripts/tail_sweep.py); frac 0 disables it.
struct TailSplit {
    int32_t rows = 0;  // rows at the end of the range in short bands (0: none)
    int32_t band = 0;
};

constexpr double kTailFrac = 1.0;
constexpr int kTailDiv = 3;

TailSplit tail_split(const gol_ctx* ctx, int64_t rows, int strips, int band, int64_t resident, int gens) {
    double frac = kTailFrac;
    int div = kTailDiv;
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

// Resident waves on the whole GPU for a launch (cached occupancy query).
int64_t resident_waves(gol_ctx* ctx, int vec, int gens, bool life, bool hash, bool clipped) {
    const int key = ((((vec * 16 + gens) * 2 + (life ? 1 : 0)) * 2 + (hash ? 1 : 0)) * 2 + (clipped ? 1 : 0)) * 8 +
                    ctx->ilv;
    auto it = ctx->occupancy_cache.find(key);
    if (it != ctx->occupancy_cache.end()) return it->second;
    const int blocks = gol::resident_blocks_per_cu(vec, gens, life, hash, clipped, ctx->ilv);
    const int64_t waves = (int64_t)blocks * gol::kWavesPerWG * ctx->num_cus;
    ctx->occupancy_cache[key] = waves;
    return waves;
}

// Rows of the plane a launch steps and the global row of its local row 0:
// the context's own (default), or gol_replay's extended block.
struct PlaneGeom {
    int32_t rows;
    int64_t grow0;
};

// Launch one pass of `gens` generations over local row ranges [lo0,hi0)
// (+ [lo1,hi1) if n == 2).  Only the main launch of a pass (whole shard, or
// the interior rows of a sharded shard) is bracketed by profiling events: it
// is the dominant kernel.
int launch_ranges(gol_ctx* ctx, int gens, const uint32_t* cur, uint32_t* nxt, const uint32_t* htop,
                  const uint32_t* hbot, int64_t halo_stride, bool wrap_y, unsigned long long* slots, int n,
                  const int32_t* lo, const int32_t* hi, int prof_kind, hipStream_t stream = nullptr,
                  const PlaneGeom* geom = nullptr) {
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
    const int sw = gol::strip_words(vec, gens);
    p.strips = (int32_t)((ctx->wwords + sw - 1) / sw);
    int64_t maxlen = 0;
    for (int k = 0; k < n; ++k) maxlen = std::max<int64_t>(maxlen, hi[k] - lo[k]);
    const bool clipped = ctx->topology == GOL_REF_CLIPPED;
    const bool life = !clipped && ctx->birth == GOL_RULE_LIFE_BIRTH && ctx->survive == GOL_RULE_LIFE_SURVIVE;
    const int64_t resident = (n == 1 && gens > 1) ? resident_waves(ctx, vec, gens, life, slots != nullptr, clipped) : 0;
    const int band = pick_band(ctx, maxlen, p.strips, gens, resident);
    int32_t rlo[2] = {0, 0}, rhi[2] = {0, 0}, rband[2] = {band, band};
    int nr = n;
    for (int k = 0; k < n; ++k) {
        rlo[k] = lo[k];
        rhi[k] = hi[k];
    }
    if (n == 1 && gens > 1) {
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

// One point-to-point operation of a pass's halo exchange: send `count`
// words from `buf` to rank `peer`, or receive them into `buf` from it.
struct HaloOp {
    bool send;
    uint32_t* buf;
    size_t count;
    int peer;
};

}  // namespace

// Loopback ring (gol_comm_init_loopback): contexts of one process -- one host
// thread each, like one process per GPU -- joined under a key run libgol's
// exact halo op list with ncclSend / ncclRecv semantics: operations between a
// (sender, receiver) pair match in FIFO order of issue, and a rank's group
// completes when all its operations have matched.  A matched pair is a
// device-to-device copy on the receiver's comm stream, ordered after the
// sender's plane was final (an event on the sender's comm stream) and before
// the sender's stream goes on (an event the sender's comm stream waits for),
// as an RCCL send / recv pair is.  Test transport: the product path is RCCL.
// A ring fails when a rank times out waiting for a peer, leaves it, or
// mismatches an all-reduce: every waiting and later operation of the other
// ranks then returns GOL_ECOMM at once instead of waiting out its timeout,
// and its key cannot be joined again while members still hold it.
struct LoopRing {
    std::mutex mu;
    std::condition_variable cv;
    int nranks = 0;
    int joined = 0;
    std::vector<bool> present;  // ranks currently joined
    bool failed = false;
    std::string why;            // first failure
    struct Op {
        gol_ctx* ctx;
        uint32_t* buf;
        size_t bytes;
        hipEvent_t ready = nullptr;  // sends: the data is final on the sender's comm stream
        bool matched = false;
        int err = GOL_OK;
    };
    std::map<std::pair<int, int>, std::deque<std::shared_ptr<Op>>> sends, recvs;  // key (src, dst)
    std::vector<uint64_t> acc, result;
    int arrived = 0;
    uint64_t round = 0;
};

namespace {

std::mutex g_loop_mu;
std::map<std::string, std::weak_ptr<LoopRing>> g_loops;

// Match the queued sends src -> dst with the receives posted for them (ring
// lock held): FIFO per pair, like NCCL point-to-point.
void loop_match(LoopRing& ring, int src, int dst) {
    auto& sq = ring.sends[{src, dst}];
    auto& rq = ring.recvs[{src, dst}];
    while (!sq.empty() && !rq.empty()) {
        auto snd = sq.front(), rcv = rq.front();
        sq.pop_front();
        rq.pop_front();
        hipError_t e = hipSuccess;
        if (snd->bytes != rcv->bytes) {
            snd->err = rcv->err = GOL_ECOMM;
        } else {
            hipEvent_t done = nullptr;
            e = hipSetDevice(rcv->ctx->device);
            if (e == hipSuccess) e = hipStreamWaitEvent(rcv->ctx->comm, snd->ready, 0);
            if (e == hipSuccess)
                e = hipMemcpyPeerAsync(rcv->buf, rcv->ctx->device, snd->buf, snd->ctx->device, snd->bytes,
                                       rcv->ctx->comm);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventRecord(done, rcv->ctx->comm);
            if (e == hipSuccess) e = hipSetDevice(snd->ctx->device);
            if (e == hipSuccess) e = hipStreamWaitEvent(snd->ctx->comm, done, 0);
            if (done) hip_note(hipEventDestroy(done), "loopback: hipEventDestroy");
            if (e != hipSuccess) {
                hip_note(e, "loopback: halo copy");
                snd->err = rcv->err = GOL_EHIP;
            }
        }
        snd->matched = rcv->matched = true;
    }
}

// How long a loopback rank waits for its peers (GOL_LOOPBACK_TIMEOUT_MS,
// default 120 s; tests shorten it).
std::chrono::milliseconds loop_timeout() {
    const char* e = getenv("GOL_LOOPBACK_TIMEOUT_MS");
    const long v = e ? atol(e) : 0;
    return std::chrono::milliseconds(v > 0 ? v : 120000);
}

// Mark the ring failed (ring lock held) and wake every waiting rank.
void loop_fail(LoopRing& ring, const std::string& why) {
    if (!ring.failed) {
        ring.failed = true;
        ring.why = why;
    }
    ring.cv.notify_all();
}

// Take this context's unmatched operations out of the ring's queues (ring
// lock held), so no peer can match them after the context stops waiting:
// they hold its plane pointers and events, which may be gone by then.
void loop_purge(LoopRing& ring, const gol_ctx* ctx) {
    for (auto* qs : {&ring.sends, &ring.recvs})
        for (auto& kv : *qs) {
            auto& q = kv.second;
            q.erase(std::remove_if(q.begin(), q.end(),
                                   [&](const std::shared_ptr<LoopRing::Op>& o) { return o->ctx == ctx && !o->matched; }),
                    q.end());
        }
}

int loop_exchange(gol_ctx* ctx, const HaloOp* ops, int n) {
    LoopRing& ring = *ctx->loop;
    std::vector<std::shared_ptr<LoopRing::Op>> mine;
    auto destroy_events = [&]() {
        for (auto& o : mine)
            if (o->ready) {
                hip_note(hipEventDestroy(o->ready), "loopback: hipEventDestroy");
                o->ready = nullptr;
            }
    };
    // Every send's event is created and recorded before any operation is
    // posted, so a failure here leaves nothing in the ring for a peer to match.
    for (int k = 0; k < n; ++k) {
        auto op = std::make_shared<LoopRing::Op>();
        op->ctx = ctx;
        op->buf = ops[k].buf;
        op->bytes = ops[k].count * sizeof(uint32_t);
        mine.push_back(op);
        if (!ops[k].send) continue;
        hipError_t e = hipEventCreateWithFlags(&op->ready, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(op->ready, ctx->comm);
        if (e != hipSuccess) {
            destroy_events();
            return hip_fail(ctx, e, "loopback: send event", __FILE__, __LINE__);
        }
    }
    {
        std::unique_lock<std::mutex> lk(ring.mu);
        if (ring.failed) {
            lk.unlock();
            destroy_events();
            return set_err(ctx, GOL_ECOMM, "loopback ring failed: %s", ring.why.c_str());
        }
        for (int k = 0; k < n; ++k) {
            auto& op = mine[k];
            if (ops[k].send) {
                ring.sends[{ctx->rank, ops[k].peer}].push_back(op);
                loop_match(ring, ctx->rank, ops[k].peer);
            } else {
                ring.recvs[{ops[k].peer, ctx->rank}].push_back(op);
                loop_match(ring, ops[k].peer, ctx->rank);
            }
        }
        ring.cv.notify_all();
        auto all_matched = [&] { return std::all_of(mine.begin(), mine.end(), [](const auto& o) { return o->matched; }); };
        ring.cv.wait_for(lk, loop_timeout(), [&] { return all_matched() || ring.failed; });
        if (!all_matched()) {
            // timed out, or the ring failed under us: nothing of ours may be
            // matched later
            loop_purge(ring, ctx);
            if (!ring.failed)
                loop_fail(ring, "rank " + std::to_string(ctx->rank) + " timed out waiting for a peer's halo operations");
            std::string why = ring.why;
            lk.unlock();
            bind(ctx);
            destroy_events();
            return set_err(ctx, GOL_ECOMM, "loopback ring: %s", why.c_str());
        }
    }
    int rc = bind(ctx);  // a match made on this thread may have switched devices
    for (auto& op : mine)
        if (op->err && !rc) rc = set_err(ctx, op->err, "loopback ring: halo operation failed");
    destroy_events();
    return rc;
}

int loop_allreduce(gol_ctx* ctx, uint64_t* values, uint32_t count) {
    LoopRing& ring = *ctx->loop;
    std::unique_lock<std::mutex> lk(ring.mu);
    if (ring.failed) return set_err(ctx, GOL_ECOMM, "loopback ring failed: %s", ring.why.c_str());
    if (ring.arrived == 0) {
        ring.acc.assign(values, values + count);
    } else if (ring.acc.size() != count) {
        loop_fail(ring, "all-reduce counts differ between ranks");
        return set_err(ctx, GOL_EINVAL, "loopback all-reduce: counts differ");
    } else {
        for (uint32_t k = 0; k < count; ++k) ring.acc[k] += values[k];
    }
    const uint64_t my_round = ring.round;
    if (++ring.arrived == ring.nranks) {
        ring.result = ring.acc;
        ring.arrived = 0;
        ++ring.round;
        ring.cv.notify_all();
    } else {
        ring.cv.wait_for(lk, loop_timeout(), [&] { return ring.round != my_round || ring.failed; });
        if (ring.round == my_round) {
            if (!ring.failed) loop_fail(ring, "rank " + std::to_string(ctx->rank) + " timed out in an all-reduce");
            return set_err(ctx, GOL_ECOMM, "loopback all-reduce: %s", ring.why.c_str());
        }
    }
    std::copy(ring.result.begin(), ring.result.end(), values);
    return GOL_OK;
}

// Leave the ring: this context's unmatched operations are withdrawn, and a
// ring left while others are still in it is failed, so they do not wait for
// a rank that is gone.
void loop_leave(gol_ctx* ctx) {
    if (!ctx->loop) return;
    std::lock_guard<std::mutex> lk(g_loop_mu);
    {
        LoopRing& ring = *ctx->loop;
        std::lock_guard<std::mutex> rl(ring.mu);
        loop_purge(ring, ctx);
        --ring.joined;
        if (ctx->rank >= 0 && (size_t)ctx->rank < ring.present.size()) ring.present[ctx->rank] = false;
        if (ring.joined > 0) loop_fail(ring, "rank " + std::to_string(ctx->rank) + " left the ring");
    }
    ctx->loop.reset();
    for (auto it = g_loops.begin(); it != g_loops.end();)
        it = it->second.expired() ? g_loops.erase(it) : std::next(it);
}

// A pass's halo operations as one RCCL group on the comm stream.
int rccl_exchange(gol_ctx* ctx, const HaloOp* ops, int nops) {
    NCCL_CHECK(ctx, ncclGroupStart());
    for (int k = 0; k < nops; ++k) {
        if (ops[k].send)
            NCCL_CHECK(ctx, ncclSend(ops[k].buf, ops[k].count, ncclUint32, ops[k].peer, ctx->nccl, ctx->comm));
        else
            NCCL_CHECK(ctx, ncclRecv(ops[k].buf, ops[k].count, ncclUint32, ops[k].peer, ctx->nccl, ctx->comm));
    }
    NCCL_CHECK(ctx, ncclGroupEnd());
    return GOL_OK;
}

// One pass of G generations (temporal blocking, G <= kMaxGensPerPass) of a
// stand-alone or RCCL-sharded context.  slots: the hash accumulators of these
// G generations (G * kHashGenStride), or null.
int one_pass(gol_ctx* ctx, int G, unsigned long long* slots) {
    uint32_t* cur = ctx->plane[ctx->cur];
    uint32_t* nxt = ctx->plane[ctx->cur ^ 1];
    const int32_t rows = (int32_t)ctx->rows;
    const bool torus = ctx->topology == GOL_TORUS;
    const int64_t pitch = ctx->pitch;
    if (!sharded(ctx)) {
        // torus: rows wrap inside the plane; clipped: outside rows are dead
        const int32_t lo[1] = {0}, hi[1] = {rows};
        int rc = launch_ranges(ctx, G, cur, nxt, ctx->zero_row, ctx->zero_row, 0, torus, slots, 1, lo, hi, kProfMain);
        if (rc) return rc;
    } else if (ctx->group) {
        return set_err(ctx, GOL_ESTATE, "context belongs to a shard group: step it with gol_group_step");
    } else {
        const int up = (ctx->rank + ctx->nranks - 1) % ctx->nranks;
        const int down = (ctx->rank + 1) % ctx->nranks;
        const bool has_up = torus || ctx->rank > 0;
        const bool has_down = torus || ctx->rank < ctx->nranks - 1;
        // G-deep halo exchange on the comm stream once the current plane is
        // final (ev_ready: recorded before this pass's interior launch, so the
        // exchange does not wait for it).  The interior launch is enqueued
        // first: the GPU starts it while the host is still inside the RCCL
        // group calls.  If it cannot be enqueued, the halo operations are
        // still posted before the error is returned: the peers' groups then
        // complete instead of blocking in ncclGroupEnd until someone aborts
        // the communicator.
        HIP_CHECK(ctx, hipEventRecord(ctx->ev_ready, ctx->compute));
        const size_t evs_before = ctx->evs_used;
        const int rc_interior = sharded_interior(ctx, G, slots, has_up, has_down);
        // the interior launch's event pair (profiling; -1 if it has none in this fold window)
        int iref = (ctx->prof && ctx->evs_used == evs_before + 1) ? (int)evs_before : -1;
        HIP_CHECK(ctx, hipStreamWaitEvent(ctx->comm, ctx->ev_ready, 0));
        const size_t cnt = (size_t)G * pitch;  // G contiguous rows (pitch padding included)
        // Issue order matters when up == down (2 ranks, or 1 rank sending to
        // itself): per-peer FIFO matching pairs my last rows with the peer's
        // top halo and my first rows with its bottom halo
        // (gameoflife/shard.py HaloPlan mirrors this order).  One op list,
        // run by RCCL or by the in-process loopback ring.
        HaloOp ops[4];
        int nops = 0;
        if (has_down) ops[nops++] = {true, cur + (int64_t)(rows - G) * pitch, cnt, down};
        if (has_up) ops[nops++] = {true, cur, cnt, up};
        if (has_up) ops[nops++] = {false, ctx->halo_top, cnt, up};
        if (has_down) ops[nops++] = {false, ctx->halo_bot, cnt, down};
        // exchange timing (gol_profile_stats): comm-stream events around the group
        EventPair* xev = nullptr;
        if (ctx->prof && rc_interior == GOL_OK) {
            xev = next_event_pair(ctx);
            if (!xev) return set_err(ctx, GOL_EHIP, "profiling event allocation failed");
            xev->kind = kProfExchange;
            if ((int)ctx->evs_used - 1 <= iref) iref = -1;  // the allocation folded the window
            xev->ref = iref;
            HIP_CHECK(ctx, hipEventRecord(xev->start, ctx->comm));
        }
        for (int k = 0; k < nops; ++k) (ops[k].send ? ctx->halo_sent : ctx->halo_recv) += ops[k].count * 4;
        const int rc_x = ctx->loop ? loop_exchange(ctx, ops, nops) : rccl_exchange(ctx, ops, nops);
        if (xev) {
            if (rc_x == GOL_OK) {
                HIP_CHECK(ctx, hipEventRecord(xev->stop, ctx->comm));
            } else {
                --ctx->evs_used;  // the pair stays unrecorded: hand it back (it was the last one taken)
            }
        }
        if (rc_interior) return rc_interior;
        if (rc_x) return rc_x;
        // The event covers the sends too: the next pass overwrites this plane
        // only after the boundary kernels, which wait for it.
        HIP_CHECK(ctx, hipEventRecord(ctx->ev_halo, ctx->comm));
        const size_t evs_mid = ctx->evs_used;
        int rc = sharded_boundary(ctx, G, slots, has_up, has_down, &ctx->ev_halo, 1);
        if (rc) return rc;
        if (ctx->prof && ctx->evs_used == evs_mid + 1 && ctx->evs[evs_mid].kind == kProfBoundary && iref >= 0 &&
            (int)evs_mid > iref)
            ctx->evs[evs_mid].ref = iref;
    }
    ctx->cur ^= 1;
    ctx->epoch += (uint64_t)G;
    return GOL_OK;
}

size_t group_size(const gol_group* g) { return g->shards.size(); }

int64_t group_min_rows(const gol_group* g) {
    int64_t m = INT64_MAX;
    for (const gol_ctx* s : g->shards) m = std::min(m, s->rows);
    return m;
}

int group_fail(gol_group* g, const gol_ctx* s, int rc) {
    g->err = "shard " + std::to_string(s->gindex) + ": " + s->err;
    return rc;
}

// One pass of G generations over every shard of an in-process group.  Each
// shard's comm stream pulls its neighbours' G edge rows into its halo
// buffers (hipMemcpyPeerAsync: the shards may live on different GPUs); the
// kernels then run exactly as in an RCCL-sharded pass.  Ordering:
//  - a pull waits for the neighbour's plane to be final (its ev_ready);
//  - a shard's boundary kernels wait for its own pulls and for its
//    neighbours' pulls (ev_halo of all three), so its next pass cannot
//    overwrite rows a neighbour is still reading, and its next pull cannot
//    overwrite halo rows its boundary kernels still read.
int group_pass(gol_group* g, int G, const std::vector<unsigned long long*>& slots) {
    const int n = (int)g->shards.size();
    for (gol_ctx* s : g->shards) {
        if (int rc = bind(s)) return group_fail(g, s, rc);
        if (hipError_t e = hipEventRecord(s->ev_ready, s->compute))
            return group_fail(g, s, hip_fail(s, e, "hipEventRecord", __FILE__, __LINE__));
    }
    for (int k = 0; k < n; ++k) {
        gol_ctx* s = g->shards[k];
        gol_ctx* up = g->shards[(k + n - 1) % n];
        gol_ctx* dn = g->shards[(k + 1) % n];
        const bool has_up = g->torus || k > 0, has_down = g->torus || k < n - 1;
        const size_t bytes = (size_t)G * s->pitch * sizeof(uint32_t);
        if (int rc = bind(s)) return group_fail(g, s, rc);
        hipError_t e = hipStreamWaitEvent(s->comm, s->ev_ready, 0);
        if (e == hipSuccess && has_up) e = hipStreamWaitEvent(s->comm, up->ev_ready, 0);
        if (e == hipSuccess && has_down) e = hipStreamWaitEvent(s->comm, dn->ev_ready, 0);
        if (e == hipSuccess && has_up)
            e = hipMemcpyPeerAsync(s->halo_top, s->device, up->plane[up->cur] + (up->rows - G) * up->pitch, up->device,
                                   bytes, s->comm);
        if (e == hipSuccess && has_down)
            e = hipMemcpyPeerAsync(s->halo_bot, s->device, dn->plane[dn->cur], dn->device, bytes, s->comm);
        if (e == hipSuccess) e = hipEventRecord(s->ev_halo, s->comm);
        if (e != hipSuccess) return group_fail(g, s, hip_fail(s, e, "halo pull", __FILE__, __LINE__));
    }
    for (int k = 0; k < n; ++k) {
        gol_ctx* s = g->shards[k];
        gol_ctx* up = g->shards[(k + n - 1) % n];
        gol_ctx* dn = g->shards[(k + 1) % n];
        const bool has_up = g->torus || k > 0, has_down = g->torus || k < n - 1;
        hipEvent_t ready[3];
        int nr = 0;
        ready[nr++] = s->ev_halo;
        if (has_up) ready[nr++] = up->ev_halo;
        if (has_down) ready[nr++] = dn->ev_halo;
        if (int rc = bind(s)) return group_fail(g, s, rc);
        if (int rc = sharded_pass_kernels(s, G, slots.empty() ? nullptr : slots[k], has_up, has_down, ready, nr))
            return group_fail(g, s, rc);
    }
    for (gol_ctx* s : g->shards) {
        s->cur ^= 1;
        s->epoch += (uint64_t)G;
    }
    return GOL_OK;
}

// Deepest pass the context may run.  Every shard of a ring must pick the
// same depths (their halo messages must match), so a sharded pass is capped
// by the smallest shard of the decomposition, floor(H / N) (a 1-rank ring
// sends G of its own rows: G <= H).
// Planned (not fixed) passes deeper than kMaxGensPlannedGeneric run only on
// the B3/S23 torus kernels: the generic-rule and clipped instances hold their
// rule masks / visibility planes in registers and drop to 2 waves per SIMD at
// G >= 10 (scripts/resource_usage.py), and the cost table is measured on the
// B3/S23 torus.
constexpr int kMaxGensPlannedGeneric = 8;

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
    const double* cost = kPassCost[hashed ? 1 : 0][wide ? 1 : 0];
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

void destroy_impl(gol_ctx* c) {
    if (!c) return;
    if (c->group) {
        // a lost shard (the analogue of DeathWatch's Terminated, BoardCreator.scala:120-121):
        // the group keeps a hole and refuses to step until it is rebuilt
        gol_group* g = c->group;
        for (auto& s : g->shards)
            if (s == c) s = nullptr;
        g->err = "shard " + std::to_string(c->gindex) + " was destroyed; rebuild the group";
        c->group = nullptr;
    }
    // gol_destroy returns nothing: a failing teardown call is logged (and
    // taken off the thread), and teardown goes on.
    hip_note(hipSetDevice(c->device), "destroy: hipSetDevice");
    for (hipStream_t st : {c->compute, c->comm, c->edge, c->xfer})
        if (st) hip_note(hipStreamSynchronize(st), "destroy: hipStreamSynchronize");
    loop_leave(c);
    if (c->nccl) {
        const hipError_t pre = hipPeekAtLastError();
        const ncclResult_t r = ncclCommDestroy(c->nccl);
        absorb_rccl_status("ncclCommDestroy", pre);
        if (r != ncclSuccess) fprintf(stderr, "libgol: destroy: ncclCommDestroy: %s\n", ncclGetErrorString(r));
        c->nccl = nullptr;
    }
    for (auto& e : c->evs) {
        if (e.start) hip_note(hipEventDestroy(e.start), "destroy: hipEventDestroy");
        if (e.stop) hip_note(hipEventDestroy(e.stop), "destroy: hipEventDestroy");
    }
    for (hipEvent_t ev : {c->ev_ready, c->ev_halo, c->ev_edge, c->ev_snap_ready, c->ev_snap_done})
        if (ev) hip_note(hipEventDestroy(ev), "destroy: hipEventDestroy");
    for (void* p : {(void*)c->snap, (void*)c->clk_buf, (void*)c->plane[0], (void*)c->plane[1], (void*)c->halo_top,
                    (void*)c->halo_bot, (void*)c->zero_row, (void*)c->slots})
        if (p) hip_note(hipFree(p), "destroy: hipFree");
    for (hipStream_t st : {c->compute, c->comm, c->edge, c->xfer})
        if (st) hip_note(hipStreamDestroy(st), "destroy: hipStreamDestroy");
    delete c;
}

struct CkptHeader {
    char magic[8];  // "GOLCKPT1"
    int64_t width, height, row0, rows;
    int64_t wwords;
    uint64_t epoch;
    int32_t topology;
    uint32_t birth, survive;
    int32_t pad;
};

}  // namespace

extern "C" {

int gol_abi_version(void) { return GOL_ABI_VERSION; }

const char* gol_strerror(int code) {
    switch (code) {
        case GOL_OK: return "ok";
        case GOL_EINVAL: return "invalid argument";
        case GOL_EHIP: return "HIP runtime error";
        case GOL_ENOMEM: return "out of memory";
        case GOL_ECOMM: return "communication (RCCL) error";
        case GOL_ESTATE: return "invalid state";
        case GOL_ENODEV: return "no HIP device";
        default: return "unknown error";
    }
}

const char* gol_last_error(const gol_ctx* ctx) {
    if (ctx) return ctx->err.c_str();
    std::lock_guard<std::mutex> lk(g_err_mu);
    static thread_local std::string copy;
    copy = g_err;
    return copy.c_str();
}

int gol_device_count(int* count) {
    if (!count) return set_err(nullptr, GOL_EINVAL, "count is null");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();  // no device: the answer is 0, not an error
        n = 0;
    }
    *count = n;
    return GOL_OK;
}

int gol_shard_rows(int64_t height, int rank, int nranks, int64_t* row0, int64_t* rows) {
    if (height <= 0 || nranks <= 0 || rank < 0 || rank >= nranks || !row0 || !rows)
        return set_err(nullptr, GOL_EINVAL, "gol_shard_rows: bad arguments");
    if (height < nranks) return set_err(nullptr, GOL_EINVAL, "gol_shard_rows: fewer rows than ranks");
    // contiguous blocks; the first (height % nranks) ranks get one extra row
    const int64_t base = height / nranks, extra = height % nranks;
    *row0 = rank * base + std::min<int64_t>(rank, extra);
    *rows = base + (rank < extra ? 1 : 0);
    return GOL_OK;
}

int gol_device_layout(int32_t topology, int64_t width, int32_t* words_per_group) {
    if (!words_per_group || width <= 0 || (topology != GOL_TORUS && topology != GOL_REF_CLIPPED))
        return set_err(nullptr, GOL_EINVAL, "gol_device_layout: bad arguments");
    *words_per_group = device_ilv(topology, (width + 31) / 32);
    return GOL_OK;
}

int gol_create(gol_ctx** out, const gol_config* cfg) {
    if (!out || !cfg) return set_err(nullptr, GOL_EINVAL, "gol_create: null argument");
    *out = nullptr;
    const gol_config& c = *cfg;
    if (c.width <= 0 || c.height <= 0) return set_err(nullptr, GOL_EINVAL, "width/height must be > 0");
    if (c.topology != GOL_TORUS && c.topology != GOL_REF_CLIPPED)
        return set_err(nullptr, GOL_EINVAL, "unknown topology %d", c.topology);
    // Column indices in the kernels (StepParams.wwords, lane columns) are
    // int32 word counts: rows below 2^31 cells keep them far inside range.
    if (c.width >= (int64_t(1) << 31))
        return set_err(nullptr, GOL_EINVAL, "width must be below 2^31 cells (got %lld)", (long long)c.width);
    if (c.topology == GOL_TORUS && c.width % 32 != 0)
        return set_err(nullptr, GOL_EINVAL, "torus width must be a multiple of 32 (got %lld)", (long long)c.width);
    if ((c.birth_mask | c.survive_mask) & ~0x1FFu)
        return set_err(nullptr, GOL_EINVAL, "rule masks must fit in 9 bits");
    const int64_t rows = c.rows > 0 ? c.rows : c.height - c.row0;
    if (c.row0 < 0 || rows <= 0 || c.row0 + rows > c.height)
        return set_err(nullptr, GOL_EINVAL, "shard rows [%lld, %lld) outside the board", (long long)c.row0,
                       (long long)(c.row0 + rows));
    const int64_t wwords = (c.width + 31) / 32;
    if (wwords > (1 << 30) || rows > (1 << 30))
        return set_err(nullptr, GOL_EINVAL, "board too large");
    if (c.topology == GOL_REF_CLIPPED) {
        // The reference never completes a generation on a board where some
        // cell has no visible neighbour: that cell's gatherer asks nobody, so
        // no StateForEpoch ever arrives to complete it
        // (NextStateCellGathererActor.scala:26-27,39-47); it retries, fails
        // (:49-53) and re-asks for neighbours forever (CellActor.scala:92-94),
        // never committing epoch 1, and every neighbour's request for that
        // epoch stays queued (:75-76).  Such boards are refused rather than
        // advanced with results the reference never produces.
        const int64_t vw = c.vis_width > 0 ? c.vis_width : c.width - 1;
        const int64_t vh = c.vis_height > 0 ? c.vis_height : c.height - 1;
        if (vw < 1 || vh < 1 || (vw == 1 && vh == 1) || c.width > vw + 1 || c.height > vh + 1)
            return set_err(nullptr, GOL_EINVAL,
                           "ref-clipped board %lld x %lld with visible extents %lld x %lld: a cell has no visible "
                           "neighbour, and the reference never completes a generation on such a board "
                           "(NextStateCellGathererActor.scala:26-27,39-58, CellActor.scala:75-76,92-94)",
                           (long long)c.width, (long long)c.height, (long long)vw, (long long)vh);
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return set_err(nullptr, GOL_ENODEV, "no HIP device available (libgol has no CPU fallback)");
    }
    if (c.device < 0 || c.device >= ndev)
        return set_err(nullptr, GOL_EINVAL, "device %d out of range (%d devices)", c.device, ndev);

    gol_ctx* ctx = new gol_ctx();
    ctx->width = c.width;
    ctx->height = c.height;
    ctx->row0 = c.row0;
    ctx->rows = rows;
    ctx->wwords = (int32_t)wwords;
    ctx->pitch = (wwords + 63) / 64 * 64;  // 256-byte aligned rows
    ctx->topology = c.topology;
    ctx->birth = c.birth_mask;
    ctx->survive = c.survive_mask;
    ctx->vis_w = c.vis_width > 0 ? c.vis_width : c.width - 1;
    ctx->vis_h = c.vis_height > 0 ? c.vis_height : c.height - 1;
    ctx->ilv = device_ilv(c.topology, wwords);
    ctx->device = c.device;
    ctx->vec_fixed = 0;
    if (hipDeviceGetAttribute(&ctx->num_cus, hipDeviceAttributeMultiprocessorCount, c.device) != hipSuccess) {
        (void)hipGetLastError();  // unknown CU count: the tuning falls back to its defaults
        ctx->num_cus = 0;
    }

    auto fail = [&](int rc) {
        (void)hipGetLastError();  // the failed call's status: reported through rc
        std::string msg = ctx->err;
        destroy_impl(ctx);
        set_err(nullptr, rc, "%s", msg.c_str());
        return rc;
    };
    if (bind(ctx)) return fail(GOL_EHIP);
    const size_t plane_bytes = (size_t)rows * ctx->pitch * sizeof(uint32_t);
    for (int k = 0; k < 2; ++k) {
        if (hipMalloc(&ctx->plane[k], plane_bytes) != hipSuccess) {
            set_err(ctx, GOL_ENOMEM, "hipMalloc of %zu bytes failed", plane_bytes);
            return fail(GOL_ENOMEM);
        }
        if (hipMemset(ctx->plane[k], 0, plane_bytes) != hipSuccess) {
            set_err(ctx, GOL_EHIP, "hipMemset failed");
            return fail(GOL_EHIP);
        }
    }
    // G-deep halos (receive buffers) and kMaxGensPerPass dead rows
    const size_t row_bytes = (size_t)gol::kMaxGensPerPass * ctx->pitch * sizeof(uint32_t);
    if (hipMalloc(&ctx->halo_top, row_bytes) != hipSuccess || hipMalloc(&ctx->halo_bot, row_bytes) != hipSuccess ||
        hipMalloc(&ctx->zero_row, row_bytes) != hipSuccess) {
        set_err(ctx, GOL_ENOMEM, "halo allocation failed");
        return fail(GOL_ENOMEM);
    }
    if (hipMemset(ctx->halo_top, 0, row_bytes) != hipSuccess || hipMemset(ctx->halo_bot, 0, row_bytes) != hipSuccess ||
        hipMemset(ctx->zero_row, 0, row_bytes) != hipSuccess) {
        set_err(ctx, GOL_EHIP, "hipMemset failed");
        return fail(GOL_EHIP);
    }
    if (hipStreamCreateWithFlags(&ctx->compute, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->comm, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->edge, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->ev_edge, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->ev_ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->ev_halo, hipEventDisableTiming) != hipSuccess) {
        set_err(ctx, GOL_EHIP, "stream/event creation failed");
        return fail(GOL_EHIP);
    }
    // Load every step kernel instance this context can launch, now: the HIP
    // runtime loads a code object on the first use of one of its kernels, and
    // each pass depth lives in its own code object (gol_step_g<G>.hip), so the
    // first gol_step that plans a new depth would otherwise stall inside the
    // caller's timed region.  The occupancy query of an instance loads it
    // (and fills the cache launch_ranges reads).
    {
        const bool clipped = ctx->topology == GOL_REF_CLIPPED;
        const bool life = !clipped && ctx->birth == GOL_RULE_LIFE_BIRTH && ctx->survive == GOL_RULE_LIFE_SURVIVE;
        for (int G = 1; G <= gol::kMaxGensPerPass; ++G)
            for (int h = 0; h < 2; ++h) (void)resident_waves(ctx, lane_words(ctx, G), G, life, h != 0, clipped);
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        set_err(ctx, GOL_EHIP, "hipDeviceSynchronize failed");
        return fail(GOL_EHIP);
    }
    *out = ctx;
    return GOL_OK;
}

void gol_destroy(gol_ctx* ctx) { destroy_impl(ctx); }

int gol_seed(gol_ctx* ctx, uint64_t seed) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (int rc = bind(ctx)) return rc;
    HIP_CHECK(ctx, gol::launch_seed(ctx->plane[ctx->cur], ctx->pitch, ctx->wwords, ctx->width, ctx->row0,
                                    (int32_t)ctx->rows, seed, ctx->ilv, ctx->compute));
    ctx->epoch = 0;
    HIP_CHECK(ctx, hipStreamSynchronize(ctx->compute));
    return GOL_OK;
}

int gol_load(gol_ctx* ctx, const uint32_t* packed, int64_t host_pitch_words) {
    if (!ctx || !packed) return set_err(ctx, GOL_EINVAL, "null argument");
    if (host_pitch_words < ctx->wwords)
        return set_err(ctx, GOL_EINVAL, "host pitch %lld < words per row %d", (long long)host_pitch_words,
                       ctx->wwords);
    // Bits beyond the board width must be dead (layout invariant).
    if (ctx->width % 32) {
        const uint32_t m = (uint32_t)((1ull << (ctx->width % 32)) - 1ull);
        for (int64_t r = 0; r < ctx->rows; ++r)
            if (packed[r * host_pitch_words + ctx->wwords - 1] & ~m)
                return set_err(ctx, GOL_EINVAL, "padding bits beyond width set in row %lld", (long long)r);
    }
    if (int rc = bind(ctx)) return rc;
    // interleaved layouts: upload into the spare plane, interleave into the current one
    uint32_t* dst = ctx->ilv > 1 ? ctx->plane[ctx->cur ^ 1] : ctx->plane[ctx->cur];
    HIP_CHECK(ctx, hipMemcpy2DAsync(dst, ctx->pitch * 4, packed, host_pitch_words * 4, (size_t)ctx->wwords * 4,
                                    ctx->rows, hipMemcpyHostToDevice, ctx->compute));
    if (ctx->ilv > 1)
        HIP_CHECK(ctx, gol::launch_convert(dst, ctx->plane[ctx->cur], ctx->pitch, ctx->wwords, (int32_t)ctx->rows,
                                           true, ctx->ilv, ctx->compute));
    HIP_CHECK(ctx, hipStreamSynchronize(ctx->compute));
    ctx->epoch = 0;
    return GOL_OK;
}

int gol_step(gol_ctx* ctx, uint32_t generations, uint64_t* hashes_out) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (int rc = bind(ctx)) return rc;
    if (generations == 0) return GOL_OK;
    constexpr uint32_t kChunk = 1024;
    if (!hashes_out) {
        for (uint32_t g0 = 0; g0 < generations; g0 += kChunk)
            for (const int G : plan_passes(ctx, std::min(kChunk, generations - g0), false))
                if (int rc = one_pass(ctx, G, nullptr)) return rc;
        return GOL_OK;
    }
    for (uint32_t g0 = 0; g0 < generations; g0 += kChunk) {
        const uint32_t n = std::min(kChunk, generations - g0);
        if (int rc = ensure_slots(ctx, n)) return rc;
        const size_t per = (size_t)gol::kHashGenStride;
        HIP_CHECK(ctx, hipMemsetAsync(ctx->slots, 0, n * per * sizeof(unsigned long long), ctx->compute));
        uint32_t g = 0;
        for (const int G : plan_passes(ctx, n, true)) {
            if (int rc = one_pass(ctx, G, ctx->slots + g * per)) return rc;
            g += (uint32_t)G;
        }
        HIP_CHECK(ctx, hipMemcpyAsync(ctx->host_slots.data(), ctx->slots, n * per * sizeof(unsigned long long),
                                      hipMemcpyDeviceToHost, ctx->compute));
        HIP_CHECK(ctx, hipStreamSynchronize(ctx->compute));
        fold_slots(ctx, n, hashes_out + g0);
    }
    return GOL_OK;
}

int gol_step_ex(gol_ctx* ctx, uint32_t generations, uint64_t* hashes_out, size_t hashes_capacity) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (hashes_out && hashes_capacity < generations)
        return set_err(ctx, GOL_EINVAL, "hashes_out holds %zu entries, %u generations requested", hashes_capacity,
                       generations);
    return gol_step(ctx, generations, hashes_out);
}

int gol_replay(gol_ctx* ctx, uint32_t generations, const uint32_t* above, const uint32_t* below,
               int64_t host_pitch_words, uint64_t* hashes_out) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (generations == 0) return GOL_OK;
    if (!above || !below) return set_err(ctx, GOL_EINVAL, "null light-cone rows");
    if (host_pitch_words < ctx->wwords)
        return set_err(ctx, GOL_EINVAL, "host pitch %lld < words per row %d", (long long)host_pitch_words,
                       ctx->wwords);
    if (ctx->group || in_ring(ctx))
        return set_err(ctx, GOL_ESTATE, "replay a shard before it joins its group or ring");
    const int64_t n = generations;
    const int64_t ext = ctx->rows + 2 * n;
    if (ext > (1 << 30)) return set_err(ctx, GOL_EINVAL, "light cone too deep");
    if (int rc = bind(ctx)) return rc;
    if (hashes_out) {
        if (int rc = ensure_slots(ctx, generations)) return rc;
        HIP_CHECK(ctx, hipMemsetAsync(ctx->slots, 0, (size_t)n * gol::kHashGenStride * sizeof(unsigned long long),
                                      ctx->compute));
    }
    const size_t bytes = (size_t)ext * ctx->pitch * sizeof(uint32_t);
    uint32_t* blk[2] = {nullptr, nullptr};
    auto release = [&]() {
        hip_note(hipStreamSynchronize(ctx->compute), "replay: hipStreamSynchronize");
        for (auto* b : blk)
            if (b) hip_note(hipFree(b), "replay: hipFree");
    };
    for (auto*& b : blk) {
        if (hipMalloc(&b, bytes) != hipSuccess) {
            (void)hipGetLastError();
            b = nullptr;
            release();
            return set_err(ctx, GOL_ENOMEM, "hipMalloc of %zu bytes for the light cone failed", bytes);
        }
    }
    // The extended block: n rows above, the shard's rows, n rows below, as
    // they were at the shard's epoch.  Host rows are row-major; a pair-layout
    // board converts them on the device (upload to the other block first).
    const int64_t pitch = ctx->pitch, hp = host_pitch_words;
    uint32_t* up = ctx->ilv > 1 ? blk[1] : blk[0];
    auto fail_hip = [&](hipError_t e, const char* what) {
        (void)hipGetLastError();
        release();
        return set_err(ctx, GOL_EHIP, "%s failed: %s", what, hipGetErrorString(e));
    };
    hipError_t e = hipMemsetAsync(blk[0], 0, bytes, ctx->compute);
    if (e == hipSuccess)
        e = hipMemcpy2DAsync(up, pitch * 4, above, hp * 4, (size_t)ctx->wwords * 4, n, hipMemcpyHostToDevice,
                             ctx->compute);
    if (e == hipSuccess)
        e = hipMemcpy2DAsync(up + (n + ctx->rows) * pitch, pitch * 4, below, hp * 4, (size_t)ctx->wwords * 4, n,
                             hipMemcpyHostToDevice, ctx->compute);
    if (e == hipSuccess && ctx->ilv > 1) {
        e = gol::launch_convert(up, blk[0], pitch, ctx->wwords, (int32_t)n, true, ctx->ilv, ctx->compute);
        if (e == hipSuccess)
            e = gol::launch_convert(up + (n + ctx->rows) * pitch, blk[0] + (n + ctx->rows) * pitch, pitch,
                                    ctx->wwords, (int32_t)n, true, ctx->ilv, ctx->compute);
    }
    if (e == hipSuccess)
        e = hipMemcpyAsync(blk[0] + n * pitch, ctx->plane[ctx->cur], (size_t)ctx->rows * pitch * 4,
                           hipMemcpyDeviceToDevice, ctx->compute);
    if (e != hipSuccess) return fail_hip(e, "light-cone upload");
    // One generation per pass over the whole block; rows beyond it read as
    // dead (their garbage moves one row per generation and never reaches the
    // shard's rows).  Each generation's partial hash covers the shard's rows.
    const PlaneGeom geom{(int32_t)ext, ctx->row0 - n};
    const int32_t lo[1] = {0}, hi[1] = {(int32_t)ext};
    int cur = 0;
    for (int64_t g = 0; g < n; ++g) {
        if (int rc = launch_ranges(ctx, 1, blk[cur], blk[cur ^ 1], ctx->zero_row, ctx->zero_row, 0, false, nullptr, 1,
                                   lo, hi, kProfNone, ctx->compute, &geom)) {
            release();
            return rc;
        }
        cur ^= 1;
        if (hashes_out) {
            e = gol::launch_hash(blk[cur] + n * pitch, pitch, ctx->wwords, ctx->row0, (int32_t)ctx->rows, ctx->ilv,
                                 ctx->slots + (size_t)g * gol::kHashGenStride, ctx->compute);
            if (e != hipSuccess) return fail_hip(e, "light-cone hash");
        }
    }
    e = hipMemcpyAsync(ctx->plane[ctx->cur], blk[cur] + n * pitch, (size_t)ctx->rows * pitch * 4,
                       hipMemcpyDeviceToDevice, ctx->compute);
    if (e == hipSuccess && hashes_out)
        e = hipMemcpyAsync(ctx->host_slots.data(), ctx->slots, (size_t)n * gol::kHashGenStride * 8,
                           hipMemcpyDeviceToHost, ctx->compute);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->compute);
    if (e != hipSuccess) return fail_hip(e, "light-cone result");
    release();
    if (hashes_out) fold_slots(ctx, generations, hashes_out);
    ctx->epoch += (uint64_t)n;
    return GOL_OK;
}

int gol_comm_abort(gol_ctx* ctx) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (ctx->loop) {
        if (int rc = bind(ctx)) return rc;
        HIP_CHECK(ctx, hipStreamSynchronize(ctx->comm));
        loop_leave(ctx);
        ctx->rank = 0;
        ctx->nranks = 1;
        return GOL_OK;
    }
    if (!ctx->nccl) return GOL_OK;
    if (int rc = bind(ctx)) return rc;
    NCCL_CHECK(ctx, ncclCommAbort(ctx->nccl));
    ctx->nccl = nullptr;
    ctx->rank = 0;
    ctx->nranks = 1;
    return GOL_OK;
}

int gol_epoch(const gol_ctx* ctx, uint64_t* epoch) {
    if (!ctx || !epoch) return set_err(nullptr, GOL_EINVAL, "null argument");
    *epoch = ctx->epoch;
    return GOL_OK;
}

int gol_sync(gol_ctx* ctx) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (int rc = bind(ctx)) return rc;
    HIP_CHECK(ctx, hipStreamSynchronize(ctx->comm));
    HIP_CHECK(ctx, hipStreamSynchronize(ctx->compute));
    return GOL_OK;
}

int gol_hash(gol_ctx* ctx, uint64_t* hash_out) {
    if (!ctx || !hash_out) return set_err(ctx, GOL_EINVAL, "null argument");
    if (int rc = bind(ctx)) return rc;
    if (int rc = ensure_slots(ctx, 1)) return rc;
    const size_t per = (size_t)gol::kHashSlots * gol::kHashSlotStride;
    HIP_CHECK(ctx, hipMemsetAsync(ctx->slots, 0, per * sizeof(unsigned long long), ctx->compute));
    HIP_CHECK(ctx, gol::launch_hash(ctx->plane[ctx->cur], ctx->pitch, ctx->wwords, ctx->row0, (int32_t)ctx->rows,
                                    ctx->ilv, ctx->slots, ctx->compute));
    HIP_CHECK(ctx, hipMemcpyAsync(ctx->host_slots.data(), ctx->slots, per * sizeof(unsigned long long),
                                  hipMemcpyDeviceToHost, ctx->compute));
    HIP_CHECK(ctx, hipStreamSynchronize(ctx->compute));
    fold_slots(ctx, 1, hash_out);
    return GOL_OK;
}

int gol_snapshot(gol_ctx* ctx, uint32_t* packed_out, int64_t host_pitch_words) {
    if (!ctx || !packed_out) return set_err(ctx, GOL_EINVAL, "null argument");
    if (host_pitch_words < ctx->wwords) return set_err(ctx, GOL_EINVAL, "host pitch too small");
    if (int rc = bind(ctx)) return rc;
    // interleaved layouts: de-interleave into the spare plane (free between
    // passes: the compute stream is ordered after every reader of the last pass)
    const uint32_t* src = ctx->plane[ctx->cur];
    if (ctx->ilv > 1) {
        HIP_CHECK(ctx, gol::launch_convert(src, ctx->plane[ctx->cur ^ 1], ctx->pitch, ctx->wwords,
                                           (int32_t)ctx->rows, false, ctx->ilv, ctx->compute));
        src = ctx->plane[ctx->cur ^ 1];
    }
    HIP_CHECK(ctx, hipMemcpy2DAsync(packed_out, host_pitch_words * 4, src, ctx->pitch * 4, (size_t)ctx->wwords * 4,
                                    ctx->rows, hipMemcpyDeviceToHost, ctx->compute));
    HIP_CHECK(ctx, hipStreamSynchronize(ctx->compute));
    return GOL_OK;
}

// Asynchronous snapshot: the board is copied on the device (de-interleaved
// for the pair layout) into `snap` in the compute stream's order -- so later
// passes cannot overwrite it first -- and from there to the host on the
// transfer stream, concurrently with the passes queued after it.
constexpr size_t kSnapChunkBytes = 256ull << 20;

int gol_snapshot_async(gol_ctx* ctx, uint32_t* packed_out, int64_t host_pitch_words) {
    if (!ctx || !packed_out) return set_err(ctx, GOL_EINVAL, "null argument");
    if (host_pitch_words < ctx->wwords) return set_err(ctx, GOL_EINVAL, "host pitch too small");
    if (ctx->snap_pending) return set_err(ctx, GOL_ESTATE, "a snapshot is in flight: call gol_snapshot_wait first");
    if (int rc = bind(ctx)) return rc;
    // The device copy is packed (wwords per row, no pitch padding), so the
    // transfer of a packed host buffer is one linear copy: a 2D
    // device-to-host copy did not overlap the passes queued after it.
    const size_t bytes = (size_t)ctx->rows * ctx->wwords * sizeof(uint32_t);
    if (!ctx->snap) {
        if (hipMalloc(&ctx->snap, bytes) != hipSuccess) {
            (void)hipGetLastError();
            ctx->snap = nullptr;
            return set_err(ctx, GOL_ENOMEM, "hipMalloc of %zu bytes for the snapshot buffer failed", bytes);
        }
    }
    if (!ctx->xfer) HIP_CHECK(ctx, hipStreamCreateWithFlags(&ctx->xfer, hipStreamNonBlocking));
    if (!ctx->ev_snap_ready) HIP_CHECK(ctx, hipEventCreateWithFlags(&ctx->ev_snap_ready, hipEventDisableTiming));
    if (!ctx->ev_snap_done) HIP_CHECK(ctx, hipEventCreateWithFlags(&ctx->ev_snap_done, hipEventDisableTiming));
    const uint32_t* src = ctx->plane[ctx->cur];
    if (ctx->ilv > 1)
        HIP_CHECK(ctx, gol::launch_convert(src, ctx->snap, ctx->pitch, ctx->wwords, (int32_t)ctx->rows, false,
                                           ctx->ilv, ctx->compute, ctx->wwords));
    else
        HIP_CHECK(ctx, hipMemcpy2DAsync(ctx->snap, (size_t)ctx->wwords * 4, src, ctx->pitch * 4,
                                        (size_t)ctx->wwords * 4, ctx->rows, hipMemcpyDeviceToDevice, ctx->compute));
    HIP_CHECK(ctx, hipEventRecord(ctx->ev_snap_ready, ctx->compute));
    HIP_CHECK(ctx, hipStreamWaitEvent(ctx->xfer, ctx->ev_snap_ready, 0));
    if (host_pitch_words == ctx->wwords) {
        // in chunks (GOL_SNAP_CHUNK_MB, 0 = one copy): see DESIGN.md section 2
        const char* env = getenv("GOL_SNAP_CHUNK_MB");
        const size_t chunk = env ? (size_t)atol(env) << 20 : kSnapChunkBytes;
        const size_t step = chunk ? chunk : bytes;
        for (size_t off = 0; off < bytes; off += step)
            HIP_CHECK(ctx, hipMemcpyAsync(reinterpret_cast<char*>(packed_out) + off,
                                          reinterpret_cast<const char*>(ctx->snap) + off, std::min(step, bytes - off),
                                          hipMemcpyDeviceToHost, ctx->xfer));
    } else
        HIP_CHECK(ctx, hipMemcpy2DAsync(packed_out, host_pitch_words * 4, ctx->snap, (size_t)ctx->wwords * 4,
                                        (size_t)ctx->wwords * 4, ctx->rows, hipMemcpyDeviceToHost, ctx->xfer));
    HIP_CHECK(ctx, hipEventRecord(ctx->ev_snap_done, ctx->xfer));
    ctx->snap_pending = true;
    ctx->snap_epoch = ctx->epoch;
    return GOL_OK;
}

int gol_snapshot_wait(gol_ctx* ctx, uint64_t* epoch_out) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (!ctx->snap_pending) return set_err(ctx, GOL_ESTATE, "no snapshot in flight");
    if (int rc = bind(ctx)) return rc;
    // The snapshot stays in flight (and the caller keeps its buffer) until the
    // transfer is known to be over: a failed wait leaves snap_pending set.
    HIP_CHECK(ctx, hipEventSynchronize(ctx->ev_snap_done));
    ctx->snap_pending = false;
    if (epoch_out) *epoch_out = ctx->snap_epoch;
    return GOL_OK;
}

int gol_snapshot_query(gol_ctx* ctx, int* landed) {
    if (!ctx || !landed) return set_err(ctx, GOL_EINVAL, "null argument");
    if (!ctx->snap_pending) return set_err(ctx, GOL_ESTATE, "no snapshot in flight");
    if (int rc = bind(ctx)) return rc;
    const hipError_t e = hipEventQuery(ctx->ev_snap_done);
    if (e == hipErrorNotReady) {
        (void)hipGetLastError();  // "not yet" is an answer, not an error
        *landed = 0;
        return GOL_OK;
    }
    HIP_CHECK(ctx, e);
    *landed = 1;
    return GOL_OK;
}

int gol_host_alloc(size_t bytes, void** out) {
    if (!out || bytes == 0) return set_err(nullptr, GOL_EINVAL, "gol_host_alloc: null pointer or zero size");
    *out = nullptr;
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        *out = nullptr;
        return set_err(nullptr, GOL_ENOMEM, "hipHostMalloc of %zu bytes failed", bytes);
    }
    return GOL_OK;
}

void gol_host_free(void* p) {
    if (p) hip_note(hipHostFree(p), "gol_host_free: hipHostFree");
}

int gol_get_cell(gol_ctx* ctx, int64_t x, int64_t y, int* state) {
    if (!ctx || !state) return set_err(ctx, GOL_EINVAL, "null argument");
    if (x < 0 || x >= ctx->width || y < ctx->row0 || y >= ctx->row0 + ctx->rows)
        return set_err(ctx, GOL_EINVAL, "cell (%lld, %lld) not in this shard", (long long)x, (long long)y);
    if (int rc = bind(ctx)) return rc;
    // row-major: bit x % 32 of word x / 32; interleave groups of k words:
    // bit (x % 32k) / k of word k (x / 32k) + x % k
    const int64_t k = ctx->ilv, span = 32 * k;
    const int64_t word = k * (x / span) + x % k;
    const int bit = (int)((x % span) / k);
    uint32_t w = 0;
    HIP_CHECK(ctx, hipMemcpyAsync(&w, ctx->plane[ctx->cur] + (y - ctx->row0) * ctx->pitch + word, 4,
                                  hipMemcpyDeviceToHost, ctx->compute));
    HIP_CHECK(ctx, hipStreamSynchronize(ctx->compute));
    *state = (int)((w >> bit) & 1u);
    return GOL_OK;
}

int gol_checkpoint_bytes(const gol_ctx* ctx, size_t* bytes) {
    if (!ctx || !bytes) return set_err(nullptr, GOL_EINVAL, "null argument");
    *bytes = sizeof(CkptHeader) + (size_t)ctx->rows * ctx->wwords * sizeof(uint32_t);
    return GOL_OK;
}

int gol_checkpoint(gol_ctx* ctx, void* host_out, size_t bytes) {
    size_t need = 0;
    if (!ctx || !host_out) return set_err(ctx, GOL_EINVAL, "null argument");
    gol_checkpoint_bytes(ctx, &need);
    if (bytes < need) return set_err(ctx, GOL_EINVAL, "checkpoint buffer too small (%zu < %zu)", bytes, need);
    CkptHeader h{};
    memcpy(h.magic, "GOLCKPT1", 8);
    h.width = ctx->width; h.height = ctx->height; h.row0 = ctx->row0; h.rows = ctx->rows;
    h.wwords = ctx->wwords; h.epoch = ctx->epoch; h.topology = ctx->topology;
    h.birth = ctx->birth; h.survive = ctx->survive;
    memcpy(host_out, &h, sizeof h);
    return gol_snapshot(ctx, reinterpret_cast<uint32_t*>(static_cast<char*>(host_out) + sizeof h), ctx->wwords);
}

int gol_checkpoint_async(gol_ctx* ctx, void* host_out, size_t bytes) {
    size_t need = 0;
    if (!ctx || !host_out) return set_err(ctx, GOL_EINVAL, "null argument");
    gol_checkpoint_bytes(ctx, &need);
    if (bytes < need) return set_err(ctx, GOL_EINVAL, "checkpoint buffer too small (%zu < %zu)", bytes, need);
    if (ctx->snap_pending) return set_err(ctx, GOL_ESTATE, "a snapshot is in flight: call gol_snapshot_wait first");
    CkptHeader h{};
    memcpy(h.magic, "GOLCKPT1", 8);
    h.width = ctx->width; h.height = ctx->height; h.row0 = ctx->row0; h.rows = ctx->rows;
    h.wwords = ctx->wwords; h.epoch = ctx->epoch; h.topology = ctx->topology;
    h.birth = ctx->birth; h.survive = ctx->survive;
    // The header goes in only once the rows' copy is under way: a failed call
    // leaves no buffer that looks like a valid checkpoint.
    memset(host_out, 0, sizeof h);
    const int rc =
        gol_snapshot_async(ctx, reinterpret_cast<uint32_t*>(static_cast<char*>(host_out) + sizeof h), ctx->wwords);
    if (rc == GOL_OK) memcpy(host_out, &h, sizeof h);
    return rc;
}

int gol_restore(gol_ctx* ctx, const void* host_in, size_t bytes) {
    if (!ctx || !host_in) return set_err(ctx, GOL_EINVAL, "null argument");
    if (bytes < sizeof(CkptHeader)) return set_err(ctx, GOL_EINVAL, "checkpoint truncated");
    CkptHeader h;
    memcpy(&h, host_in, sizeof h);
    if (memcmp(h.magic, "GOLCKPT1", 8) != 0) return set_err(ctx, GOL_EINVAL, "bad checkpoint magic");
    if (h.width != ctx->width || h.height != ctx->height || h.row0 != ctx->row0 || h.rows != ctx->rows ||
        h.topology != ctx->topology || h.birth != ctx->birth || h.survive != ctx->survive)
        return set_err(ctx, GOL_EINVAL, "checkpoint geometry/rule does not match this context");
    if (bytes < sizeof h + (size_t)h.rows * h.wwords * 4) return set_err(ctx, GOL_EINVAL, "checkpoint truncated");
    int rc = gol_load(ctx, reinterpret_cast<const uint32_t*>(static_cast<const char*>(host_in) + sizeof h), h.wwords);
    if (rc) return rc;
    ctx->epoch = h.epoch;
    return GOL_OK;
}

int gol_comm_unique_id(uint8_t id_out[GOL_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == GOL_UNIQUE_ID_BYTES, "ncclUniqueId size");
    if (!id_out) return set_err(nullptr, GOL_EINVAL, "null argument");
    ncclUniqueId id;
    NCCL_CHECK(nullptr, ncclGetUniqueId(&id));
    memcpy(id_out, &id, sizeof id);
    return GOL_OK;
}

int gol_comm_init(gol_ctx* ctx, const uint8_t id[GOL_UNIQUE_ID_BYTES], int rank, int nranks) {
    if (!ctx || !id) return set_err(ctx, GOL_EINVAL, "null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) return set_err(ctx, GOL_EINVAL, "bad rank/nranks");
    if (in_ring(ctx)) return set_err(ctx, GOL_ESTATE, "communicator already initialised");
    if (int rc = bind(ctx)) return rc;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    NCCL_CHECK(ctx, ncclCommInitRank(&ctx->nccl, nranks, uid, rank));
    ctx->rank = rank;
    ctx->nranks = nranks;
    return GOL_OK;
}

int gol_comm_init_loopback(gol_ctx* ctx, const char* key, int rank, int nranks) {
    if (!ctx || !key) return set_err(ctx, GOL_EINVAL, "null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) return set_err(ctx, GOL_EINVAL, "bad rank/nranks");
    if (in_ring(ctx)) return set_err(ctx, GOL_ESTATE, "communicator already initialised");
    if (ctx->group) return set_err(ctx, GOL_ESTATE, "context belongs to a shard group");
    std::lock_guard<std::mutex> lk(g_loop_mu);
    std::shared_ptr<LoopRing> ring = g_loops[key].lock();
    if (!ring) {
        ring = std::make_shared<LoopRing>();
        ring->nranks = nranks;
        g_loops[key] = ring;
    }
    std::lock_guard<std::mutex> rl(ring->mu);
    if (ring->nranks != nranks) return set_err(ctx, GOL_EINVAL, "loopback ring %s has %d ranks", key, ring->nranks);
    if (ring->failed) return set_err(ctx, GOL_ESTATE, "loopback ring %s has failed (%s): join a new key", key, ring->why.c_str());
    if (ring->joined >= nranks) return set_err(ctx, GOL_ESTATE, "loopback ring %s is full", key);
    if (ring->present.empty()) ring->present.assign(nranks, false);
    if (ring->present[rank]) return set_err(ctx, GOL_EINVAL, "loopback ring %s: rank %d already joined", key, rank);
    ring->present[rank] = true;
    ++ring->joined;
    ctx->loop = ring;
    ctx->rank = rank;
    ctx->nranks = nranks;
    return GOL_OK;
}

int gol_comm_allreduce_u64(gol_ctx* ctx, uint64_t* values, uint32_t count) {
    if (!ctx || (!values && count)) return set_err(ctx, GOL_EINVAL, "null argument");
    if (!in_ring(ctx)) return set_err(ctx, GOL_ECOMM, "no communicator (call gol_comm_init)");
    if (count == 0) return GOL_OK;
    if (ctx->loop) return loop_allreduce(ctx, values, count);
    if (int rc = bind(ctx)) return rc;
    uint64_t* d = nullptr;
    HIP_CHECK(ctx, hipMallocAsync((void**)&d, count * sizeof(uint64_t), ctx->comm));
    HIP_CHECK(ctx, hipMemcpyAsync(d, values, count * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->comm));
    NCCL_CHECK(ctx, ncclAllReduce(d, d, count, ncclUint64, ncclSum, ctx->nccl, ctx->comm));
    HIP_CHECK(ctx, hipMemcpyAsync(values, d, count * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->comm));
    HIP_CHECK(ctx, hipFreeAsync(d, ctx->comm));
    HIP_CHECK(ctx, hipStreamSynchronize(ctx->comm));
    return GOL_OK;
}

int gol_profile_enable(gol_ctx* ctx, int enable) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    const char* probe = getenv("GOL_CLOCK_PROBE");  // "0": no in-kernel clock probe (A/B)
    if (enable && !ctx->clk_buf && !(probe && probe[0] == '0')) {
        if (int rc = bind(ctx)) return rc;
        const size_t bytes = (size_t)kClockSlots * gol::kClockSlotWords * sizeof(unsigned long long);
        if (hipMalloc(&ctx->clk_buf, bytes) != hipSuccess) {
            (void)hipGetLastError();
            ctx->clk_buf = nullptr;
            return set_err(ctx, GOL_ENOMEM, "clock-probe buffer allocation failed");
        }
        HIP_CHECK(ctx, hipMemset(ctx->clk_buf, 0, bytes));
    }
    ctx->prof = enable != 0;
    return GOL_OK;
}

int gol_profile_clock(gol_ctx* ctx, double* ghz) {
    if (!ctx || !ghz) return set_err(ctx, GOL_EINVAL, "null argument");
    if (int rc = bind(ctx)) return rc;
    if (int rc = fold_profile(ctx)) return rc;
    *ghz = ctx->prof_clk_ms > 0.0 ? ctx->prof_clk_ms_ghz / ctx->prof_clk_ms : 0.0;
    return GOL_OK;
}

int gol_profile_read(gol_ctx* ctx, double* total_ms, uint64_t* launches, uint64_t* generations) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (int rc = bind(ctx)) return rc;
    if (int rc = fold_profile(ctx)) return rc;
    if (total_ms) *total_ms = ctx->prof_ms;
    if (launches) *launches = ctx->prof_launches;
    if (generations) *generations = ctx->prof_gens;
    return GOL_OK;
}

int gol_profile_reset(gol_ctx* ctx) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (int rc = bind(ctx)) return rc;
    if (int rc = fold_profile(ctx)) return rc;
    ctx->prof_ms = 0.0;
    ctx->prof_launches = 0;
    ctx->prof_gens = 0;
    ctx->prof_clk_ms_ghz = ctx->prof_clk_ms = 0.0;
    ctx->prof_xchg_ms = ctx->prof_bnd_ms = 0.0;
    ctx->prof_xchg_exposed_ms = ctx->prof_tail_ms = 0.0;
    ctx->prof_xchg = ctx->prof_bnd = 0;
    ctx->halo_sent = ctx->halo_recv = 0;
    return GOL_OK;
}

int gol_profile_stats_read(gol_ctx* ctx, gol_profile_stats* out) {
    if (!ctx || !out) return set_err(ctx, GOL_EINVAL, "null argument");
    if (int rc = bind(ctx)) return rc;
    if (int rc = fold_profile(ctx)) return rc;
    *out = gol_profile_stats{};
    out->kernel_ms = ctx->prof_ms;
    out->launches = ctx->prof_launches;
    out->generations = ctx->prof_gens;
    out->exchange_ms = ctx->prof_xchg_ms;
    out->exchanges = ctx->prof_xchg;
    out->boundary_ms = ctx->prof_bnd_ms;
    out->boundary_launches = ctx->prof_bnd;
    out->halo_bytes_sent = ctx->halo_sent;
    out->halo_bytes_received = ctx->halo_recv;
    out->clock_ghz = ctx->prof_clk_ms > 0.0 ? ctx->prof_clk_ms_ghz / ctx->prof_clk_ms : 0.0;
    out->exchange_exposed_ms = ctx->prof_xchg_exposed_ms;
    out->pass_tail_ms = ctx->prof_tail_ms;
    return GOL_OK;
}

int gol_runtime_info_get(gol_runtime_info* out) {
    if (!out) return set_err(nullptr, GOL_EINVAL, "null argument");
    *out = gol_runtime_info{};
    out->abi_version = GOL_ABI_VERSION;
    int v = 0;
    if (hipRuntimeGetVersion(&v) == hipSuccess) out->hip_runtime_version = v;
    else (void)hipGetLastError();
    v = 0;
    if (hipDriverGetVersion(&v) == hipSuccess) out->hip_driver_version = v;
    else (void)hipGetLastError();
    v = 0;
    if (ncclGetVersion(&v) == ncclSuccess) out->rccl_version = v;
    // the files the dynamic linker bound these symbols to
    auto path_of = [](const void* sym, char* dst, size_t cap) {
        Dl_info info{};
        if (dladdr(sym, &info) && info.dli_fname) snprintf(dst, cap, "%s", info.dli_fname);
    };
    path_of(reinterpret_cast<const void*>(&hipRuntimeGetVersion), out->hip_library, sizeof out->hip_library);
    path_of(reinterpret_cast<const void*>(&ncclGetVersion), out->rccl_library, sizeof out->rccl_library);
    path_of(reinterpret_cast<const void*>(&gol_runtime_info_get), out->gol_library, sizeof out->gol_library);
    return GOL_OK;
}

int gol_set_tuning(gol_ctx* ctx, int32_t band_rows, int32_t gens_per_pass, int32_t words_per_lane) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (band_rows < 0 || gens_per_pass < 0 || gens_per_pass > gol::kMaxGensPerPass)
        return set_err(ctx, GOL_EINVAL, "tuning out of range (band_rows >= 0, 0 <= gens_per_pass <= %d)",
                       gol::kMaxGensPerPass);
    if (words_per_lane != 0 && words_per_lane != 1 && words_per_lane != 2 && words_per_lane != 4)
        return set_err(ctx, GOL_EINVAL, "words_per_lane must be 0 (auto), 1, 2 or 4");
    if (words_per_lane > 0 && ctx->wwords % words_per_lane != 0)
        return set_err(ctx, GOL_EINVAL, "words_per_lane %d does not divide the %d words of a row", words_per_lane,
                       ctx->wwords);
    if (words_per_lane == 4 && !life_torus(ctx) && gens_per_pass > gol::kMaxGensVec4Generic)
        return set_err(ctx, GOL_EINVAL,
                       "words_per_lane 4 with gens_per_pass %d > %d: the generic-rule / clipped kernel instance "
                       "would spill registers to scratch (not built)",
                       gens_per_pass, gol::kMaxGensVec4Generic);
    ctx->band_rows = band_rows;
    ctx->gens_per_pass = gens_per_pass;
    ctx->vec_fixed = words_per_lane;
    return GOL_OK;
}

int gol_pass_plan(gol_ctx* ctx, uint32_t generations, int32_t with_hashes, int32_t* depths, int32_t max,
                  int32_t* count) {
    if (!ctx || !count || (max > 0 && !depths)) return set_err(ctx, GOL_EINVAL, "null argument");
    if (generations > 1024) return set_err(ctx, GOL_EINVAL, "plans cover at most 1024 generations");
    const std::vector<int> plan = plan_passes(ctx, generations, with_hashes != 0);
    for (size_t k = 0; k < plan.size() && (int32_t)k < max; ++k) depths[k] = plan[k];
    *count = (int32_t)plan.size();
    return GOL_OK;
}

int gol_occupancy(gol_ctx* ctx, int32_t gens_per_pass, int32_t* waves_per_cu, int32_t* strip_words) {
    if (!ctx) return set_err(nullptr, GOL_EINVAL, "null context");
    if (gens_per_pass < 1 || gens_per_pass > gol::kMaxGensPerPass)
        return set_err(ctx, GOL_EINVAL, "gens_per_pass out of range");
    if (int rc = bind(ctx)) return rc;
    const bool clipped = ctx->topology == GOL_REF_CLIPPED;
    const bool life = !clipped && ctx->birth == GOL_RULE_LIFE_BIRTH && ctx->survive == GOL_RULE_LIFE_SURVIVE;
    const int vec = lane_words(ctx, gens_per_pass);
    const int blocks =
        gol::resident_blocks_per_cu(vec, gens_per_pass, life, false, clipped, ctx->ilv);
    if (waves_per_cu) *waves_per_cu = blocks * gol::kWavesPerWG;
    if (strip_words) *strip_words = gol::strip_words(vec, gens_per_pass);
    return GOL_OK;
}

int gol_selftest(int device, uint32_t* report) {
    // report[256]: see gol::selftest_kernel.  Diagnoses the DPP wave shifts,
    // v_alignbit and SMEM loads the step kernel relies on.
    if (!report) return set_err(nullptr, GOL_EINVAL, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return set_err(nullptr, GOL_ENODEV, "no HIP device available");
    }
    HIP_CHECK(nullptr, hipSetDevice(device));
    uint32_t h_in[64];
    for (int i = 0; i < 64; ++i) h_in[i] = 0x01000193u * (uint32_t)(i + 1) ^ (uint32_t)(i << 24);
    uint32_t *d_in = nullptr, *d_out = nullptr;
    HIP_CHECK(nullptr, hipMalloc(&d_in, sizeof h_in));
    HIP_CHECK(nullptr, hipMalloc(&d_out, 256 * sizeof(uint32_t)));
    HIP_CHECK(nullptr, hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice));
    HIP_CHECK(nullptr, gol::launch_selftest(d_in, d_out, nullptr));
    HIP_CHECK(nullptr, hipMemcpy(report, d_out, 256 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    hip_note(hipFree(d_in), "selftest: hipFree");
    hip_note(hipFree(d_out), "selftest: hipFree");
    return GOL_OK;
}

int gol_group_create(gol_group** out, gol_ctx* const* shards, int n) {
    if (!out || !shards || n < 1) return set_err(nullptr, GOL_EINVAL, "gol_group_create: bad arguments");
    *out = nullptr;
    const gol_ctx* a = shards[0];
    int64_t next_row = 0;
    for (int k = 0; k < n; ++k) {
        const gol_ctx* s = shards[k];
        if (!s) return set_err(nullptr, GOL_EINVAL, "shard %d is null", k);
        if (s->group || in_ring(s))
            return set_err(nullptr, GOL_ESTATE, "shard %d already belongs to a group or an RCCL ring", k);
        if (s->width != a->width || s->height != a->height || s->topology != a->topology ||
            s->birth != a->birth || s->survive != a->survive || s->vis_w != a->vis_w || s->vis_h != a->vis_h)
            return set_err(nullptr, GOL_EINVAL, "shard %d: board geometry or rule differs from shard 0", k);
        if (s->epoch != a->epoch) return set_err(nullptr, GOL_ESTATE, "shard %d is at a different epoch", k);
        if (s->row0 != next_row)
            return set_err(nullptr, GOL_EINVAL, "shard %d starts at row %lld, expected %lld (row order, no gaps)", k,
                           (long long)s->row0, (long long)next_row);
        next_row += s->rows;
    }
    if (next_row != a->height)
        return set_err(nullptr, GOL_EINVAL, "shards cover %lld of %lld rows", (long long)next_row,
                       (long long)a->height);
    gol_group* g = new gol_group();
    g->torus = a->topology == GOL_TORUS;
    for (int k = 0; k < n; ++k) {
        g->shards.push_back(shards[k]);
        shards[k]->group = g;
        shards[k]->gindex = k;
    }
    // peer access between neighbouring shards on different GPUs (best effort:
    // hipMemcpyPeerAsync falls back to staging without it)
    for (int k = 0; k < n; ++k) {
        gol_ctx* s = g->shards[k];
        gol_ctx* dn = g->shards[(k + 1) % n];
        if (s->device != dn->device) {
            int ok = 0;
            if (hipDeviceCanAccessPeer(&ok, s->device, dn->device) != hipSuccess) {
                (void)hipGetLastError();
                ok = 0;
            }
            if (ok) {
                for (auto [from, to] : {std::pair<int, int>{s->device, dn->device}, {dn->device, s->device}}) {
                    hip_note(hipSetDevice(from), "group: hipSetDevice");
                    const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
                    if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();  // an earlier group did it
                    else hip_note(e, "group: hipDeviceEnablePeerAccess");
                }
            }
        }
    }
    *out = g;
    return GOL_OK;
}

const char* gol_group_last_error(const gol_group* g) { return g ? g->err.c_str() : ""; }

int gol_diag_take_hip_error(int* code) {
    if (!code) return set_err(nullptr, GOL_EINVAL, "null argument");
    *code = (int)hipGetLastError();
    return GOL_OK;
}

int gol_diag_absorbed(uint64_t* count, char* last, size_t cap) {
    std::lock_guard<std::mutex> lk(g_absorb_mu);
    if (count) *count = g_absorbed;
    if (last && cap > 0) snprintf(last, cap, "%s", g_absorbed_last.c_str());
    return GOL_OK;
}

int gol_group_step(gol_group* g, uint32_t generations, uint64_t* hashes_out) {
    return gol_group_step_partials(g, generations, hashes_out, nullptr);
}

int gol_group_step_partials(gol_group* g, uint32_t generations, uint64_t* hashes_out, uint64_t* partials_out) {
    if (!g) return set_err(nullptr, GOL_EINVAL, "null group");
    if (partials_out && !hashes_out) {
        g->err = "partials_out needs hashes_out";
        return GOL_EINVAL;
    }
    for (const gol_ctx* s : g->shards)
        if (!s) return GOL_ESTATE;  // g->err names the lost shard
    if (generations == 0) return GOL_OK;
    const size_t per = (size_t)gol::kHashGenStride;
    const int n = (int)g->shards.size();
    constexpr uint32_t kChunk = 1024;
    std::vector<uint64_t> part;
    for (uint32_t g0 = 0; g0 < generations; g0 += kChunk) {
        const uint32_t cnt = std::min(kChunk, generations - g0);
        std::vector<unsigned long long*> base;
        if (hashes_out) {
            for (gol_ctx* s : g->shards) {
                if (int rc = bind(s)) return group_fail(g, s, rc);
                if (int rc = ensure_slots(s, cnt)) return group_fail(g, s, rc);
                if (hipError_t e = hipMemsetAsync(s->slots, 0, cnt * per * sizeof(unsigned long long), s->compute))
                    return group_fail(g, s, hip_fail(s, e, "hipMemsetAsync", __FILE__, __LINE__));
                base.push_back(s->slots);
            }
        }
        uint32_t done = 0;
        for (const int G : plan_passes(g->shards[0], cnt, hashes_out != nullptr)) {
            std::vector<unsigned long long*> slots;
            for (unsigned long long* b : base) slots.push_back(b + done * per);
            if (int rc = group_pass(g, G, slots)) return rc;
            done += (uint32_t)G;
        }
        if (hashes_out) {
            for (uint32_t k = 0; k < cnt; ++k) hashes_out[g0 + k] = 0;
            part.resize(cnt);
            for (int k = 0; k < n; ++k) {
                gol_ctx* s = g->shards[k];
                if (int rc = bind(s)) return group_fail(g, s, rc);
                hipError_t e = hipMemcpyAsync(s->host_slots.data(), s->slots, cnt * per * sizeof(unsigned long long),
                                              hipMemcpyDeviceToHost, s->compute);
                if (e == hipSuccess) e = hipStreamSynchronize(s->compute);
                if (e != hipSuccess) return group_fail(g, s, hip_fail(s, e, "hash readback", __FILE__, __LINE__));
                fold_slots(s, cnt, part.data());
                for (uint32_t j = 0; j < cnt; ++j) hashes_out[g0 + j] += part[j];
                if (partials_out)
                    std::copy(part.begin(), part.end(), partials_out + (size_t)k * generations + g0);
            }
        }
    }
    return GOL_OK;
}

int gol_group_sync(gol_group* g) {
    if (!g) return set_err(nullptr, GOL_EINVAL, "null group");
    for (gol_ctx* s : g->shards) {
        if (!s) continue;
        if (int rc = gol_sync(s)) return group_fail(g, s, rc);
    }
    return GOL_OK;
}

void gol_group_destroy(gol_group* g) {
    if (!g) return;
    for (gol_ctx* s : g->shards) {
        if (!s) continue;
        hip_note(hipSetDevice(s->device), "group destroy: hipSetDevice");
        hip_note(hipStreamSynchronize(s->comm), "group destroy: hipStreamSynchronize");
        hip_note(hipStreamSynchronize(s->compute), "group destroy: hipStreamSynchronize");
        s->group = nullptr;
        s->gindex = 0;
    }
    delete g;
}

}  // extern "C"
