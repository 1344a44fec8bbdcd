// gol_ctx.h -- libgol's host-side internals shared by the C-ABI units.  Not
// installed; the boundary is include/gol.h.
//
//   gol_capi.cpp       error state, context lifetime, seeding, stepping, hashes,
//                      tuning and the remaining small entry points
//   gol_schedule.cpp   pass planner, band / tail / XCD tuning, kernel launches
//                      of a pass (whole shard, interior and boundary rows)
//   gol_ring.cpp       the ring schedule: RCCL and loopback halo exchange,
//                      one_pass, gol_comm_*
//   gol_group.cpp      in-process shard groups (gol_group_*)
//   gol_checkpoint.cpp snapshots, checkpoints, restore and light-cone replay
//   gol_profile.cpp    kernel timing, the in-kernel clock probe, gol_profile_*
//
// Reference correspondence (src/main/scala/gameoflife/ of the reference):
//   gol_create   <- BoardCreator.createAllInitialActors (BoardCreator.scala:79-89)
//   gol_seed     <- initialState = Random.nextBoolean() per cell (BoardCreator.scala:23)
//   gol_step     <- NextStep tick -> CurrentEpochMsg -> gatherer -> SetNewStateMsg
//                   (BoardCreator.scala:113-116, CellActor.scala:63-91,
//                    NextStateCellGathererActor.scala:25-48)
//   gol_snapshot <- CellStateMsg -> LoggerActor (CellActor.scala:89, LoggerActor.scala:30-46)
//   gol_comm_*   <- cross-backend GetStateFromEpoch/StateForEpoch over Akka remote
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/gol.h"
#include "gol_kernels.h"

struct LoopRing;  // gol_ring.cpp

// In-process shard group: shards in row order, linked into a ring (torus) or
// a chain (clipped); each shard's comm stream pulls its neighbours' edge rows.
struct gol_group {
    std::vector<gol_ctx*> shards;
    bool torus = true;
    std::string err;
};

#pragma GCC visibility push(hidden)
namespace golc {

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

}  // namespace golc
#pragma GCC visibility pop

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
    uint32_t slots_clean = 0;  // leading generations of `slots` known to be zero (left so by read_hashes)
    unsigned long long* host_folded = nullptr;      // [slots_gens] page-locked, mapped: per-generation sums
    unsigned long long* host_folded_dev = nullptr;  // ... its device address (fold_kernel stores there)
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
    std::vector<golc::EventPair> evs;
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
    mutable std::map<int, int64_t> occupancy_cache;  // resident_waves (a cache: const callers may fill it)
    std::string err;
};

#pragma GCC visibility push(hidden)
namespace golc {

// ---- errors and HIP / RCCL status discipline (gol_capi.cpp) ----------------

int set_err(gol_ctx* ctx, int code, const char* fmt, ...);

// HIP status discipline: a failing HIP call also
// leaves its status pending on the calling thread (hipGetLastError).  A
// failure libgol reports through its own return code is taken off the
// thread here, so no later call -- ours or the caller's -- inherits it.
int hip_fail(gol_ctx* ctx, hipError_t e, const char* expr, const char* file, int line);

#define HIP_CHECK(ctx, expr)                                                   \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) return golc::hip_fail((ctx), e_, #expr, __FILE__, __LINE__); \
    } while (0)

// A status whose failure only gets logged (teardown, best-effort calls):
// reported on stderr and taken off the thread.
void hip_note(hipError_t e, const char* what);

// RCCL runs HIP calls of its own on the calling thread and does not take the
// statuses it discards off the thread: after every RCCL call libgol makes,
// such a leftover is taken, counted and logged once (gol_diag_absorbed).
void absorb_rccl_status(const char* call, hipError_t pending_before);

#define NCCL_CHECK(ctx, expr)                                                                       \
    do {                                                                                            \
        const hipError_t pre_ = hipPeekAtLastError();                                               \
        ncclResult_t r_ = (expr);                                                                   \
        golc::absorb_rccl_status(#expr, pre_);                                                      \
        if (r_ != ncclSuccess)                                                                      \
            return golc::set_err((ctx), GOL_ECOMM, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(r_), \
                                 __FILE__, __LINE__);                                               \
    } while (0)

// ---- context state (gol_capi.cpp) ------------------------------------------

// Any attached communicator runs the ring schedule, a 1-rank one included.
bool sharded(const gol_ctx* c);
bool in_ring(const gol_ctx* c);
// The B3/S23 torus: the only boards the fast-path kernel instances serve.
bool life_torus(const gol_ctx* c);
int bind(gol_ctx* ctx);
int device_ilv(int32_t topology, int64_t wwords);
void destroy_impl(gol_ctx* c);

// ---- pass schedule (gol_schedule.cpp) --------------------------------------

int ensure_slots(gol_ctx* ctx, uint32_t gens);
// Before a hashed chunk: the first `gens` generations' accumulators zero
// (a memset unless read_hashes left them so); marks them in use.
int clear_slots(gol_ctx* ctx, uint32_t gens);
// After the chunk's passes on the compute stream: its `gens` generations'
// hashes into out[], folded on the device straight into mapped host memory,
// the accumulators cleared again; synchronises.
int read_hashes(gol_ctx* ctx, uint32_t gens, uint64_t* out);
int lane_words(const gol_ctx* ctx, int gens);
int64_t resident_waves(const gol_ctx* ctx, int vec, int gens, bool life, bool hash, bool clipped);
// Load every step kernel instance the context can launch at its current
// tuning (the occupancy query of an instance loads its code object).
void preload_instances(gol_ctx* ctx);

// Rows of the plane a launch steps and the global row of its local row 0:
// the context's own (default), or gol_replay's extended block.
struct PlaneGeom {
    int32_t rows;
    int64_t grow0;
};

int launch_ranges(gol_ctx* ctx, int gens, const uint32_t* cur, uint32_t* nxt, const uint32_t* htop,
                  const uint32_t* hbot, int64_t halo_stride, bool wrap_y, unsigned long long* slots, int n,
                  const int32_t* lo, const int32_t* hi, int prof_kind, hipStream_t stream = nullptr,
                  const PlaneGeom* geom = nullptr);
int sharded_interior(gol_ctx* ctx, int G, unsigned long long* slots, bool has_up, bool has_down);
int sharded_boundary(gol_ctx* ctx, int G, unsigned long long* slots, bool has_up, bool has_down,
                     const hipEvent_t* halo_ready, int nready);
int sharded_pass_kernels(gol_ctx* ctx, int G, unsigned long long* slots, bool has_up, bool has_down,
                         const hipEvent_t* halo_ready, int nready);
int depth_cap(const gol_ctx* ctx);
std::vector<int> plan_passes(const gol_ctx* ctx, uint32_t n, bool hashed);

// ---- ring schedule (gol_ring.cpp) ------------------------------------------

// One point-to-point operation of a pass's halo exchange: send `count`
// words from `buf` to rank `peer`, or receive them into `buf` from it.
struct HaloOp {
    bool send;
    uint32_t* buf;
    size_t count;
    int peer;
};

int one_pass(gol_ctx* ctx, int G, unsigned long long* slots);
void loop_leave(gol_ctx* ctx);

// ---- shard groups (gol_group.cpp) ------------------------------------------

size_t group_size(const gol_group* g);
int64_t group_min_rows(const gol_group* g);

// ---- profiling (gol_profile.cpp) -------------------------------------------

EventPair* next_event_pair(gol_ctx* ctx);
int fold_profile(gol_ctx* ctx);

// ---- checkpoints (gol_checkpoint.cpp) --------------------------------------

struct CkptHeader {
    char magic[8];  // "GOLCKPT1"
    int64_t width, height, row0, rows;
    int64_t wwords;
    uint64_t epoch;
    int32_t topology;
    uint32_t birth, survive;
    int32_t pad;
};

}  // namespace golc
#pragma GCC visibility pop
