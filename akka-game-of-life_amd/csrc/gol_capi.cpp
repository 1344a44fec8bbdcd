// gol_capi.cpp -- C ABI of libgol (include/gol.h): error state, context
// lifetime, seeding and loading, stepping (gol_step: the pass plan of
// gol_schedule.cpp run by gol_ring.cpp's one_pass), state hashes, tuning and
// the small host-side entry points.  The other entry points live in
// gol_ring.cpp, gol_group.cpp, gol_checkpoint.cpp and gol_profile.cpp; the
// unit map and the reference correspondence are in gol_ctx.h.
#include <dlfcn.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "gol_ctx.h"

namespace {

std::mutex g_err_mu;
std::string g_err;  // process-wide last error (gol_create failures)

// RCCL leftovers absorbed after libgol's RCCL calls (absorb_rccl_status).
std::mutex g_absorb_mu;
uint64_t g_absorbed = 0;
std::string g_absorbed_last;
std::map<std::string, int> g_absorb_seen;

}  // namespace

namespace golc {

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

int hip_fail(gol_ctx* ctx, hipError_t e, const char* expr, const char* file, int line) {
    (void)hipGetLastError();
    return set_err(ctx, GOL_EHIP, "%s failed: %s (%s:%d)", expr, hipGetErrorString(e), file, line);
}

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
//
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
    if (c->host_folded) hip_note(hipHostFree(c->host_folded), "destroy: hipHostFree");
    for (hipStream_t st : {c->compute, c->comm, c->edge, c->xfer})
        if (st) hip_note(hipStreamDestroy(st), "destroy: hipStreamDestroy");
    delete c;
}

}  // namespace golc

using namespace golc;

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
    // caller's timed region (gol_set_tuning repeats this when it changes the
    // lane width).
    preload_instances(ctx);
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
        if (int rc = clear_slots(ctx, n)) return rc;
        uint32_t g = 0;
        for (const int G : plan_passes(ctx, n, true)) {
            if (int rc = one_pass(ctx, G, ctx->slots + g * per)) return rc;
            g += (uint32_t)G;
        }
        if (int rc = read_hashes(ctx, n, hashes_out + g0)) return rc;
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
    if (int rc = clear_slots(ctx, 1)) return rc;
    HIP_CHECK(ctx, gol::launch_hash(ctx->plane[ctx->cur], ctx->pitch, ctx->wwords, ctx->row0, (int32_t)ctx->rows,
                                    ctx->ilv, ctx->slots, ctx->compute));
    return read_hashes(ctx, 1, hash_out);
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
    const bool lanes_changed = ctx->vec_fixed != words_per_lane;
    ctx->vec_fixed = words_per_lane;
    // a new lane width selects other instances: load them now, not inside the
    // caller's first (timed) step
    if (lanes_changed) {  // the occupancy queries load the code objects; nothing to wait for on the device
        if (int rc = bind(ctx)) return rc;
        preload_instances(ctx);
    }
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
    if (strip_words)
        *strip_words = gol::whole_row_fits(vec, gens_per_pass, life, clipped, ctx->ilv, ctx->topology == GOL_TORUS,
                                           ctx->wwords)
                           ? gol::kWaveLanes * vec  // whole-row waves: no halo lanes
                           : gol::strip_words(vec, gens_per_pass);
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

}  // extern "C"
