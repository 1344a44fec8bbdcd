// gol_checkpoint.cpp -- the board leaving and re-entering a context:
// snapshots (synchronous, and asynchronous on the transfer stream while later
// passes run), shard checkpoints and restore, and gol_replay -- a restored
// block stepped alone through its light cone, the re-spawn path of
// BoardCreator.scala:120-154 (CellActor.scala:34,71-74,86 is the history
// replay it stands for).  The LoggerActor path (CellActor.scala:89,
// LoggerActor.scala:30-46) reads snapshots.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "gol_ctx.h"

using namespace golc;

namespace {

// Asynchronous snapshot: the board is copied on the device (de-interleaved
// for the pair layout) into `snap` in the compute stream's order -- so later
// passes cannot overwrite it first -- and from there to the host on the
// transfer stream, concurrently with the passes queued after it.
constexpr size_t kSnapChunkBytes = 256ull << 20;

}  // namespace

extern "C" {

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
        if (int rc = clear_slots(ctx, generations)) return rc;
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
    if (e != hipSuccess) return fail_hip(e, "light-cone result");
    if (hashes_out) {
        if (int rc = read_hashes(ctx, generations, hashes_out)) {  // synchronises
            release();
            return rc;
        }
    }
    e = hipStreamSynchronize(ctx->compute);
    if (e != hipSuccess) return fail_hip(e, "light-cone result");
    release();
    ctx->epoch += (uint64_t)n;
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

}  // extern "C"
