// gol_ring.cpp -- the ring schedule of a sharded context: one pass of G
// generations = the interior rows' launch || a G-deep halo exchange with the
// ring neighbours (one RCCL send/recv group on the comm stream, or the
// in-process loopback ring that tests use in its place), then the boundary
// rows.  Replaces the cross-backend GetStateFromEpoch / StateForEpoch traffic
// of the reference (CellActor.scala:71-77, NextStateCellGathererActor.scala:32-36).
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>
#include <chrono>
#include <condition_variable>
#include <deque>

#include "gol_ctx.h"

using namespace golc;

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

}  // namespace

namespace golc {

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

}  // namespace golc

extern "C" {

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

}  // extern "C"
