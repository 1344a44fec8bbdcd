// gol_group.cpp -- in-process shard groups (gol_group_*): the shards of one
// board in row order, stepped together; each shard's comm stream pulls its
// neighbours' G edge rows (hipMemcpyPeerAsync: the shards may live on
// different GPUs) and the kernels run as in an RCCL-sharded pass.  A
// destroyed shard leaves a hole the group refuses to step past -- the
// analogue of DeathWatch's Terminated (BoardCreator.scala:120-121).
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

}  // namespace

namespace golc {

size_t group_size(const gol_group* g) { return g->shards.size(); }

int64_t group_min_rows(const gol_group* g) {
    int64_t m = INT64_MAX;
    for (const gol_ctx* s : g->shards) m = std::min(m, s->rows);
    return m;
}

}  // namespace golc

extern "C" {

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
                if (int rc = clear_slots(s, cnt)) return group_fail(g, s, rc);
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
                if (int rc = read_hashes(s, cnt, part.data())) return group_fail(g, s, rc);
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
