// gol_profile.cpp -- kernel timing of a context (gol_profile_*): HIP event
// pairs around the dominant launch of every pass (and, on a ring, around the
// halo exchange and the boundary launch), folded into running totals, and the
// in-kernel clock probe (gol_stencil.h clock_probe_*) each timed launch
// writes into its own slot.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "gol_ctx.h"

namespace {

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

}  // namespace

namespace golc {

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

}  // namespace golc

using namespace golc;

extern "C" {

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

}  // extern "C"
