// exchange.cpp -- see exchange.hpp.
//
// Wire format of one rank's cluster lists (merge_clusters): a sequence of
//   u32 slice, u32 refined, u32 count, count x u32 rep, count x f32 weight
// for each slice the rank refined.  Slices are dealt to ranks by the caller;
// every slice must be reported by at most one rank.
#include "exchange.hpp"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>

#include "../../../include/alvrl.h"

namespace alvrl {
namespace host {

namespace {
void call(const alvrl_exchange& ex, const void* send, uint64_t bytes, void* recv)
{
    if (!ex.allgather) throw CommError(ALVRL_ERR_INVALID, "alvrl_exchange: no allgather callback");
    const int rc = ex.allgather(ex.user, send, bytes, recv);
    if (rc != 0) throw CommError(ALVRL_ERR_COMM, "alvrl_exchange: allgather callback failed (" + std::to_string(rc) + ")");
}

template <class T>
void put(std::vector<uint8_t>* b, const T& v)
{
    const size_t o = b->size();
    b->resize(o + sizeof(T));
    std::memcpy(b->data() + o, &v, sizeof(T));
}

template <class T>
T get(const uint8_t* p, uint64_t n, uint64_t* at)
{
    if (*at + sizeof(T) > n) throw CommError(ALVRL_ERR_COMM, "alvrl_exchange: truncated cluster message");
    T v;
    std::memcpy(&v, p + *at, sizeof(T));
    *at += sizeof(T);
    return v;
}
}  // namespace

std::vector<uint64_t> allgather_counts(const alvrl_exchange& ex, uint32_t world, uint64_t bytes)
{
    std::vector<uint64_t> counts(world, 0);
    if (world == 1) { counts[0] = bytes; return counts; }
    call(ex, &bytes, sizeof(bytes), counts.data());
    return counts;
}

std::vector<uint8_t> allgatherv(const alvrl_exchange& ex, uint32_t world, const void* send, uint64_t bytes,
                                std::vector<uint64_t>* counts_out)
{
    const std::vector<uint64_t> counts = allgather_counts(ex, world, bytes);
    if (counts_out) *counts_out = counts;
    uint64_t mx = 0, total = 0;
    for (uint64_t c : counts) { mx = std::max(mx, c); total += c; }
    std::vector<uint8_t> out(total);
    if (world == 1) {
        if (bytes) std::memcpy(out.data(), send, bytes);
        return out;
    }
    if (mx == 0) return out;
    // pad every rank's message to the largest, gather, compact
    std::vector<uint8_t> pad(mx, 0), all((size_t)mx * world);
    if (bytes) std::memcpy(pad.data(), send, bytes);
    call(ex, pad.data(), mx, all.data());
    uint64_t at = 0;
    for (uint32_t r = 0; r < world; r++) {
        if (counts[r]) std::memcpy(out.data() + at, all.data() + (size_t)r * mx, counts[r]);
        at += counts[r];
    }
    return out;
}

void or_reduce(const alvrl_exchange& ex, uint32_t world, uint8_t* buf, uint64_t n)
{
    if (world == 1 || n == 0) return;
    std::vector<uint8_t> all((size_t)n * world);
    call(ex, buf, n, all.data());
    for (uint32_t r = 0; r < world; r++) {
        const uint8_t* p = all.data() + (size_t)r * n;
        for (uint64_t i = 0; i < n; i++) buf[i] |= p[i];
    }
}

SliceClusters merge_clusters(const alvrl_exchange& ex, uint32_t world, uint32_t nslices, uint32_t n_local,
                             const uint32_t* local_slice, const int* local_refined, const uint32_t* local_off,
                             const uint32_t* local_reps, const float* local_w)
{
    std::vector<uint8_t> msg;
    for (uint32_t k = 0; k < n_local; k++) {
        const uint32_t cnt = local_off[k + 1] - local_off[k];
        put<uint32_t>(&msg, local_slice[k]);
        put<uint32_t>(&msg, local_refined[k] ? 1u : 0u);
        put<uint32_t>(&msg, cnt);
        for (uint32_t i = 0; i < cnt; i++) put<uint32_t>(&msg, local_reps[local_off[k] + i]);
        for (uint32_t i = 0; i < cnt; i++) put<float>(&msg, local_w[local_off[k] + i]);
    }
    const std::vector<uint8_t> all = allgatherv(ex, world, msg.data(), msg.size(), nullptr);
    // per slice: where its record starts in 'all'
    std::vector<uint64_t> where(nslices, UINT64_MAX);
    std::vector<uint32_t> cnt(nslices, 0);
    std::vector<int> refined(nslices, 0);
    uint64_t at = 0;
    const uint64_t n = all.size();
    while (at < n) {
        const uint32_t s = get<uint32_t>(all.data(), n, &at);
        const uint32_t ref = get<uint32_t>(all.data(), n, &at);
        const uint32_t c = get<uint32_t>(all.data(), n, &at);
        if (s >= nslices) throw CommError(ALVRL_ERR_COMM, "alvrl_exchange: slice id out of range");
        if (where[s] != UINT64_MAX) throw CommError(ALVRL_ERR_COMM, "alvrl_exchange: slice reported twice");
        if (at + (uint64_t)c * 8 > n) throw CommError(ALVRL_ERR_COMM, "alvrl_exchange: truncated cluster message");
        where[s] = at;
        cnt[s] = c;
        refined[s] = ref ? 1 : 0;
        at += (uint64_t)c * 8;
    }
    SliceClusters out;
    out.refined = refined;
    out.off.assign(nslices + 1, 0);
    for (uint32_t s = 0; s < nslices; s++) out.off[s + 1] = out.off[s] + cnt[s];
    out.reps.resize(out.off[nslices]);
    out.w.resize(out.off[nslices]);
    for (uint32_t s = 0; s < nslices; s++) {
        if (!cnt[s]) continue;
        std::memcpy(out.reps.data() + out.off[s], all.data() + where[s], (size_t)cnt[s] * 4);
        std::memcpy(out.w.data() + out.off[s], all.data() + where[s] + (uint64_t)cnt[s] * 4, (size_t)cnt[s] * 4);
    }
    return out;
}

}  // namespace host
}  // namespace alvrl

using namespace alvrl::host;

namespace alvrl {
namespace host {
extern thread_local std::string g_host_err;
}
}  // namespace alvrl

#define XGUARD(...)                                         \
    try {                                                   \
        __VA_ARGS__;                                        \
    } catch (const CommError& e) {                          \
        g_host_err = e.what();                              \
        return e.code;                                      \
    } catch (const std::exception& e) {                     \
        g_host_err = e.what();                              \
        return ALVRL_ERR_INVALID;                           \
    }

extern "C" {

ALVRL_API int alvrl_exchange_allgatherv(const alvrl_exchange* ex, uint32_t world, const void* send,
                                        uint64_t bytes, void* recv, uint64_t cap, uint64_t* counts)
{
    if (!ex || world == 0 || !counts || (bytes && !send)) {
        g_host_err = "alvrl_exchange_allgatherv: bad argument";
        return ALVRL_ERR_INVALID;
    }
    XGUARD({
        if (!recv) {
            const std::vector<uint64_t> c = allgather_counts(*ex, world, bytes);
            std::copy(c.begin(), c.end(), counts);
            return ALVRL_OK;
        }
        std::vector<uint64_t> c;
        const std::vector<uint8_t> all = allgatherv(*ex, world, send, bytes, &c);
        std::copy(c.begin(), c.end(), counts);
        if (all.size() > cap) {
            g_host_err = "alvrl_exchange_allgatherv: buffer too small";
            return ALVRL_ERR_INVALID;
        }
        if (!all.empty()) std::memcpy(recv, all.data(), all.size());
    });
    return ALVRL_OK;
}

ALVRL_API int alvrl_exchange_or(const alvrl_exchange* ex, uint32_t world, uint8_t* buf, uint64_t n)
{
    if (!ex || world == 0 || (n && !buf)) {
        g_host_err = "alvrl_exchange_or: bad argument";
        return ALVRL_ERR_INVALID;
    }
    XGUARD(or_reduce(*ex, world, buf, n));
    return ALVRL_OK;
}

ALVRL_API int alvrl_exchange_clusters(const alvrl_exchange* ex, uint32_t world, uint32_t nslices,
                                      uint32_t n_local, const uint32_t* local_slice,
                                      const int* local_refined, const uint32_t* local_off,
                                      const uint32_t* local_reps, const float* local_w, int* refined,
                                      uint32_t* slice_off, uint32_t* reps, float* weights, uint64_t cap,
                                      uint64_t* total)
{
    if (!ex || world == 0 || !refined || !slice_off || !total ||
        (n_local && (!local_slice || !local_refined || !local_off))) {
        g_host_err = "alvrl_exchange_clusters: bad argument";
        return ALVRL_ERR_INVALID;
    }
    XGUARD({
        const SliceClusters m = merge_clusters(*ex, world, nslices, n_local, local_slice, local_refined,
                                               local_off, local_reps, local_w);
        *total = m.reps.size();
        std::copy(m.refined.begin(), m.refined.end(), refined);
        std::copy(m.off.begin(), m.off.end(), slice_off);
        if (m.reps.size() > cap || (!m.reps.empty() && (!reps || !weights))) {
            g_host_err = "alvrl_exchange_clusters: buffer too small";
            return ALVRL_ERR_INVALID;
        }
        std::copy(m.reps.begin(), m.reps.end(), reps);
        std::copy(m.w.begin(), m.w.end(), weights);
    });
    return ALVRL_OK;
}

/* ---- the in-process exchange: one thread per device, one process ------ */
}  // extern "C"

// Ranks are threads of this process (the Mitsuba plugin's amdDevices: one
// library integrator per GPU, renderproc.cpp:119-135 / mitsuba.cpp:280-282
// keep everything in one process).  allgather: every rank posts its send
// buffer, the last to arrive opens the round, each copies all posted buffers
// into its own recv, and a second barrier keeps every send buffer alive until
// all ranks have copied.  A rank that waits longer than the timeout fails the
// call (and so the prepass) instead of hanging.
struct alvrl_local_exchange {
    uint32_t world = 0;
    std::mutex mu;
    std::condition_variable cv;
    uint64_t gen = 0;           // rounds completed (two barriers per allgather)
    uint32_t arrived = 0;
    uint64_t bytes = 0;
    bool broken = false;
    std::vector<const void*> send;
    std::vector<alvrl_exchange> ex;
    struct Rank { alvrl_local_exchange* g; uint32_t r; };
    std::vector<Rank> ranks;
    double timeout_s = 600.0;

    // barrier; false on timeout or a broken group
    bool arrive(std::unique_lock<std::mutex>& lk)
    {
        if (broken) return false;
        const uint64_t g0 = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(lk, std::chrono::duration<double>(timeout_s),
                                    [&] { return gen != g0 || broken; });
        if (!ok || broken) { broken = true; cv.notify_all(); return false; }
        return true;
    }

    static int allgather(void* user, const void* snd, uint64_t n, void* recv)
    {
        Rank* rk = static_cast<Rank*>(user);
        alvrl_local_exchange& G = *rk->g;
        std::unique_lock<std::mutex> lk(G.mu);
        if (G.arrived == 0) G.bytes = n;
        else if (G.bytes != n) { G.broken = true; G.cv.notify_all(); return 2; }
        G.send[rk->r] = snd;
        if (!G.arrive(lk)) return 1;
        lk.unlock();
        for (uint32_t q = 0; q < G.world; q++)
            if (n) std::memcpy(static_cast<uint8_t*>(recv) + (size_t)q * n, G.send[q], n);
        lk.lock();
        return G.arrive(lk) ? 0 : 1;
    }
};

extern "C" {

ALVRL_API int alvrl_local_exchange_create(uint32_t world, alvrl_local_exchange** out)
{
    if (!out || world == 0) { g_host_err = "alvrl_local_exchange_create: bad argument"; return ALVRL_ERR_INVALID; }
    alvrl_local_exchange* g = new alvrl_local_exchange();
    g->world = world;
    g->send.assign(world, nullptr);
    g->ranks.resize(world);
    g->ex.resize(world);
    for (uint32_t r = 0; r < world; r++) {
        g->ranks[r] = alvrl_local_exchange::Rank{g, r};
        g->ex[r] = alvrl_exchange{&g->ranks[r], &alvrl_local_exchange::allgather};
    }
    *out = g;
    return ALVRL_OK;
}

ALVRL_API const alvrl_exchange* alvrl_local_exchange_rank(alvrl_local_exchange* g, uint32_t rank)
{
    return (g && rank < g->world) ? &g->ex[rank] : nullptr;
}

ALVRL_API void alvrl_local_exchange_destroy(alvrl_local_exchange* g) { delete g; }

ALVRL_API void alvrl_local_exchange_abort(alvrl_local_exchange* g)
{
    if (!g) return;
    std::lock_guard<std::mutex> lk(g->mu);
    g->broken = true;
    g->cv.notify_all();
}

}  // extern "C"
