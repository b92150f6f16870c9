// device_exchange.hip -- the slice-sharded prepass's collective and the
// framebuffer reduce for ranks that are the GPUs of ONE process (the Mitsuba
// plugin's amdDevices: one library integrator per GPU, one host thread each;
// the reference keeps a render in one process with a worker per core,
// src/mitsuba/mitsuba.cpp:280-282, src/librender/renderproc.cpp:119-160).
//
// One RCCL communicator per device from ncclCommInitAll, so the bytes move
// over xGMI between the devices' HBM:
//   * allgather (alvrl_exchange): the rank's host buffer is staged on its
//     device, ncclAllGather, the world * bytes copied back -- the non-zero
//     mask OR and the cluster-list merge of alvrl_integrator_prepass_dist;
//   * alvrl_device_exchange_reduce_frame: ncclReduce (sum) of the ranks'
//     framebuffers into rank 0's, in place; the tiles partition the frame, so
//     every pixel is its owner's value plus zeros, bit for bit.
// RCCL rejects a device listed twice: a one-GPU rehearsal of several ranks
// uses alvrl_local_exchange (host memory) instead.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "alvrl.h"
#include "alvrl_host.h"

namespace alvrl {
namespace host {
extern thread_local std::string g_host_err;
}
}  // namespace alvrl
using alvrl::host::g_host_err;

struct alvrl_device_exchange {
    struct Rank {
        alvrl_device_exchange* g = nullptr;
        uint32_t r = 0;
        int device = 0;
        ncclComm_t comm = nullptr;
        hipStream_t stream = nullptr;
        uint8_t* d_send = nullptr;   // grow-only staging of allgather
        uint8_t* d_recv = nullptr;
        uint64_t cap_send = 0, cap_recv = 0;
    };
    uint32_t world = 0;
    std::vector<Rank> ranks;
    std::vector<alvrl_exchange> ex;

    static int grow(uint8_t** p, uint64_t* cap, uint64_t n)
    {
        if (n <= *cap) return 0;
        if (*p) (void)hipFree(*p);
        *p = nullptr;
        *cap = 0;
        if (hipMalloc(p, n) != hipSuccess) return 1;
        *cap = n;
        return 0;
    }

    // every rank passes the same byte count and gets world * bytes in rank order
    static int allgather(void* user, const void* send, uint64_t bytes, void* recv)
    {
        Rank* rk = static_cast<Rank*>(user);
        const alvrl_device_exchange& G = *rk->g;
        if (bytes == 0) return 0;   // every rank skips (the byte count is common)
        if (!rk->comm) return 2;    // aborted group
        if (hipSetDevice(rk->device) != hipSuccess) return 1;
        if (grow(&rk->d_send, &rk->cap_send, bytes) || grow(&rk->d_recv, &rk->cap_recv, bytes * G.world)) return 1;
        if (hipMemcpyAsync(rk->d_send, send, bytes, hipMemcpyHostToDevice, rk->stream) != hipSuccess) return 1;
        if (ncclAllGather(rk->d_send, rk->d_recv, bytes, ncclUint8, rk->comm, rk->stream) != ncclSuccess) return 2;
        if (hipMemcpyAsync(recv, rk->d_recv, bytes * G.world, hipMemcpyDeviceToHost, rk->stream) != hipSuccess)
            return 1;
        return hipStreamSynchronize(rk->stream) == hipSuccess ? 0 : 1;
    }

    ~alvrl_device_exchange()
    {
        for (Rank& r : ranks) {
            (void)hipSetDevice(r.device);
            if (r.stream) (void)hipStreamSynchronize(r.stream);
            if (r.comm) (void)ncclCommDestroy(r.comm);
            if (r.d_send) (void)hipFree(r.d_send);
            if (r.d_recv) (void)hipFree(r.d_recv);
            if (r.stream) (void)hipStreamDestroy(r.stream);
        }
    }
};

extern "C" {

ALVRL_API int alvrl_device_exchange_create(const int* devices, uint32_t world, alvrl_device_exchange** out)
{
    if (!out || !devices || world == 0) {
        g_host_err = "alvrl_device_exchange_create: bad argument";
        return ALVRL_ERR_INVALID;
    }
    for (uint32_t i = 0; i < world; i++)
        for (uint32_t j = 0; j < i; j++)
            if (devices[i] == devices[j] || devices[i] < 0) {
                g_host_err = "alvrl_device_exchange_create: devices must be distinct (RCCL); rehearse on one GPU "
                             "with alvrl_local_exchange";
                return ALVRL_ERR_INVALID;
            }
    auto* g = new alvrl_device_exchange();
    g->world = world;
    g->ranks.resize(world);
    g->ex.resize(world);
    std::vector<ncclComm_t> comms(world, nullptr);
    std::vector<int> devs(devices, devices + world);
    const ncclResult_t nr = ncclCommInitAll(comms.data(), (int)world, devs.data());
    if (nr != ncclSuccess) {
        g_host_err = std::string("alvrl_device_exchange_create: ncclCommInitAll: ") + ncclGetErrorString(nr);
        delete g;
        return ALVRL_ERR_COMM;
    }
    for (uint32_t r = 0; r < world; r++) {
        auto& rk = g->ranks[r];
        rk.g = g;
        rk.r = r;
        rk.device = devices[r];
        rk.comm = comms[r];
        if (hipSetDevice(rk.device) != hipSuccess ||
            hipStreamCreateWithFlags(&rk.stream, hipStreamNonBlocking) != hipSuccess) {
            g_host_err = "alvrl_device_exchange_create: stream";
            delete g;
            return ALVRL_ERR_HIP;
        }
        g->ex[r] = alvrl_exchange{&rk, &alvrl_device_exchange::allgather};
    }
    *out = g;
    return ALVRL_OK;
}

ALVRL_API const alvrl_exchange* alvrl_device_exchange_rank(alvrl_device_exchange* g, uint32_t rank)
{
    return (g && rank < g->world) ? &g->ex[rank] : nullptr;
}

ALVRL_API int alvrl_device_exchange_reduce_frame(alvrl_device_exchange* g, uint32_t rank, float* d_fb, uint64_t n,
                                                 void* stream)
{
    if (!g || rank >= g->world || (n && !d_fb)) {
        g_host_err = "alvrl_device_exchange_reduce_frame: bad argument";
        return ALVRL_ERR_INVALID;
    }
    auto& rk = g->ranks[rank];
    if (hipSetDevice(rk.device) != hipSuccess) { g_host_err = "alvrl_device_exchange_reduce_frame: hipSetDevice"; return ALVRL_ERR_HIP; }
    if (n == 0) return ALVRL_OK;
    if (!rk.comm) { g_host_err = "alvrl_device_exchange_reduce_frame: the group was aborted"; return ALVRL_ERR_COMM; }
    const ncclResult_t nr = ncclReduce(d_fb, d_fb, n, ncclFloat, ncclSum, 0, rk.comm,
                                       stream ? static_cast<hipStream_t>(stream) : rk.stream);
    if (nr != ncclSuccess) {
        g_host_err = std::string("alvrl_device_exchange_reduce_frame: ncclReduce: ") + ncclGetErrorString(nr);
        return ALVRL_ERR_COMM;
    }
    return ALVRL_OK;
}

ALVRL_API void alvrl_device_exchange_destroy(alvrl_device_exchange* g) { delete g; }

ALVRL_API void alvrl_device_exchange_abort(alvrl_device_exchange* g)
{
    if (!g) return;
    for (auto& r : g->ranks)
        if (r.comm) {
            (void)ncclCommAbort(r.comm);   // also frees the communicator
            r.comm = nullptr;
        }
}

}  // extern "C"
