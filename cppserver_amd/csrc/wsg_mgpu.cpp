// wsg_mgpu.cpp — the multi-GPU entry of the C-ABI:
// a batch of frames sharded round-robin over the GPUs of a node, encoded
// where it lies, and the framed output gathered to one rank over RCCL/xGMI
// (BASELINE config C5).
//
// Frames are independent (a frame's key phase is the offset inside its own
// payload), so the only exchange is the gather.  Chunks of `chunk`
// consecutive frames are dealt round-robin, chunk c to rank c % world; a
// rank's local batch is its chunks in order.  Every rank encodes its batch
// with wsg_encode_batch, the ranks learn each other's chunk byte sizes (one
// small all-gather), and one grouped set of point-to-point transfers moves
// every chunk straight to its place in the root's output (each sender on its
// own xGMI link into the root), together with the chunk's frame offsets,
// which one kernel on the root rebases into the job's wire offsets.
//
// Two ways to build the communicator:
//   wsg_mgpu_create      one process drives several GPUs (ncclCommInitAll),
//                        e.g. a C++ server owning the node;
//   wsg_mgpu_create_rank one rank per process (ncclCommInitRank), the
//                        torch.distributed layout of bench.py; the caller
//                        moves the 128-byte id from rank 0 to the others.
//
// RCCL is loaded at run time (dlopen, RTLD_LOCAL) from $WSG_RCCL_LIB or the
// ROCm install, so that a host process which already carries another RCCL
// (PyTorch bundles one) keeps the two apart.
#include "wsg_internal.h"
#include "wsg_env.h"
#include "wsg_trace.h"

#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <type_traits>
#include <vector>

namespace {

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
};

const Rccl* rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* names[] = {wsg::envp("WSG_RCCL_LIB"), "/opt/rocm/lib/librccl.so.1", "librccl.so.1",
                               "librccl.so"};
        for (const char* n : names) {
            if (!n || !*n)
                continue;
            r.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
            if (r.h)
                break;
        }
        if (!r.h)
            return;
        auto sym = [](auto& fn, const char* name) { fn = reinterpret_cast<std::decay_t<decltype(fn)>>(dlsym(r.h, name)); };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommInitAll, "ncclCommInitAll");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.AllGather, "ncclAllGather");
    });
    const bool ok = r.h && r.GetUniqueId && r.CommInitRank && r.CommInitAll && r.CommDestroy && r.GroupStart &&
                    r.GroupEnd && r.Send && r.Recv && r.AllGather;
    return ok ? &r : nullptr;
}

#define WSG_HIP(expr)                                                                                        \
    do {                                                                                                     \
        if ((expr) != hipSuccess)                                                                            \
            return WSG_EHIP;                                                                                 \
    } while (0)
#define WSG_NCCL(expr)                                                                                       \
    do {                                                                                                     \
        if ((expr) != ncclSuccess)                                                                           \
            return WSG_EHIP;                                                                                 \
    } while (0)

// Test hook ($WSG_TEST_NULL_SPIN_US; tests/test_gpu_c5.py::
// test_mgpu_rank_form_copy_ordering): before each host->device round of the
// gather and before its transfers, park the device's null stream for that
// long.  Plain hipMemcpy / hipMemset calls go to the null stream, which the
// contexts' non-blocking streams do not wait for, so a copy that is not
// ordered on the stream its consumer runs on lands after that consumer every
// time instead of rarely.  Unset (the product): nothing is launched.
uint32_t test_null_spin_us()
{
    static const uint32_t us = [] {
        const char* e = wsg::envp("WSG_TEST_NULL_SPIN_US");
        return e ? uint32_t(std::strtoul(e, nullptr, 10)) : 0u;
    }();
    return us;
}

void test_park_null_stream(int device)
{
    if (const uint32_t us = test_null_spin_us())
        if (hipSetDevice(device) == hipSuccess)
            (void)wsg::launch_test_spin(nullptr, us);
}

inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// frames owned by `rank`: chunks r, r + world, ... of `chunk` frames each
uint64_t shard_count(uint64_t n_total, uint32_t chunk, int world, int rank)
{
    const uint64_t n_chunks = ceil_div(n_total, chunk);
    if (uint64_t(rank) >= n_chunks)
        return 0;
    const uint64_t mine = (n_chunks - 1 - uint64_t(rank)) / uint64_t(world) + 1;
    uint64_t frames = mine * chunk;
    const uint64_t last = n_chunks - 1;   // the only short chunk
    if (last % uint64_t(world) == uint64_t(rank))
        frames -= last * chunk + chunk - n_total;
    return frames;
}

struct Local {
    int device = 0;
    int rank = 0;
    wsg_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    uint64_t* d_sizes = nullptr;   // this rank's chunk sizes | every rank's (all-gather)
    uint64_t sizes_cap = 0;
    uint64_t* d_status = nullptr;  // rank form: status all-gather (1 + world words, made at create)
    uint64_t* d_stage = nullptr;   // root: every rank's local frame offsets, rank by rank (n_total)
    uint64_t stage_cap = 0;
    uint64_t* d_goff = nullptr;    // root: global offset of every chunk, then every rank's stage base
    uint64_t goff_cap = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr, e3 = nullptr;   // encode start/end, gather end/start
    hipEvent_t done = nullptr;     // one-process form: this rank's transfers to the root are queued before it
};

template <class T>
int grow(T*& p, uint64_t& cap, uint64_t want)
{
    want = std::max<uint64_t>(want, 1);
    if (want <= cap)
        return WSG_OK;
    if (p)
        WSG_HIP(hipFree(p));
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, want * sizeof(T)) != hipSuccess)
        return WSG_ENOMEM;
    cap = want;
    return WSG_OK;
}

// Runs of a host batch split over `parts` contexts: run k is frames
// [cut[k], cut[k + 1]), about wire_len / parts wire bytes each, cut at frame
// starts.  Every cut is a frame starting inside the wire (frames starting at
// or past its end stay with the last run) and run 0 holds frame 0, so run k
// covers wire bytes [k ? fs[cut[k]] : 0, cut[k + 1] < n ? fs[cut[k + 1]] : wire_len).
std::vector<uint32_t> host_runs(const uint64_t* fs, uint32_t n, uint64_t wire_len, int parts)
{
    std::vector<uint32_t> cut(size_t(parts) + 1, n);
    cut[0] = 0;
    const uint32_t inside = uint32_t(std::lower_bound(fs, fs + n, wire_len) - fs);
    for (int k = 1; k < parts; ++k) {
        const uint64_t target = uint64_t(double(wire_len) * k / parts);
        uint32_t idx = uint32_t(std::lower_bound(fs, fs + inside, target) - fs);
        idx = std::max<uint32_t>(idx, 1);
        if (idx >= inside)
            idx = n;   // no frame starts inside the wire past the target
        cut[size_t(k)] = std::max(idx, cut[size_t(k) - 1]);
    }
    return cut;
}

// Run fn(i) for i in [0, parts) on threads of their own (i = 0 on the
// caller's), each with ctxs[i]'s device current.  fn must not throw (the
// callers catch inside it); a thread that cannot be started runs its part
// on the caller's thread afterwards.
template <class Fn>
void on_contexts(wsg_ctx* const* ctxs, int parts, Fn fn)
{
    std::vector<std::thread> th;
    std::vector<int> inline_parts;
    for (int i = 1; i < parts; ++i) {
        try {
            th.emplace_back([&, i] {
                (void)hipSetDevice(wsg::ctx_device(ctxs[i]));
                fn(i);
            });
        } catch (...) {
            inline_parts.push_back(i);
        }
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(wsg::ctx_device(ctxs[0]));
    fn(0);
    for (int i : inline_parts) {
        (void)hipSetDevice(wsg::ctx_device(ctxs[i]));
        fn(i);
    }
    (void)hipSetDevice(prev);
    for (auto& t : th)
        t.join();
}

// The contexts a split uses: the first of each device.  Two pipelines on
// one GPU share its PCIe link and copy engines and measured slower than one
// (C2 from pinned memory: 29-40 GiB/s on one context, 15-20 on two or four of
// one device, tools/host_multi.py); $WSG_HOST_MULTI_SHARE=1 keeps every
// context (the one-GPU tests exercise the split that way).
std::vector<wsg_ctx*> one_per_device(wsg_ctx* const* ctxs, int nctx)
{
    const bool share = nctx > 0 && wsg::ctx_multi_share(ctxs[0]);   // (read at wsg_create, not per call)
    std::vector<wsg_ctx*> v;
    std::vector<int> seen;
    for (int i = 0; i < nctx; ++i) {
        const int d = wsg::ctx_device(ctxs[i]);
        if (!share && std::find(seen.begin(), seen.end(), d) != seen.end())
            continue;
        seen.push_back(d);
        v.push_back(ctxs[i]);
    }
    return v;
}

// A per-run status that is not about the frames (HIP, memory) wins; the
// frames' own errors are recomputed over the whole batch.
inline bool frame_status(int rc) { return rc == WSG_OK || rc == WSG_EINVAL || rc == WSG_ETRUNC; }

} // namespace

struct wsg_mgpu {
    int world = 0;
    // wsg_mgpu_create: every rank lives in this process (one or more per
    // device): the exchange is host bookkeeping plus device copies (xGMI
    // peer copies between GPUs, plain copies within one); wsg_mgpu_create_rank:
    // one rank here, the others in their processes, over RCCL
    bool all_local = false;
    std::vector<Local> local;   // ranks driven by this process
};

namespace {

std::vector<wsg_ctx*> local_ctxs(wsg_mgpu* g)
{
    std::vector<wsg_ctx*> v;
    for (Local& l : g->local)
        v.push_back(l.ctx);
    return v;
}

} // namespace

extern "C" {

int wsg_mgpu_unique_id(uint8_t* id)
{
    if (!id)
        return WSG_EINVAL;
    wsg::hip_init_once();
    const Rccl* r = rccl();
    if (!r)
        return WSG_EHIP;
    ncclUniqueId u;
    WSG_NCCL(r->GetUniqueId(&u));
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return WSG_OK;
}

int wsg_mgpu_destroy(wsg_mgpu* g)
{
    if (!g)
        return WSG_EINVAL;
    const Rccl* r = rccl();
    for (Local& l : g->local) {
        (void)hipSetDevice(l.device);
        if (l.comm && r)
            r->CommDestroy(l.comm);
        (void)hipFree(l.d_sizes);
        (void)hipFree(l.d_status);
        (void)hipFree(l.d_stage);
        (void)hipFree(l.d_goff);
        for (hipEvent_t e : {l.e0, l.e1, l.e2, l.e3, l.done})
            if (e)
                (void)hipEventDestroy(e);
        if (l.ctx)
            wsg_destroy(l.ctx);
    }
    delete g;
    return WSG_OK;
}

namespace {

int init_locals(wsg_mgpu* g)
{
    for (Local& l : g->local) {
        if (int rc = wsg_create(l.device, &l.ctx))
            return rc;
        WSG_HIP(hipSetDevice(l.device));
        for (hipEvent_t* e : {&l.e0, &l.e1, &l.e2, &l.e3})
            WSG_HIP(hipEventCreate(e));
        WSG_HIP(hipEventCreateWithFlags(&l.done, hipEventDisableTiming));
        // the status exchange must never fail to allocate (every rank has
        // to reach it, whatever went wrong before)
        if (hipMalloc(&l.d_status, (uint64_t(g->world) + 1) * sizeof(uint64_t)) != hipSuccess)
            return WSG_ENOMEM;
    }
    return WSG_OK;
}

// direct xGMI access between every two distinct devices of the group, where
// the platform offers it (hipMemcpyPeerAsync works either way)
void enable_peers(const int* devices, int ndev)
{
    for (int i = 0; i < ndev; ++i)
        for (int j = 0; j < ndev; ++j) {
            if (devices[i] == devices[j])
                continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, devices[i], devices[j]) != hipSuccess || !can)
                continue;
            if (hipSetDevice(devices[i]) == hipSuccess)
                (void)hipDeviceEnablePeerAccess(devices[j], 0);   // "already enabled" is fine
            (void)hipGetLastError();
        }
}

} // namespace

int wsg_mgpu_create(const int* devices, int ndev, wsg_mgpu** out)
{
    if (!out || !devices || ndev <= 0)
        return WSG_EINVAL;
    wsg::hip_init_once();
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess)
        return WSG_EHIP;
    for (int i = 0; i < ndev; ++i)
        if (devices[i] < 0 || devices[i] >= count)
            return WSG_EINVAL;
    wsg_mgpu* g = new (std::nothrow) wsg_mgpu();
    if (!g)
        return WSG_ENOMEM;
    g->world = ndev;
    g->all_local = true;   // a device may be listed more than once: one rank each
    g->local.resize(size_t(ndev));
    for (int i = 0; i < ndev; ++i) {
        g->local[size_t(i)].device = devices[i];
        g->local[size_t(i)].rank = i;
    }
    if (int rc = init_locals(g)) {
        wsg_mgpu_destroy(g);
        return rc;
    }
    enable_peers(devices, ndev);
    *out = g;
    return WSG_OK;
}

int wsg_mgpu_create_rank(int device, const uint8_t* id, int rank, int world, wsg_mgpu** out)
{
    if (!out || !id || world <= 0 || rank < 0 || rank >= world)
        return WSG_EINVAL;
    wsg::hip_init_once();
    *out = nullptr;
    const Rccl* r = rccl();
    if (!r)
        return WSG_EHIP;
    wsg_mgpu* g = new (std::nothrow) wsg_mgpu();
    if (!g)
        return WSG_ENOMEM;
    g->world = world;
    g->local.resize(1);
    g->local[0].device = device;
    g->local[0].rank = rank;
    if (int rc = init_locals(g)) {
        wsg_mgpu_destroy(g);
        return rc;
    }
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    if (hipSetDevice(device) != hipSuccess || r->CommInitRank(&g->local[0].comm, world, u, rank) != ncclSuccess) {
        wsg_mgpu_destroy(g);
        return WSG_EHIP;
    }
    *out = g;
    return WSG_OK;
}

int wsg_mgpu_info(wsg_mgpu* g, int* world, int* nlocal, int* first_rank)
{
    if (!g)
        return WSG_EINVAL;
    if (world)
        *world = g->world;
    if (nlocal)
        *nlocal = int(g->local.size());
    if (first_rank)
        *first_rank = g->local.empty() ? 0 : g->local[0].rank;
    return WSG_OK;
}

wsg_ctx* wsg_mgpu_ctx(wsg_mgpu* g, int i)
{
    if (!g || i < 0 || size_t(i) >= g->local.size())
        return nullptr;
    return g->local[size_t(i)].ctx;
}

uint64_t wsg_mgpu_shard_count(uint64_t n_total, uint32_t chunk, int world, int rank)
{
    if (chunk == 0 || world <= 0 || rank < 0 || rank >= world)
        return 0;
    return shard_count(n_total, chunk, world, rank);
}

} // extern "C"

namespace {

int encode_gather(wsg_mgpu* g, uint64_t n_total, uint32_t chunk, const uint8_t* const* d_payload,
                  const wsg_send_desc* const* d_desc, const uint32_t* n_local, uint8_t* const* d_wire,
                  const uint64_t* wire_cap, uint64_t* const* d_wire_off, int root, uint8_t* d_out, uint64_t out_cap,
                  uint64_t* d_out_off, double* times)
{
    if (!g || chunk == 0 || root < 0 || root >= g->world || !n_local || !d_wire || !wire_cap || !d_wire_off ||
        !d_payload || !d_desc)
        return WSG_EINVAL;
    const bool all_local = g->all_local;
    const Rccl* r = all_local ? nullptr : rccl();
    if (!all_local && !r)
        return WSG_EHIP;
    const int world = g->world;
    const size_t nl = g->local.size();
    if (n_total == 0) {   // nothing to encode or move, on every rank alike
        for (size_t i = 0; i < nl; ++i)
            if (g->local[i].rank == root && d_out_off) {
                WSG_HIP(hipSetDevice(g->local[i].device));
                hipStream_t s = static_cast<hipStream_t>(wsg_stream(g->local[i].ctx));
                WSG_HIP(hipMemsetAsync(d_out_off, 0, sizeof(uint64_t), s));
                WSG_HIP(hipStreamSynchronize(s));
            }
        if (times)
            times[0] = times[1] = 0.0;
        return WSG_OK;
    }
    const uint64_t n_chunks = ceil_div(n_total, chunk);
    const uint64_t maxq = ceil_div(n_chunks, uint64_t(world));   // chunks per rank, at most
    auto stream_of = [](const Local& l) { return static_cast<hipStream_t>(wsg_stream(l.ctx)); };

    // In the rank-per-process form every rank must reach every collective
    // below, whatever failed locally: local failures go into `status`, which
    // the ranks exchange (exchange_status) before anything depends on it.
    int status = WSG_OK;
    auto fail = [&](int rc) {
        if (rc && !status)
            status = rc;
    };
    auto exchange_status = [&]() -> int {
        if (all_local)
            return status;
        for (Local& l : g->local) {
            test_park_null_stream(l.device);
            WSG_HIP(hipSetDevice(l.device));
            const uint64_t mine = uint64_t(uint32_t(-status));
            // on the stream the all-gather runs on, landed before it (host
            // data into device memory by a plain hipMemcpy is not ordered
            // with the context's non-blocking stream)
            WSG_HIP(hipMemcpyAsync(l.d_status, &mine, sizeof(uint64_t), hipMemcpyHostToDevice, stream_of(l)));
            WSG_HIP(hipStreamSynchronize(stream_of(l)));
        }
        WSG_NCCL(r->GroupStart());
        for (Local& l : g->local)
            WSG_NCCL(r->AllGather(l.d_status, l.d_status + 1, 1, ncclUint64, l.comm, stream_of(l)));
        WSG_NCCL(r->GroupEnd());
        std::vector<uint64_t> st(uint64_t(world), 0);
        Local& l = g->local[0];
        WSG_HIP(hipSetDevice(l.device));
        WSG_HIP(hipStreamSynchronize(stream_of(l)));
        WSG_HIP(hipMemcpy(st.data(), l.d_status + 1, st.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
        for (uint64_t e : st)
            if (e && !status)
                status = -int(e);
        return status;
    };

    Local* root_l = nullptr;
    std::vector<bool> ok(nl, true);
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
        if (uint64_t(n_local[i]) != shard_count(n_total, chunk, world, l.rank)) {
            fail(WSG_EINVAL);   // not this rank's round-robin share of the job
            ok[i] = false;
        }
        if (l.rank == root) {
            root_l = &l;
            if (!d_out)
                fail(WSG_EINVAL);
        }
    }

    // 1. every local rank encodes its shard (concurrently, one stream each)
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
        if (!ok[i] || hipSetDevice(l.device) != hipSuccess) {
            fail(WSG_EINVAL);
            ok[i] = false;
            continue;
        }
        hipStream_t s = stream_of(l);
        if (hipEventRecord(l.e0, s) != hipSuccess)
            fail(WSG_EHIP);
        if (int rc = wsg_encode_batch(l.ctx, d_payload[i], d_desc[i], n_local[i], d_wire[i], wire_cap[i],
                                      d_wire_off[i], s)) {
            fail(rc);
            ok[i] = false;
        }
        if (hipEventRecord(l.e1, s) != hipSuccess)
            fail(WSG_EHIP);
    }
    // 2. each local rank's frame offsets and chunk byte sizes (host); the
    // buffers the exchange needs are made before the status round
    std::vector<std::vector<uint64_t>> loff(nl);
    std::vector<std::vector<uint64_t>> sizes(nl, std::vector<uint64_t>(maxq, 0));
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
        loff[i].assign(size_t(n_local[i]) + 1, 0);
        if (!ok[i] || hipSetDevice(l.device) != hipSuccess)
            continue;
        if (int rc = wsg_sync(l.ctx, stream_of(l))) {
            fail(rc);
            continue;
        }
        if (hipMemcpy(loff[i].data(), d_wire_off[i], loff[i].size() * sizeof(uint64_t), hipMemcpyDeviceToHost) !=
            hipSuccess) {
            fail(WSG_EHIP);
            continue;
        }
        for (uint64_t q = 0; q * chunk < n_local[i]; ++q)
            sizes[i][q] = loff[i][std::min<uint64_t>((q + 1) * chunk, n_local[i])] - loff[i][q * chunk];
        if (!all_local)
            fail(grow(l.d_sizes, l.sizes_cap, maxq * (uint64_t(world) + 1)));
        if (l.rank == root) {
            fail(grow(l.d_stage, l.stage_cap, n_total));
            fail(grow(l.d_goff, l.goff_cap, n_chunks + 1 + uint64_t(world) + 1));
        }
    }
    if (exchange_status())
        return status;

    // 3. every rank's chunk sizes -> the job's chunk offsets (global order)
    std::vector<uint64_t> all(maxq * uint64_t(world), 0);
    if (all_local) {
        for (size_t i = 0; i < nl; ++i)
            std::copy(sizes[i].begin(), sizes[i].end(), all.begin() + ptrdiff_t(uint64_t(g->local[i].rank) * maxq));
    } else {
        for (size_t i = 0; i < nl; ++i) {
            Local& l = g->local[i];
            test_park_null_stream(l.device);
            WSG_HIP(hipSetDevice(l.device));
            WSG_HIP(hipMemcpyAsync(l.d_sizes, sizes[i].data(), maxq * sizeof(uint64_t), hipMemcpyHostToDevice,
                                   stream_of(l)));
            WSG_HIP(hipStreamSynchronize(stream_of(l)));
        }
        WSG_NCCL(r->GroupStart());
        for (Local& l : g->local)
            WSG_NCCL(r->AllGather(l.d_sizes, l.d_sizes + maxq, maxq, ncclUint64, l.comm, stream_of(l)));
        WSG_NCCL(r->GroupEnd());
        Local& l = g->local[0];
        WSG_HIP(hipSetDevice(l.device));
        WSG_HIP(hipStreamSynchronize(stream_of(l)));
        WSG_HIP(hipMemcpy(all.data(), l.d_sizes + maxq, all.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
    // goff[c]: where chunk c goes in the root's output; then every rank's
    // base in the root's offset stage (its frames, rank by rank)
    std::vector<uint64_t> goff(n_chunks + 1 + uint64_t(world) + 1, 0);
    for (uint64_t c = 0; c < n_chunks; ++c)
        goff[c + 1] = goff[c] + all[(c % uint64_t(world)) * maxq + c / uint64_t(world)];
    const uint64_t total = goff[n_chunks];
    uint64_t* rank_base = goff.data() + n_chunks + 1;
    for (int k = 0; k < world; ++k)
        rank_base[k + 1] = rank_base[k] + shard_count(n_total, chunk, world, k);
    if (root_l && total > out_cap)
        fail(WSG_ENOMEM);
    if (root_l && !status) {
        test_park_null_stream(root_l->device);
        // on the root's stream (k_rebase_offsets reads it there), landed
        // before the host vector goes
        if (hipSetDevice(root_l->device) != hipSuccess ||
            hipMemcpyAsync(root_l->d_goff, goff.data(), goff.size() * sizeof(uint64_t), hipMemcpyHostToDevice,
                           stream_of(*root_l)) != hipSuccess ||
            hipStreamSynchronize(stream_of(*root_l)) != hipSuccess)
            fail(WSG_EHIP);
    }
    // a short root buffer must stop every rank before the transfers, or the
    // others would wait for it
    if (exchange_status())
        return status;

    // 4. the transfers: every chunk straight to its place in the root's
    // output; every rank's frame offsets in one piece to the root's stage.
    // Per group: one data transfer per chunk (the output is in job order, a
    // rank's chunks are not adjacent there) + one offsets transfer per rank.
    for (Local& l : g->local) {
        test_park_null_stream(l.device);
        WSG_HIP(hipSetDevice(l.device));
        WSG_HIP(hipEventRecord(l.e3, stream_of(l)));
    }
    if (all_local) {
        const int rdev = root_l->device;
        for (size_t i = 0; i < nl; ++i) {
            Local& l = g->local[i];
            hipStream_t s = stream_of(l);
            WSG_HIP(hipSetDevice(l.device));
            auto copy = [&](void* dst, const void* src, uint64_t bytes) -> hipError_t {
                if (!bytes)
                    return hipSuccess;
                return l.device == rdev ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s)
                                        : hipMemcpyPeerAsync(dst, rdev, src, l.device, bytes, s);
            };
            for (uint64_t c = uint64_t(l.rank), q = 0; c < n_chunks; c += uint64_t(world), ++q)
                WSG_HIP(copy(d_out + goff[c], d_wire[i] + loff[i][q * chunk], goff[c + 1] - goff[c]));
            WSG_HIP(copy(root_l->d_stage + rank_base[l.rank], d_wire_off[i], uint64_t(n_local[i]) * sizeof(uint64_t)));
            WSG_HIP(hipEventRecord(l.done, s));
        }
        WSG_HIP(hipSetDevice(rdev));
        for (Local& l : g->local)   // the root's stream goes on once every rank's copies are done
            if (&l != root_l)
                WSG_HIP(hipStreamWaitEvent(stream_of(*root_l), l.done, 0));
    } else {
        WSG_NCCL(r->GroupStart());
        for (size_t i = 0; i < nl; ++i) {
            Local& l = g->local[i];
            hipStream_t s = stream_of(l);
            if (l.rank == root) {
                for (uint64_t c = uint64_t(l.rank), q = 0; c < n_chunks; c += uint64_t(world), ++q)
                    if (goff[c + 1] > goff[c])
                        WSG_HIP(hipMemcpyAsync(d_out + goff[c], d_wire[i] + loff[i][q * chunk], goff[c + 1] - goff[c],
                                               hipMemcpyDeviceToDevice, s));
                if (n_local[i])
                    WSG_HIP(hipMemcpyAsync(root_l->d_stage + rank_base[l.rank], d_wire_off[i],
                                           uint64_t(n_local[i]) * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
                for (uint64_t c = 0; c < n_chunks; ++c) {
                    const int owner = int(c % uint64_t(world));
                    if (owner != root && goff[c + 1] > goff[c])
                        WSG_NCCL(r->Recv(d_out + goff[c], goff[c + 1] - goff[c], ncclUint8, owner, l.comm, s));
                }
                for (int k = 0; k < world; ++k)
                    if (k != root && rank_base[k + 1] > rank_base[k])
                        WSG_NCCL(r->Recv(root_l->d_stage + rank_base[k], rank_base[k + 1] - rank_base[k], ncclUint64, k,
                                         l.comm, s));
                continue;
            }
            for (uint64_t c = uint64_t(l.rank), q = 0; c < n_chunks; c += uint64_t(world), ++q)
                if (goff[c + 1] > goff[c])
                    WSG_NCCL(r->Send(d_wire[i] + loff[i][q * chunk], goff[c + 1] - goff[c], ncclUint8, root, l.comm, s));
            if (n_local[i])
                WSG_NCCL(r->Send(d_wire_off[i], n_local[i], ncclUint64, root, l.comm, s));
        }
        WSG_NCCL(r->GroupEnd());
    }
    if (root_l) {
        hipStream_t s = stream_of(*root_l);
        WSG_HIP(hipSetDevice(root_l->device));
        if (d_out_off)
            WSG_HIP(wsg::launch_rebase_offsets(s, root_l->d_stage, root_l->d_goff, root_l->d_goff + n_chunks + 1,
                                               n_total, chunk, uint32_t(world), d_out_off, total));
    }
    for (Local& l : g->local) {
        WSG_HIP(hipSetDevice(l.device));
        WSG_HIP(hipEventRecord(l.e2, stream_of(l)));
    }
    double enc = 0.0, gat = 0.0;
    for (Local& l : g->local) {
        WSG_HIP(hipSetDevice(l.device));
        WSG_HIP(hipEventSynchronize(l.e2));
        float a = 0.f, b = 0.f;
        WSG_HIP(hipEventElapsedTime(&a, l.e0, l.e1));
        WSG_HIP(hipEventElapsedTime(&b, l.e3, l.e2));
        enc = std::max(enc, double(a));
        gat = std::max(gat, double(b));
    }
    if (times) {
        times[0] = enc;
        times[1] = gat;
    }
    return WSG_OK;
}

} // namespace

extern "C" {

int wsg_mgpu_encode_gather(wsg_mgpu* g, uint64_t n_total, uint32_t chunk, const uint8_t* const* d_payload,
                           const wsg_send_desc* const* d_desc, const uint32_t* n_local, uint8_t* const* d_wire,
                           const uint64_t* wire_cap, uint64_t* const* d_wire_off, int root, uint8_t* d_out,
                           uint64_t out_cap, uint64_t* d_out_off, double* times)
{
    const wsg::TraceRange trace_range("wsg.mgpu_encode_gather");
    try {   // no C++ exception leaves the ABI (host vectors: WSG_ENOMEM)
        return encode_gather(g, n_total, chunk, d_payload, d_desc, n_local, d_wire, wire_cap, d_wire_off, root, d_out,
                             out_cap, d_out_off, times);
    } catch (...) {
        return WSG_ENOMEM;
    }
}

} // extern "C"

namespace {

int decode_host_multi(wsg_ctx* const* ctxs, int nctx, const uint8_t* wire, uint64_t wire_len,
                      const uint64_t* frame_start, uint32_t n, uint8_t* out, wsg_recv_info* info)
{
    if (!ctxs || nctx <= 0 || (wire_len && (!wire || !out)) || (n && (!frame_start || !info)))
        return WSG_EINVAL;
    for (int i = 0; i < nctx; ++i)
        if (!ctxs[i])
            return WSG_EINVAL;
    const std::vector<wsg_ctx*> use = one_per_device(ctxs, nctx);
    ctxs = use.data();
    nctx = int(use.size());
    bool sorted = true;
    for (uint32_t i = 1; i < n && sorted; ++i)
        sorted = frame_start[i] > frame_start[i - 1];
    const int parts = int(std::min<uint64_t>(uint64_t(nctx), std::max<uint64_t>(n, 1)));
    if (parts == 1 || !sorted)
        return wsg_decode_batch_host(ctxs[0], wire, wire_len, frame_start, n, out, info);

    const std::vector<uint32_t> cut = host_runs(frame_start, n, wire_len, parts);
    std::vector<int> rc(size_t(parts), WSG_OK);
    on_contexts(ctxs, parts, [&](int k) {
        const uint32_t a = cut[size_t(k)], b = cut[size_t(k) + 1];
        if (a == b)
            return;
        const uint64_t lo = a ? frame_start[a] : 0, hi = b < n ? frame_start[b] : wire_len;
        try {
            std::vector<uint64_t> fs(frame_start + a, frame_start + b);
            for (uint64_t& x : fs)
                x -= lo;
            rc[size_t(k)] = wsg_decode_batch_host(ctxs[k], wire + lo, hi - lo, fs.data(), b - a, out + lo, info + a);
        } catch (...) {
            rc[size_t(k)] = WSG_ENOMEM;
            return;
        }
        if (lo)
            for (uint32_t i = a; i < b; ++i)
                info[i].payload_off += lo;
    });
    for (int r : rc)
        if (!frame_status(r))
            return r;
    // the batch's frame errors as the one-context call states them: a frame
    // that runs into the next one overlaps it (EINVAL) when its whole length
    // lies inside the wire (a run's last frame only saw its run's bytes)
    int first = WSG_OK;
    for (uint32_t i = 0; i < n; ++i) {
        wsg_recv_info& r = info[i];
        if (r.error == WSG_ETRUNC && i + 1 < n && frame_start[i] < wire_len) {
            wsg_recv_info h;
            if (wsg_header_unpack(wire + frame_start[i], wire_len - frame_start[i], &h) == WSG_OK &&
                h.len <= wire_len - frame_start[i] - h.hdr_len)
                r.error = int8_t(WSG_EINVAL);
        }
        if (r.error && !first)
            first = r.error;
    }
    return first;
}

int encode_host_multi(wsg_ctx* const* ctxs, int nctx, const uint8_t* payload, uint64_t payload_len,
                      const wsg_send_desc* desc, uint32_t n, uint8_t* wire, uint64_t wire_cap, uint64_t* wire_off)
{
    if (!ctxs || nctx <= 0 || !wire_off || (n && (!desc || !wire)) || (payload_len && !payload))
        return WSG_EINVAL;
    for (int i = 0; i < nctx; ++i)
        if (!ctxs[i])
            return WSG_EINVAL;
    const std::vector<wsg_ctx*> use = one_per_device(ctxs, nctx);
    ctxs = use.data();
    nctx = int(use.size());
    const int parts = int(std::min<uint64_t>(uint64_t(nctx), std::max<uint64_t>(n, 1)));
    if (parts == 1)
        return wsg_encode_batch_host(ctxs[0], payload, payload_len, desc, n, wire, wire_cap, wire_off);
    // frame offsets (and argument checks) as the one-context call makes them
    wire_off[0] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const wsg_send_desc& d = desc[i];
        if (d.len > payload_len || d.src_off > payload_len - d.len)
            return WSG_EINVAL;
        wire_off[i + 1] = wire_off[i] + wsg_frame_size(d.opcode, d.mask, d.len, d.status);
    }
    if (wire_off[n] > wire_cap)
        return WSG_ENOMEM;
    // runs of about equal wire bytes
    std::vector<uint32_t> cut(size_t(parts) + 1, n);
    cut[0] = 0;
    for (int k = 1; k < parts; ++k) {
        const uint64_t target = uint64_t(double(wire_off[n]) * k / parts);
        const uint32_t idx = uint32_t(std::lower_bound(wire_off, wire_off + n, target) - wire_off);
        cut[size_t(k)] = std::max(std::min(idx, n), cut[size_t(k) - 1]);
    }
    std::vector<int> rc(size_t(parts), WSG_OK);
    on_contexts(ctxs, parts, [&](int k) {
        const uint32_t a = cut[size_t(k)], b = cut[size_t(k) + 1];
        if (a == b)
            return;
        try {
            std::vector<uint64_t> off(size_t(b - a) + 1);
            rc[size_t(k)] = wsg_encode_batch_host(ctxs[k], payload, payload_len, desc + a, b - a, wire + wire_off[a],
                                                  wire_off[b] - wire_off[a], off.data());
        } catch (...) {
            rc[size_t(k)] = WSG_ENOMEM;
        }
    });
    for (int r : rc)
        if (r)
            return r;
    return WSG_OK;
}

} // namespace

extern "C" {

// no C++ exception leaves the ABI (allocation failures become WSG_ENOMEM)
int wsg_decode_batch_host_multi(wsg_ctx* const* ctxs, int nctx, const uint8_t* wire, uint64_t wire_len,
                                const uint64_t* frame_start, uint32_t n, uint8_t* out, wsg_recv_info* info)
{
    const wsg::TraceRange trace_range("wsg.decode_batch_host_multi");
    try {
        return decode_host_multi(ctxs, nctx, wire, wire_len, frame_start, n, out, info);
    } catch (...) {
        return WSG_ENOMEM;
    }
}

int wsg_encode_batch_host_multi(wsg_ctx* const* ctxs, int nctx, const uint8_t* payload, uint64_t payload_len,
                                const wsg_send_desc* desc, uint32_t n, uint8_t* wire, uint64_t wire_cap,
                                uint64_t* wire_off)
{
    const wsg::TraceRange trace_range("wsg.encode_batch_host_multi");
    try {
        return encode_host_multi(ctxs, nctx, payload, payload_len, desc, n, wire, wire_cap, wire_off);
    } catch (...) {
        return WSG_ENOMEM;
    }
}

int wsg_mgpu_decode_batch_host(wsg_mgpu* g, const uint8_t* wire, uint64_t wire_len, const uint64_t* frame_start,
                               uint32_t n, uint8_t* out, wsg_recv_info* info)
{
    if (!g || g->local.empty())
        return WSG_EINVAL;
    try {
        const std::vector<wsg_ctx*> v = local_ctxs(g);
        return decode_host_multi(v.data(), int(v.size()), wire, wire_len, frame_start, n, out, info);
    } catch (...) {
        return WSG_ENOMEM;
    }
}

int wsg_mgpu_encode_batch_host(wsg_mgpu* g, const uint8_t* payload, uint64_t payload_len, const wsg_send_desc* desc,
                               uint32_t n, uint8_t* wire, uint64_t wire_cap, uint64_t* wire_off)
{
    if (!g || g->local.empty())
        return WSG_EINVAL;
    try {
        const std::vector<wsg_ctx*> v = local_ctxs(g);
        return encode_host_multi(v.data(), int(v.size()), payload, payload_len, desc, n, wire, wire_cap, wire_off);
    } catch (...) {
        return WSG_ENOMEM;
    }
}

} // extern "C"
