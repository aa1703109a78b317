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
        const char* names[] = {std::getenv("WSG_RCCL_LIB"), "/opt/rocm/lib/librccl.so.1", "librccl.so.1",
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
    uint64_t* d_stage = nullptr;   // root: gathered local frame offsets (n_total)
    uint64_t stage_cap = 0;
    uint64_t* d_goff = nullptr;    // root: global offset of every chunk
    uint64_t goff_cap = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr, e3 = nullptr;   // encode start/end, gather end/start
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
    const char* e = std::getenv("WSG_HOST_MULTI_SHARE");
    const bool share = e && *e == '1';
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
        (void)hipFree(l.d_stage);
        (void)hipFree(l.d_goff);
        for (hipEvent_t e : {l.e0, l.e1, l.e2, l.e3})
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
    }
    return WSG_OK;
}

} // namespace

int wsg_mgpu_create(const int* devices, int ndev, wsg_mgpu** out)
{
    if (!out || !devices || ndev <= 0)
        return WSG_EINVAL;
    *out = nullptr;
    const Rccl* r = rccl();
    if (!r)
        return WSG_EHIP;
    wsg_mgpu* g = new (std::nothrow) wsg_mgpu();
    if (!g)
        return WSG_ENOMEM;
    g->world = ndev;
    g->local.resize(size_t(ndev));
    for (int i = 0; i < ndev; ++i) {
        g->local[size_t(i)].device = devices[i];
        g->local[size_t(i)].rank = i;
    }
    if (int rc = init_locals(g)) {
        wsg_mgpu_destroy(g);
        return rc;
    }
    std::vector<ncclComm_t> comms(size_t(ndev), nullptr);
    if (r->CommInitAll(comms.data(), ndev, devices) != ncclSuccess) {
        wsg_mgpu_destroy(g);
        return WSG_EHIP;
    }
    for (int i = 0; i < ndev; ++i)
        g->local[size_t(i)].comm = comms[size_t(i)];
    *out = g;
    return WSG_OK;
}

int wsg_mgpu_create_rank(int device, const uint8_t* id, int rank, int world, wsg_mgpu** out)
{
    if (!out || !id || world <= 0 || rank < 0 || rank >= world)
        return WSG_EINVAL;
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
    const Rccl* r = rccl();
    if (!r)
        return WSG_EHIP;
    const int world = g->world;
    const size_t nl = g->local.size();
    if (n_total == 0) {   // nothing to encode or move, on every rank alike
        for (size_t i = 0; i < nl; ++i)
            if (g->local[i].rank == root && d_out_off) {
                WSG_HIP(hipSetDevice(g->local[i].device));
                WSG_HIP(hipMemset(d_out_off, 0, sizeof(uint64_t)));
            }
        if (times)
            times[0] = times[1] = 0.0;
        return WSG_OK;
    }
    const uint64_t n_chunks = ceil_div(n_total, chunk);
    const uint64_t maxq = ceil_div(n_chunks, uint64_t(world));   // chunks per rank, at most
    Local* root_l = nullptr;
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
        if (uint64_t(n_local[i]) != shard_count(n_total, chunk, world, l.rank))
            return WSG_EINVAL;   // not this rank's round-robin share of the job
        if (l.rank == root) {
            root_l = &l;
            if (!d_out)
                return WSG_EINVAL;
        }
    }

    // 1. every local rank encodes its shard (concurrently, one stream each)
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
        WSG_HIP(hipSetDevice(l.device));
        hipStream_t s = static_cast<hipStream_t>(wsg_stream(l.ctx));
        WSG_HIP(hipEventRecord(l.e0, s));
        if (int rc = wsg_encode_batch(l.ctx, d_payload[i], d_desc[i], n_local[i], d_wire[i], wire_cap[i],
                                      d_wire_off[i], s))
            return rc;
        WSG_HIP(hipEventRecord(l.e1, s));
    }
    // 2. chunk byte sizes of every local rank (host), then all ranks' sizes
    std::vector<std::vector<uint64_t>> loff(nl);
    std::vector<uint64_t> send(maxq);
    int status = WSG_OK;
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
        WSG_HIP(hipSetDevice(l.device));
        hipStream_t s = static_cast<hipStream_t>(wsg_stream(l.ctx));
        if (int rc = wsg_sync(l.ctx, s))
            status = status ? status : rc;   // keep the collectives matched across ranks
        loff[i].resize(size_t(n_local[i]) + 1);
        WSG_HIP(hipMemcpy(loff[i].data(), d_wire_off[i], loff[i].size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
        std::fill(send.begin(), send.end(), 0);
        for (uint64_t q = 0; q * chunk < n_local[i]; ++q)
            send[q] = loff[i][std::min<uint64_t>((q + 1) * chunk, n_local[i])] - loff[i][q * chunk];
        if (int rc = grow(l.d_sizes, l.sizes_cap, maxq * (uint64_t(world) + 1)))
            return rc;
        WSG_HIP(hipMemcpy(l.d_sizes, send.data(), maxq * sizeof(uint64_t), hipMemcpyHostToDevice));
    }
    WSG_NCCL(r->GroupStart());
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
        WSG_NCCL(r->AllGather(l.d_sizes, l.d_sizes + maxq, maxq, ncclUint64, l.comm,
                              static_cast<hipStream_t>(wsg_stream(l.ctx))));
    }
    WSG_NCCL(r->GroupEnd());
    std::vector<uint64_t> all(maxq * uint64_t(world));
    {
        Local& l = g->local[0];
        WSG_HIP(hipSetDevice(l.device));
        WSG_HIP(hipStreamSynchronize(static_cast<hipStream_t>(wsg_stream(l.ctx))));
        WSG_HIP(hipMemcpy(all.data(), l.d_sizes + maxq, all.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
    // 3. the job's chunk offsets (global chunk order)
    std::vector<uint64_t> goff(n_chunks + 1, 0);
    for (uint64_t c = 0; c < n_chunks; ++c)
        goff[c + 1] = goff[c] + all[(c % uint64_t(world)) * maxq + c / uint64_t(world)];
    const uint64_t total = goff[n_chunks];
    if (root_l && total > out_cap)
        status = status ? status : WSG_ENOMEM;
    // an encode error or a short root buffer on any rank must stop every
    // rank before the transfers, or the others would wait for it: the
    // status goes round in a second all-gather
    {
        std::vector<uint64_t> st(uint64_t(world), 0);
        for (size_t i = 0; i < nl; ++i) {
            Local& l = g->local[i];
            WSG_HIP(hipSetDevice(l.device));
            const uint64_t mine = uint64_t(uint32_t(-status));
            WSG_HIP(hipMemcpy(l.d_sizes, &mine, sizeof(uint64_t), hipMemcpyHostToDevice));
        }
        WSG_NCCL(r->GroupStart());
        for (size_t i = 0; i < nl; ++i) {
            Local& l = g->local[i];
            WSG_NCCL(r->AllGather(l.d_sizes, l.d_sizes + maxq, 1, ncclUint64, l.comm,
                                  static_cast<hipStream_t>(wsg_stream(l.ctx))));
        }
        WSG_NCCL(r->GroupEnd());
        Local& l = g->local[0];
        WSG_HIP(hipSetDevice(l.device));
        WSG_HIP(hipStreamSynchronize(static_cast<hipStream_t>(wsg_stream(l.ctx))));
        WSG_HIP(hipMemcpy(st.data(), l.d_sizes + maxq, st.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
        for (uint64_t e : st)
            if (e && !status)
                status = -int(e);
    }
    if (status)
        return status;

    // 4. one grouped transfer: each chunk to its place in the root's output,
    // with its frame offsets
    if (root_l) {
        WSG_HIP(hipSetDevice(root_l->device));
        // the senders always send their chunks' frame offsets (8 B a frame):
        // they cannot know whether the root wants them
        if (int rc = grow(root_l->d_stage, root_l->stage_cap, n_total))
            return rc;
        if (int rc = grow(root_l->d_goff, root_l->goff_cap, n_chunks + 1))
            return rc;
        WSG_HIP(hipMemcpy(root_l->d_goff, goff.data(), goff.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    }
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
        WSG_HIP(hipSetDevice(l.device));
        WSG_HIP(hipEventRecord(l.e3, static_cast<hipStream_t>(wsg_stream(l.ctx))));
    }
    WSG_NCCL(r->GroupStart());
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
        hipStream_t s = static_cast<hipStream_t>(wsg_stream(l.ctx));
        for (uint64_t c = uint64_t(l.rank), q = 0; c < n_chunks; c += uint64_t(world), ++q) {
            const uint64_t lo = loff[i][q * chunk];
            const uint64_t bytes = goff[c + 1] - goff[c];
            const uint64_t frames = std::min<uint64_t>(chunk, n_local[i] - q * chunk);
            if (l.rank == root) {
                if (bytes)
                    WSG_HIP(hipMemcpyAsync(d_out + goff[c], d_wire[i] + lo, bytes, hipMemcpyDeviceToDevice, s));
                WSG_HIP(hipMemcpyAsync(root_l->d_stage + c * chunk, d_wire_off[i] + q * chunk,
                                       frames * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
                continue;
            }
            if (bytes)
                WSG_NCCL(r->Send(d_wire[i] + lo, bytes, ncclUint8, root, l.comm, s));
            WSG_NCCL(r->Send(d_wire_off[i] + q * chunk, frames, ncclUint64, root, l.comm, s));
        }
        if (l.rank != root)
            continue;
        for (uint64_t c = 0; c < n_chunks; ++c) {
            const int owner = int(c % uint64_t(world));
            if (owner == root)
                continue;
            const uint64_t bytes = goff[c + 1] - goff[c];
            const uint64_t frames = std::min<uint64_t>(chunk, n_total - c * chunk);
            if (bytes)
                WSG_NCCL(r->Recv(d_out + goff[c], bytes, ncclUint8, owner, l.comm, s));
            WSG_NCCL(r->Recv(root_l->d_stage + c * chunk, frames, ncclUint64, owner, l.comm, s));
        }
    }
    WSG_NCCL(r->GroupEnd());
    if (root_l) {
        hipStream_t s = static_cast<hipStream_t>(wsg_stream(root_l->ctx));
        WSG_HIP(hipSetDevice(root_l->device));
        if (d_out_off)
            WSG_HIP(wsg::launch_rebase_offsets(s, root_l->d_stage, root_l->d_goff, n_total, chunk, d_out_off, total));
    }
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
        WSG_HIP(hipSetDevice(l.device));
        WSG_HIP(hipEventRecord(l.e2, static_cast<hipStream_t>(wsg_stream(l.ctx))));
    }
    double enc = 0.0, gat = 0.0;
    for (size_t i = 0; i < nl; ++i) {
        Local& l = g->local[i];
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
